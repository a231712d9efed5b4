# Pruned (exact bounds) Lloyd step: GPU tests, headline bench with the pruned probe, --prune bench,
# kernel stats of the pruned bench
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/prune
timeout -k 10 300 python -u -m pytest tests/test_kmeans_prune.py -x -v -m gpu --timeout 200 --timeout-method thread > gpurun_out/prune/pytest.log 2>&1 || { tail -40 gpurun_out/prune/pytest.log; exit 1; }
tail -1 gpurun_out/prune/pytest.log
timeout -k 10 300 python bench.py --steps 20 --warmup 3 > gpurun_out/prune/bench.json 2> gpurun_out/prune/bench.err || { tail -20 gpurun_out/prune/bench.err; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/prune/bench.json'));print(d['value'],d['ms_per_step'],d['extra'])"
timeout -k 10 300 python bench.py --steps 20 --warmup 3 --prune > gpurun_out/prune/bench_prune.json 2> gpurun_out/prune/bench_prune.err || { tail -20 gpurun_out/prune/bench_prune.err; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/prune/bench_prune.json'));print(d['value'],d['ms_per_step'],d['extra'])"
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prune/prof -o prune -- python3 bench.py --steps 10 --warmup 3 --prune > gpurun_out/prune/prof.log 2>&1 || { tail -20 gpurun_out/prune/prof.log; exit 1; }
find gpurun_out/prune/prof -name "*kernel_stats.csv" | head -3
