# Incremental-sums KMeans: GPU tests, then the headline bench and its kernel stats
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/prof_bench
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_kmeans_incremental_gpu.py tests/test_kmeans_kernels_gpu.py -x -v -m gpu --timeout 120 --timeout-method thread > gpurun_out/pytest_km.log 2>&1 || { grep -E "FAIL|Error|error|assert" gpurun_out/pytest_km.log | head -30; tail -30 gpurun_out/pytest_km.log; exit 1; }
tail -2 gpurun_out/pytest_km.log
timeout -k 10 300 python bench.py --steps 20 --warmup 3 > gpurun_out/bench_inc.json 2> gpurun_out/bench_inc.err || { tail -20 gpurun_out/bench_inc.err; exit 1; }
cat gpurun_out/bench_inc.json
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_bench -o bench -- python3 bench.py --steps 10 --warmup 2 > gpurun_out/prof_bench/bench.log 2>&1
