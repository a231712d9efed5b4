# Round-end validation: full GPU suite, smoke, headline bench, rocprofv3 kernel stats of the headline
# bench (only the stats CSV is kept: the trace files exceed gpurun's 64 MiB copy-back)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/final
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 200 --timeout-method thread > gpurun_out/final/pytest_gpu.log 2>&1 || { grep -E "FAIL|Error" gpurun_out/final/pytest_gpu.log | head -20; tail -20 gpurun_out/final/pytest_gpu.log; exit 1; }
tail -1 gpurun_out/final/pytest_gpu.log
timeout -k 10 180 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/final/smoke.log 2>&1 || { tail -20 gpurun_out/final/smoke.log; exit 1; }
tail -1 gpurun_out/final/smoke.log
timeout -k 10 300 python bench.py --steps 20 --warmup 3 > gpurun_out/final/bench.json 2> gpurun_out/final/bench.err || { tail -20 gpurun_out/final/bench.err; exit 1; }
cat gpurun_out/final/bench.json
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/prof_final -o bench -- python3 bench.py --steps 10 --warmup 2 > gpurun_out/final/prof_bench.log 2>&1 || { tail -20 gpurun_out/final/prof_bench.log; exit 1; }
for f in $(find /tmp/prof_final -name "*kernel_stats.csv"); do cp $f gpurun_out/final/bench_kernel_stats.csv; done
python3 -c "import csv;[print(r[\"Name\"][:100], r[\"Calls\"], r[\"Percentage\"]) for r in list(csv.DictReader(open(\"gpurun_out/final/bench_kernel_stats.csv\")))[:14]]"
