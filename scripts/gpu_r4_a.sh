# Round 4 first GPU pass: full GPU suite (no -x: see every failure), smoke, headline bench (API fit)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r4a
timeout -k 10 600 python -u -m pytest tests -v -m gpu --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/r4a/pytest_gpu.log 2>&1
rc=$?
tail -5 gpurun_out/r4a/pytest_gpu.log
grep -E "FAILED|ERROR" gpurun_out/r4a/pytest_gpu.log | head -40
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 180 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r4a/smoke.log 2>&1 || { tail -20 gpurun_out/r4a/smoke.log; exit 1; }
grep -v amdgpu.ids gpurun_out/r4a/smoke.log
timeout -k 10 400 python bench.py > gpurun_out/r4a/bench.json 2> gpurun_out/r4a/bench.err || { tail -20 gpurun_out/r4a/bench.err; exit 1; }
cat gpurun_out/r4a/bench.json
