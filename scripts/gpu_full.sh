# Full GPU test suite + smoke + headline bench + pipeline trace
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/benches
timeout -k 10 600 python -u -m pytest tests -x -v -m gpu --timeout 200 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { grep -E "FAIL|Error|assert" gpurun_out/pytest_gpu.log | head -30; tail -30 gpurun_out/pytest_gpu.log; exit 1; }
tail -1 gpurun_out/pytest_gpu.log
timeout -k 10 180 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { tail -20 gpurun_out/smoke.log; exit 1; }
tail -1 gpurun_out/smoke.log
timeout -k 10 300 python bench.py --steps 20 --warmup 3 > gpurun_out/bench.json 2> gpurun_out/bench.err || { tail -20 gpurun_out/bench.err; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/bench.json'));print(d['value'],d['ms_per_step'],d['extra'])"
CML_TRACE=1 timeout -k 10 600 python bench.py --workload pipeline --steps 2 --warmup 1 > gpurun_out/benches/pipeline_trace.log 2>&1 || { tail -20 gpurun_out/benches/pipeline_trace.log; exit 1; }
grep -v amdgpu.ids gpurun_out/benches/pipeline_trace.log | tail -12 | cut -c1-200
