set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/benches
timeout -k 10 400 python -u -m pytest tests/test_kmeans_incremental_gpu.py tests/test_kmeans_kernels_gpu.py tests/test_distributed_gpu_gloo.py -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/pytest_km.log 2>&1 || { grep -E "FAIL|Error|assert" gpurun_out/pytest_km.log | head -30; tail -30 gpurun_out/pytest_km.log; exit 1; }
tail -1 gpurun_out/pytest_km.log
timeout -k 10 300 python bench.py --steps 20 --warmup 3 > gpurun_out/bench_inc.json 2> gpurun_out/bench_inc.err || { tail -20 gpurun_out/bench_inc.err; exit 1; }
cut -c1-100 gpurun_out/bench_inc.json
CML_TRACE=1 timeout -k 10 600 python bench.py --workload pipeline --steps 2 --warmup 1 > gpurun_out/benches/pipeline_trace.log 2>&1; rc=$?
grep -v amdgpu.ids gpurun_out/benches/pipeline_trace.log | tail -12 | cut -c1-200
exit $rc
