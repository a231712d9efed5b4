set -o pipefail
cd "$GRAFT_REPO_ROOT"
export PYTHONPATH="$GRAFT_REPO_ROOT${PYTHONPATH:+:$PYTHONPATH}"
mkdir -p gpurun_out/dist
timeout -k 10 400 python -u -m pytest tests/test_distributed_gpu_gloo.py tests/test_kmeans_stream_gpu.py -x -v -m gpu --timeout 300 --timeout-method thread > gpurun_out/dist/tests.log 2>&1
rc=$?; tail -12 gpurun_out/dist/tests.log; [ $rc -eq 0 ] || exit $rc
CML_COMM_SELF=1 timeout -k 10 200 python -u bench.py --rows 12500000 --breakdown > gpurun_out/dist/self_rccl_12.5M.log 2>&1 || exit 4
tail -1 gpurun_out/dist/self_rccl_12.5M.log | cut -c1-200
timeout -k 10 200 python -u bench.py --rows 12500000 --breakdown > gpurun_out/dist/single_12.5M.log 2>&1 || exit 5
tail -1 gpurun_out/dist/single_12.5M.log | cut -c1-200
