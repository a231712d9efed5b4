# KMeans GPU tests touched in round 4 + a tol=1e-4 API-fit kernel trace (no per-step host sync check)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/r4b
timeout -k 10 300 python -u -m pytest tests/test_kmeans_api_gpu.py tests/test_kmeans_prune.py tests/test_gpu_frame_kernels.py tests/test_kmeans_stream_gpu.py -v -m gpu --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/r4b/pytest.log 2>&1
rc=$?
tail -3 gpurun_out/r4b/pytest.log
grep -E "FAILED|ERROR" gpurun_out/r4b/pytest.log | head -20
[ $rc -le 1 ] || exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --runtime-trace -d gpurun_out/r4b/tol -o tol -- python3 bench.py --warmup 2 --no-overlap --tol 1e-4 --steps 40 > gpurun_out/r4b/tol.log 2>&1 || { tail -5 gpurun_out/r4b/tol.log; exit 1; }
grep '^{' gpurun_out/r4b/tol.log | cut -c1-700
