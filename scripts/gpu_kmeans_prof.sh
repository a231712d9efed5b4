# KMeans GPU tests + rocprofv3 kernel stats of the headline bench (prebuilt in-tree .so)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/prof_bench
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_kmeans_kernels_gpu.py -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/pytest_km.log 2>&1 || { tail -30 gpurun_out/pytest_km.log; exit 1; }
tail -2 gpurun_out/pytest_km.log
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_bench -o bench -- python3 bench.py --steps 10 --warmup 2 > gpurun_out/prof_bench/bench.log 2>&1
rc=$?; grep -v amdgpu.ids gpurun_out/prof_bench/bench.log | tail -2
for f in $(find gpurun_out/prof_bench -name "*kernel_stats.csv"); do cut -d, -f1-4 $f | head -12 | cut -c1-200; done
exit $rc
