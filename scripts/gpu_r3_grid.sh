#!/bin/bash
# Sum grid + kpp scan + tightened kernel bands + exact forest stats: the GPU test modules, the headline
# bench, then the first-chunk size A/B of the k-means|| round 1.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export PYTHONPATH="$GRAFT_REPO_ROOT${PYTHONPATH:+:$PYTHONPATH}"
mkdir -p gpurun_out/r3/grid
timeout -k 10 900 python -u -m pytest tests/test_kmeans_incremental_gpu.py tests/test_kmeans_kernels_gpu.py tests/test_gpu_glm_trees.py tests/test_kmeans_prune.py tests/test_kmeans_init_gpu.py tests/test_kmeans_rr_m32_gpu.py tests/test_distributed_gpu_gloo.py -v -m gpu --timeout 300 --timeout-method thread > gpurun_out/r3/grid/tests.log 2>&1
rc=$?; tail -4 gpurun_out/r3/grid/tests.log; [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 300 python -u bench.py --breakdown > gpurun_out/r3/grid/bench.log 2>&1 || exit 2
tail -1 gpurun_out/r3/grid/bench.log | cut -c1-400
for f in 256 128; do
  CML_KMEANS_INIT_FIRST=$f timeout -k 10 200 python -u bench.py --breakdown > gpurun_out/r3/grid/first$f.log 2>&1 || exit 2
done
exit $rc
