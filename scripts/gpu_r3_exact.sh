#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r3
: || AMD_SERIALIZE_KERNEL=3 timeout -k 10 300 python -u -m pytest tests/test_kmeans_exact_gpu.py -x -v -m gpu --timeout 120 --timeout-method thread > gpurun_out/r3/exact_tests.log 2>&1

timeout -k 10 600 python -u -m pytest tests/test_kmeans_init_gpu.py tests/test_kmeans_prune.py tests/test_kmeans_kernels_gpu.py tests/test_kmeans_incremental_gpu.py tests/test_distributed_gpu_gloo.py tests/test_distributed_gloo.py -x -q -m gpu --timeout 200 --timeout-method thread > gpurun_out/r3/kmeans_gpu_tests.log 2>&1
rc=$?; tail -5 gpurun_out/r3/kmeans_gpu_tests.log; exit $rc
