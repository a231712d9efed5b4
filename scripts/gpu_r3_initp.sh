#!/bin/bash
# Pruned k-means|| candidate pass: init tests, then the headline bench.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export PYTHONPATH="$GRAFT_REPO_ROOT${PYTHONPATH:+:$PYTHONPATH}"
mkdir -p gpurun_out/r3
timeout -k 10 600 python -u -m pytest tests/test_kmeans_init_gpu.py tests/test_kmeans_prune.py -x -v -m gpu --timeout 200 --timeout-method thread \
  > gpurun_out/r3/initp_tests.log 2>&1
rc=$?; tail -8 gpurun_out/r3/initp_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py --breakdown > gpurun_out/r3/bench_initp.log 2>&1
rc=$?; tail -1 gpurun_out/r3/bench_initp.log | cut -c1-1200; exit $rc
