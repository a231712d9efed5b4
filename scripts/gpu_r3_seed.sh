#!/bin/bash
# Seeded first step + 32x32 K9r tests, then the headline bench.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export PYTHONPATH="$GRAFT_REPO_ROOT${PYTHONPATH:+:$PYTHONPATH}"
mkdir -p gpurun_out/r3
timeout -k 10 600 python -u -m pytest tests/test_kmeans_init_gpu.py tests/test_kmeans_rr_m32_gpu.py tests/test_kmeans_prune.py -x -v -m gpu --timeout 200 --timeout-method thread \
  > gpurun_out/r3/seed_tests.log 2>&1
rc=$?; tail -8 gpurun_out/r3/seed_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py --breakdown > gpurun_out/r3/bench_seed.log 2>&1
rc=$?; tail -3 gpurun_out/r3/bench_seed.log; exit $rc
