#!/bin/bash
# 32x32-MFMA K9r: correctness tests, then the mode microbench with the 16x16 form for comparison.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r3
export PYTHONPATH="$GRAFT_REPO_ROOT${PYTHONPATH:+:$PYTHONPATH}"
: || timeout -k 10 300 python -u -m pytest tests/test_kmeans_rr_m32_gpu.py -x -v -m gpu --timeout 120 --timeout-method thread \
  > gpurun_out/r3/m32_tests.log 2>&1
:
timeout -k 10 300 python -u scripts/mb_rr_modes.py > gpurun_out/r3/mb_rr_modes_m32.log 2>&1 || exit 3
CML_KMEANS_RR_M32=0 timeout -k 10 300 python -u scripts/mb_rr_modes.py > gpurun_out/r3/mb_rr_modes_m16.log 2>&1 || exit 4
cat gpurun_out/r3/mb_rr_modes_m32.log gpurun_out/r3/mb_rr_modes_m16.log
