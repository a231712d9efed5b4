#!/bin/bash
# Split-graph multi-rank pruned steps: two-rank GPU tests, then the 12.5M-row per-rank emulation.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
export PYTHONPATH="$GRAFT_REPO_ROOT${PYTHONPATH:+:$PYTHONPATH}"
mkdir -p gpurun_out/r3/small
timeout -k 10 600 python -u -m pytest tests/test_distributed_gpu_gloo.py tests/test_kmeans_init_gpu.py -x -v -m gpu --timeout 300 --timeout-method thread \
  > gpurun_out/r3/small/tests.log 2>&1
rc=$?; tail -6 gpurun_out/r3/small/tests.log; [ $rc -eq 0 ] || exit $rc
bash scripts/gpu_r3_small.sh
