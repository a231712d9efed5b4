#!/bin/bash
# Full GPU test suite in one process, then smoke() and a 1-GPU bench run.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r3
timeout -k 10 900 python -u -m pytest tests -x -v -m gpu --timeout 200 --timeout-method thread \
  > gpurun_out/r3/gpu_tests_full.log 2>&1
rc=$?; tail -5 gpurun_out/r3/gpu_tests_full.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u -c 'import __graft_entry__ as g; g.smoke(); print("smoke ok")' \
  > gpurun_out/r3/smoke.log 2>&1
rc=$?; tail -3 gpurun_out/r3/smoke.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py > gpurun_out/r3/bench_default.log 2>&1
rc=$?; tail -2 gpurun_out/r3/bench_default.log; exit $rc
