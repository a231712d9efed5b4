#!/bin/bash
# Round 3: device pruned step — kernel tests, prune tests, then the whole-fit bench with breakdown.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r3
AMD_SERIALIZE_KERNEL=3 timeout -k 10 300 python -u -m pytest tests/test_kmeans_prune.py -x -v -m gpu --timeout 120 --timeout-method thread -k "rr_ or centre_stats" > gpurun_out/r3/prune_kernel_tests.log 2>&1
rc=$?; tail -15 gpurun_out/r3/prune_kernel_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u -m pytest tests/test_kmeans_prune.py -x -v -m gpu --timeout 120 --timeout-method thread > gpurun_out/r3/prune_tests.log 2>&1
rc=$?; tail -15 gpurun_out/r3/prune_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py --steps 20 --warmup 3 --breakdown > gpurun_out/r3/bench_pdev.json 2> gpurun_out/r3/bench_pdev.err
rc=$?; tail -c 3000 gpurun_out/r3/bench_pdev.json; tail -5 gpurun_out/r3/bench_pdev.err; exit $rc
