#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r3
AMD_SERIALIZE_KERNEL=3 timeout -k 10 300 python -u -m pytest tests/test_kmeans_init_gpu.py -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/r3/init_tests.log 2>&1
rc=$?; tail -3 gpurun_out/r3/init_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u -m pytest tests/test_kmeans_prune.py -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/r3/prune_tests.log 2>&1
rc=$?; tail -3 gpurun_out/r3/prune_tests.log; [ $rc -eq 0 ] || exit $rc
PYTHONPATH=. timeout -k 10 300 python -u scripts/mb_rr_modes.py 20000000 256 256 > gpurun_out/r3/mb_rr_modes.log 2>&1
rc=$?; grep -v amdgpu.ids gpurun_out/r3/mb_rr_modes.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py --steps 20 --warmup 3 --breakdown > gpurun_out/r3/bench_init.json 2> gpurun_out/r3/bench_init.err
rc=$?; tail -c 1500 gpurun_out/r3/bench_init.json; [ $rc -eq 0 ] || exit $rc
rm -rf gpurun_out/r3/prof_init
cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/gpurun_out/r3/prof_init" -o run -- python3 "$GRAFT_REPO_ROOT/bench.py" --steps 20 --warmup 2 > "$GRAFT_REPO_ROOT/gpurun_out/r3/prof_init.log" 2>&1
