#!/bin/bash
# Iteration loop on the GPU box: selected GPU test modules, the headline bench, and a kernel-trace
# profile of it. usage: scripts/gpu_iter.sh TAG "tests/a.py tests/b.py" (empty test list: bench only)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export PYTHONPATH="$GRAFT_REPO_ROOT${PYTHONPATH:+:$PYTHONPATH}"
tag=$1
tests=$2
out=gpurun_out/iter/$tag
mkdir -p $out
rc=0
if [ -n "$tests" ]; then
  timeout -k 10 600 python -u -m pytest $tests -x -q -m gpu --timeout 200 --timeout-method thread > $out/tests.log 2>&1
  rc=$?; tail -3 $out/tests.log; [ $rc -eq 0 ] || exit $rc
fi
timeout -k 10 300 python -u bench.py --breakdown > $out/bench.log 2>&1 || exit 4
tail -1 $out/bench.log | cut -c1-300
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace -d "$GRAFT_REPO_ROOT/$out/prof" -o run -- python3 "$GRAFT_REPO_ROOT/bench.py" --steps 20 --warmup 1 > "$GRAFT_REPO_ROOT/$out/prof.log" 2>&1 || exit 5
cd "$GRAFT_REPO_ROOT" && python scripts/rocpd_timeline.py $out/prof/run_results.db --after row_pass_kernel --skip 1 --stats --limit 25 > $out/stats.txt && head -14 $out/stats.txt
exit $rc
