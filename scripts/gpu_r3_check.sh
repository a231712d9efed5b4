#!/bin/bash
# Round-3 re-entry check: full GPU suite, smoke, headline bench with the phase breakdown, kernel stats.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export PYTHONPATH="$GRAFT_REPO_ROOT${PYTHONPATH:+:$PYTHONPATH}"
out=gpurun_out/r3/check5
mkdir -p $out
timeout -k 10 900 python -u -m pytest tests -x -m gpu -q --timeout 300 --timeout-method thread > $out/tests.log 2>&1
rc=$?; tail -6 $out/tests.log; [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > $out/smoke.log 2>&1 || exit 3
tail -1 $out/smoke.log
timeout -k 10 300 python -u bench.py --breakdown > $out/bench.log 2>&1 || exit 4
tail -1 $out/bench.log | cut -c1-600
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/$out/prof" -o run -- python3 "$GRAFT_REPO_ROOT/bench.py" --steps 20 --warmup 1 > "$GRAFT_REPO_ROOT/$out/prof.log" 2>&1 || exit 5
exit $rc
