#!/bin/bash
# Kernel trace of the whole-fit bench (one timed fit).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
export PYTHONPATH="$GRAFT_REPO_ROOT${PYTHONPATH:+:$PYTHONPATH}"
mkdir -p gpurun_out/r3/trace
timeout -k 10 400 rocprofv3 --kernel-trace -d gpurun_out/r3/trace/fit -o fit -- python3 bench.py > gpurun_out/r3/trace/fit.log 2>&1 || exit 1
tail -1 gpurun_out/r3/trace/fit.log | cut -c1-300
