#!/bin/bash
# Round-3 baseline: whole-fit headline (default engine), prune on, with per-iteration breakdown.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r3
timeout -k 10 300 python -u bench.py --steps 20 --warmup 3 --breakdown > gpurun_out/r3/base_default.json 2> gpurun_out/r3/base_default.err &&
timeout -k 10 300 python -u bench.py --steps 20 --warmup 3 --breakdown --prune on > gpurun_out/r3/base_prune.json 2> gpurun_out/r3/base_prune.err &&
cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/gpurun_out/r3/prof_base" -o run -- python3 "$GRAFT_REPO_ROOT/bench.py" --steps 20 --warmup 0 > "$GRAFT_REPO_ROOT/gpurun_out/r3/prof_base.log" 2>&1
