#!/bin/bash
# Config-5 pipeline (VectorAssembler -> StandardScaler(fp8) -> KMeans k=128 -> LogReg), 125M x 512 per GPU.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export PYTHONPATH="$GRAFT_REPO_ROOT${PYTHONPATH:+:$PYTHONPATH}"
mkdir -p gpurun_out/pipe
timeout -k 10 500 python -u bench.py --workload pipeline --steps 2 --warmup 1 > gpurun_out/pipe/pipeline.log 2>&1 || exit 3
tail -1 gpurun_out/pipe/pipeline.log | cut -c1-400
