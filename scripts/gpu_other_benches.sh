#!/bin/bash
# The other bench workloads (logreg L-BFGS, logreg SGD, CSV ingest) still run end to end.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export PYTHONPATH="$GRAFT_REPO_ROOT${PYTHONPATH:+:$PYTHONPATH}"
mkdir -p gpurun_out/other
timeout -k 10 300 python -u bench.py --workload logreg --steps 10 --warmup 2 > gpurun_out/other/logreg.log 2>&1 || exit 3
tail -1 gpurun_out/other/logreg.log | cut -c1-300
timeout -k 10 300 python -u bench.py --workload logreg --solver sgd --steps 50 --warmup 5 > gpurun_out/other/sgd.log 2>&1 || exit 4
tail -1 gpurun_out/other/sgd.log | cut -c1-300
timeout -k 10 300 python -u bench.py --workload csv --steps 2 --warmup 1 > gpurun_out/other/csv.log 2>&1 || exit 5
tail -1 gpurun_out/other/csv.log | cut -c1-300
