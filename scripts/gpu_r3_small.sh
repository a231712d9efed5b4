#!/bin/bash
# One rank's share of the 8-GPU run (12.5M rows): graph vs eager steps, and a kernel trace (eager).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
export PYTHONPATH="$GRAFT_REPO_ROOT${PYTHONPATH:+:$PYTHONPATH}"
mkdir -p gpurun_out/r3/small
timeout -k 10 200 python -u bench.py --rows 12500000 --breakdown > gpurun_out/r3/small/graph.log 2>&1 || exit 1
CML_KMEANS_GRAPH=0 timeout -k 10 200 python -u bench.py --rows 12500000 --breakdown > gpurun_out/r3/small/eager.log 2>&1 || exit 2
CML_KMEANS_GRAPH=0 timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/r3/small/tr -o tr -- python3 bench.py --rows 12500000 > gpurun_out/r3/small/trace.log 2>&1 || exit 3
echo ok
