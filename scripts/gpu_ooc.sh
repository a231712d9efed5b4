#!/bin/bash
# Out-of-core KMeans bench (pinned host rows streamed through two device buffers) + an A/B of the
# seeded step's exact upper bounds on the headline bench.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export PYTHONPATH="$GRAFT_REPO_ROOT${PYTHONPATH:+:$PYTHONPATH}"
out=gpurun_out/ooc
mkdir -p $out
CML_KMEANS_SEED_UB=0 timeout -k 10 200 python -u bench.py --breakdown > $out/bench_noub.log 2>&1 || exit 3
tail -1 $out/bench_noub.log | cut -c1-250
timeout -k 10 300 python -u bench.py --workload kmeans_ooc --ooc-rows 50000000 --steps 2 > $out/ooc50M.log 2>&1 || exit 4
tail -1 $out/ooc50M.log
timeout -k 10 500 python -u bench.py --workload kmeans_ooc --steps 3 > $out/ooc250M.log 2>&1 || exit 5
tail -1 $out/ooc250M.log
