#!/bin/bash
# A/B of the k-means|| first-round full-pass chunk (CML_KMEANS_INIT_FIRST) on the headline fit.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export PYTHONPATH="$GRAFT_REPO_ROOT${PYTHONPATH:+:$PYTHONPATH}"
out=gpurun_out/first_ab; mkdir -p $out
for f in 0 256 192 128; do
  if [ $f = 0 ]; then unset CML_KMEANS_INIT_FIRST; else export CML_KMEANS_INIT_FIRST=$f; fi
  timeout -k 10 200 python -u bench.py --breakdown > $out/first$f.log 2>&1 || exit 3
  tail -1 $out/first$f.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); e=d['extra']; print($f, e['fit_s'], e['init_s'], e['breakdown']['init_ms'], e['breakdown']['iteration_ms'][:3], e['breakdown']['init_pruned_rounds_rank0'])"
done
