set -o pipefail
cd "$GRAFT_REPO_ROOT"
export PYTHONPATH="$GRAFT_REPO_ROOT${PYTHONPATH:+:$PYTHONPATH}"
out=gpurun_out/graphab; mkdir -p $out
for r in 100000000 12500000; do
  for g in 1 0; do
    CML_KMEANS_GRAPH=$g timeout -k 10 200 python -u bench.py --rows $r --breakdown > $out/g${g}_$r.log 2>&1 || exit 3
    tail -1 $out/g${g}_$r.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); e=d['extra']; print($r, $g, e['fit_s'], e['init_s'], e['breakdown']['init_ms'], e['breakdown']['iteration_ms'][:5], e['steady_state_ms_per_step'])"
  done
done
