# Pruned-step candidate cap: overlap-data headline fits and the config-5 pipeline by cap
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-r4cap2}
mkdir -p $O
for cap in 0.3 0.6 0.9; do
  CML_KMEANS_PRUNE_CAP=$cap timeout -k 10 300 python3 bench.py --data overlap --warmup 1 --breakdown --no-overlap > $O/overlap_cap$cap.json 2> $O/overlap_cap$cap.err || { tail -5 $O/overlap_cap$cap.err; exit 1; }
  tail -1 $O/overlap_cap$cap.json | python3 -c "
import json,sys; d=json.loads(sys.stdin.read()); e=d['extra']; b=e['breakdown']
print('overlap cap $cap: fit ms', round(e['fit_s']*1000,1), 'init', b['init_ms'], 'steps', [round(t,1) for t in b['iteration_ms']], 'hist', [h[1] for h in b.get('prune_history_rank0', [])][:20])"
done
for cap in 0.3 0.9; do
  CML_KMEANS_PRUNE_CAP=$cap CML_TRACE=1 timeout -k 10 500 python3 bench.py --workload pipeline --steps 2 --warmup 1 > $O/pipe_cap$cap.json 2> $O/pipe_cap$cap.err || { tail -20 $O/pipe_cap$cap.err; exit 1; }
  echo "pipeline cap $cap"; cut -c1-200 $O/pipe_cap$cap.json
  grep -A10 "^range" $O/pipe_cap$cap.err
done
