# Overlap-data fits (blob centres 8x closer) by the pruned step's candidate cap
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/${1:-r4cap}
mkdir -p $O
for cap in 0.3 0.5 0.7 0.9; do
  CML_KMEANS_PRUNE_CAP=$cap timeout -k 10 300 python3 bench.py --data overlap --warmup 2 --breakdown > $O/overlap_cap$cap.json 2> $O/overlap_cap$cap.err || { tail -5 $O/overlap_cap$cap.err; exit 1; }
  tail -1 $O/overlap_cap$cap.json | python3 -c "
import json,sys; d=json.loads(sys.stdin.read()); e=d['extra']; b=e['breakdown']
print('cap $cap: fit ms', round(e['fit_s']*1000,1), 'init', b['init_ms'], 'steps', [round(t,1) for t in b['iteration_ms']], 'full', e.get('full_step_ms'))"
done
