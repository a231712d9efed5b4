# config-2 f32 certified fit: tol = 0 against a tol that never triggers (per-step convergence read)
set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONPATH=$GRAFT_REPO_ROOT
O=gpurun_out/${1:-tolsync}
mkdir -p $O
for t in 0 1e-12 0 1e-12; do
timeout -k 10 300 python3 bench.py --rows 10000000 --dim 128 --k 64 --dtype f32 --warmup 1 --steps 20 --no-overlap --tol $t > $O/cfg2_$t.json 2> $O/cfg2_$t.err || { tail -5 $O/cfg2_$t.err; exit 1; }
tail -1 $O/cfg2_$t.json | python3 -c "
import json,sys; d=json.loads(sys.stdin.read()); e=d['extra']
print('tol $t', e['precision'], 'iters', e.get('iterations'), 'fit ms', e['fit_s']*1000, 'engine', e['engine_fit_ms'])"
done
