# KMeans GPU tests + shard-size (self-comm) and headline benches after the init host-sync cuts
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/${1:-r4c}
O=gpurun_out/${1:-r4c}
timeout -k 10 400 python -u -m pytest tests -k "kmeans or distributed or cluster or pipeline or screen" -v -m gpu --timeout 120 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1
rc=$?
tail -3 $O/pytest.log
grep -E "FAILED|ERROR" $O/pytest.log | head -20
[ $rc -le 1 ] || exit $rc
CML_COMM_SELF=1 timeout -k 10 300 python3 bench.py --rows 12500000 --warmup 3 --no-overlap --breakdown > $O/shard.json 2> $O/shard.err || { tail -5 $O/shard.err; exit 1; }
python3 -c "
import json; d=json.load(open('$O/shard.json')); e=d['extra']
print('shard fit ms', e['fit_s']*1000, 'engine', e['engine_fit_ms'], 'init', e['breakdown']['init_ms'], 'iters', e['breakdown']['iteration_ms'][:4], 'steady', e['steady_state_ms_per_step'])"
timeout -k 10 300 python3 bench.py --no-overlap > $O/bench.json 2> $O/bench.err || { tail -5 $O/bench.err; exit 1; }
python3 -c "
import json; d=json.load(open('$O/bench.json')); e=d['extra']
print('100M fit ms', e['fit_s']*1000, 'engine', e['engine_fit_ms'], 'value', d['value'])"
timeout -k 10 300 python3 scripts/mb_dropna.py > $O/mb_dropna.log 2>&1 || { tail -5 $O/mb_dropna.log; exit 1; }
tail -10 $O/mb_dropna.log
timeout -k 10 300 python3 bench.py --rows 10000000 --dim 128 --k 64 --dtype f32 --warmup 1 --steps 20 --breakdown > $O/cfg2_f32_exact.json 2> $O/cfg2_f32_exact.err || { tail -5 $O/cfg2_f32_exact.err; exit 1; }
python3 -c "
import json; d=json.load(open('$O/cfg2_f32_exact.json')); e=d['extra']
print('cfg2 f32 exact fit ms', e['fit_s']*1000, 'precision', e['precision'], 'breakdown', e['breakdown']['init_ms'], e['breakdown']['iteration_ms'][:5])"
timeout -k 10 300 python3 bench.py --rows 10000000 --dim 128 --k 64 --warmup 1 --steps 20 > $O/cfg2_bf16.json 2> $O/cfg2_bf16.err || { tail -5 $O/cfg2_bf16.err; exit 1; }
python3 -c "
import json; d=json.load(open('$O/cfg2_bf16.json')); e=d['extra']
print('cfg2 bf16 fit ms', e['fit_s']*1000, 'steady', e.get('steady_state_ms_per_step'))"
timeout -k 10 300 python3 bench.py --rows 10000000 --dim 128 --k 64 --dtype f32 --precision exact --warmup 1 --steps 20 > $O/cfg2_f32_exactonly.json 2> $O/cfg2_f32_exactonly.err || { tail -5 $O/cfg2_f32_exactonly.err; exit 1; }
python3 -c "
import json; d=json.load(open('$O/cfg2_f32_exactonly.json')); e=d['extra']
print('cfg2 f32 EXACT fit ms', e['fit_s']*1000, 'precision', e['precision'])"
