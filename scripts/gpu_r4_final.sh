# Round-4 final check on one tree: whole GPU suite, smoke(), headline bench (public API), overlap-data
# fit, config-2 f32 certified fit, config-5 pipeline
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
export PYTHONPATH=$GRAFT_REPO_ROOT
O=gpurun_out/${1:-r4final}
mkdir -p $O
timeout -k 10 1000 python -u -m pytest tests -m gpu -q --timeout 200 --timeout-method thread -p no:cacheprovider > $O/pytest_gpu.log 2>&1
rc=$?
tail -2 $O/pytest_gpu.log
grep -E "FAILED|Error" $O/pytest_gpu.log | head -20
[ $rc -le 1 ] || exit $rc
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || { tail -5 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 400 python3 bench.py > $O/bench.json 2> $O/bench.err || { tail -5 $O/bench.err; exit 1; }
tail -1 $O/bench.json | python3 -c "
import json,sys; d=json.loads(sys.stdin.read()); e=d['extra']
print('headline', d['value'], 'fit ms', e['fit_s']*1000, 'engine', e['engine_fit_ms'], 'steady', e.get('steady_state_ms_per_step'), 'full', e.get('full_step_ms'), e.get('full_step_from_scratch_ms'), 'overlap', (e.get('overlap') or {}).get('fit_ms'))"
timeout -k 10 300 python3 bench.py --rows 10000000 --dim 128 --k 64 --dtype f32 --warmup 1 --steps 20 > $O/cfg2_f32.json 2> $O/cfg2_f32.err || { tail -5 $O/cfg2_f32.err; exit 1; }
tail -1 $O/cfg2_f32.json | python3 -c "
import json,sys; d=json.loads(sys.stdin.read()); e=d['extra']
print('cfg2 f32', e['precision'], 'fit ms', e['fit_s']*1000, 'engine', e['engine_fit_ms'])"
CML_TRACE=1 timeout -k 10 500 python3 bench.py --workload pipeline --steps 2 --warmup 1 > $O/pipe.json 2> $O/pipe.err || { tail -20 $O/pipe.err; exit 1; }
cut -c1-220 $O/pipe.json
grep -A10 "^range" $O/pipe.err
