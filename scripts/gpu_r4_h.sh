# Screen path after the padding fix and the coalesced exact_dist: screen/exact tests, config-2 bench and
# kernel profile (DBs under /tmp; only summaries come back)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
export PYTHONPATH=$GRAFT_REPO_ROOT
O=gpurun_out/${1:-r4h}
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_kmeans_screen_gpu.py tests/test_kmeans_exact_gpu.py -v -m gpu --timeout 200 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1
rc=$?
tail -3 $O/pytest.log
grep -E "FAILED|Error" $O/pytest.log | head -20
[ $rc -le 1 ] || exit $rc
timeout -k 10 300 python3 bench.py --rows 10000000 --dim 128 --k 64 --dtype f32 --warmup 1 --steps 20 --breakdown > $O/cfg2_screen.json 2> $O/cfg2_screen.err || { tail -5 $O/cfg2_screen.err; exit 1; }
tail -1 $O/cfg2_screen.json | python3 -c "
import json,sys; d=json.loads(sys.stdin.read()); e=d['extra']; b=e['breakdown']
print('cfg2 f32 screen fit ms', e['fit_s']*1000, 'engine', e['engine_fit_ms'], e['precision'], 'init', b['init_ms'], b['iteration_ms'])
print('rechecked', b.get('screen_rechecked_rank0')); print('cert', b.get('certified_steps_rank0'))"
timeout -k 10 300 rocprofv3 --kernel-trace -d /tmp/scr -o scr -- python3 bench.py --rows 10000000 --dim 128 --k 64 --dtype f32 --warmup 1 --steps 20 --no-overlap > $O/scr.log 2>&1 || { tail -5 $O/scr.log; exit 1; }
python3 scripts/rocpd_stats.py /tmp/scr/scr_results.db --top 30 > $O/cfg2_screen_stats.txt
head -32 $O/cfg2_screen_stats.txt
