# Certified pruned screen step: kernel/step tests, exact + screen fits, config-2 f32 bench + kernel profile
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-r4f}
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_kmeans_screen_gpu.py tests/test_kmeans_exact_gpu.py tests/test_kmeans_init_gpu.py tests/test_distributed_gpu_gloo.py tests/test_kmeans_api_gpu.py tests/test_gpu_glm_trees.py -v -m gpu --timeout 200 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1
rc=$?
tail -3 $O/pytest.log
grep -E "FAILED|ERROR|Error" $O/pytest.log | head -20
[ $rc -le 1 ] || exit $rc
timeout -k 10 300 python3 bench.py --rows 10000000 --dim 128 --k 64 --dtype f32 --warmup 1 --steps 20 --breakdown > $O/cfg2_screen.json 2> $O/cfg2_screen.err || { tail -5 $O/cfg2_screen.err; exit 1; }
tail -1 $O/cfg2_screen.json | python3 -c "
import json,sys; d=json.loads(sys.stdin.read()); e=d['extra']; b=e['breakdown']
print('cfg2 f32 screen fit ms', e['fit_s']*1000, 'engine', e['engine_fit_ms'], e['precision'], 'init', b['init_ms'], b['iteration_ms'])
print('rechecked', b.get('screen_rechecked_rank0')); print('cert', b.get('certified_steps_rank0'))"
timeout -k 10 300 rocprofv3 --kernel-trace -d $O/scr -o scr -- python3 bench.py --rows 10000000 --dim 128 --k 64 --dtype f32 --warmup 1 --steps 20 --no-overlap > $O/scr.log 2>&1 || { tail -5 $O/scr.log; exit 1; }
python3 scripts/rocpd_stats.py $O/scr/scr_results.db --marker to_bf16_err --index 1 --top 30
CML_TRACE=1 timeout -k 10 500 python3 bench.py --workload pipeline --steps 2 --warmup 1 > $O/pipe.json 2> $O/pipe.err || { tail -20 $O/pipe.err; exit 1; }
cut -c1-300 $O/pipe.json
grep -A12 "^range" $O/pipe.err
export CML_COMM_SELF=1
timeout -k 10 300 python3 bench.py --rows 12500000 --warmup 3 --no-overlap --breakdown > $O/shard.json 2> $O/shard.err || { tail -5 $O/shard.err; exit 1; }
tail -1 $O/shard.json | python3 -c "
import json,sys; d=json.loads(sys.stdin.read()); e=d['extra']; b=e['breakdown']
print('shard fit ms', e['fit_s']*1000, 'engine', e['engine_fit_ms'], 'init', b['init_ms'], 'its', b['iteration_ms'])"
timeout -k 10 300 rocprofv3 --kernel-trace --runtime-trace -d $O/sh -o sh -- python3 bench.py --rows 12500000 --warmup 3 --no-overlap > $O/sh.log 2>&1 || { tail -5 $O/sh.log; exit 1; }
python3 scripts/rocpd_stats.py $O/sh/sh_results.db --marker row_pass_kernel --index 1 --top 30 > $O/shard_stats.txt
python3 scripts/rocpd_syncs.py $O/sh/sh_results.db --marker row_pass_kernel --index 1 --show 60 > $O/shard_syncs.txt
head -32 $O/shard_stats.txt
