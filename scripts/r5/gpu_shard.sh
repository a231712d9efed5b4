# 8-GPU shard (12.5M rows, one-rank RCCL group): fit breakdown, kernel stats and host-sync gaps of the
# timed engine fit (DBs under /tmp; only summaries come back)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
export PYTHONPATH=$GRAFT_REPO_ROOT
export CML_COMM_SELF=1
O=gpurun_out/${1:-r5shard}
mkdir -p $O
timeout -k 10 300 python3 bench.py --rows 12500000 --warmup 3 --no-overlap --breakdown > $O/shard.json 2> $O/shard.err || { tail -5 $O/shard.err; exit 1; }
tail -1 $O/shard.json | python3 -c "
import json,sys; d=json.loads(sys.stdin.read()); e=d['extra']; b=e['breakdown']
print('shard fit ms', e['fit_s']*1000, 'engine', e['engine_fit_ms'], 'init', b['init_ms'], 'its', b['iteration_ms'], 'steady', e.get('steady_state_ms_per_step'), 'full', e.get('full_step_ms'), e.get('full_step_from_scratch_ms'))"
timeout -k 10 300 rocprofv3 --kernel-trace --runtime-trace -d /tmp/sh -o sh -- python3 bench.py --rows 12500000 --warmup 3 --no-overlap > $O/sh.log 2>&1 || { tail -5 $O/sh.log; exit 1; }
python3 scripts/rocpd_stats.py /tmp/sh/sh_results.db --marker row_pass_kernel --index 1 --top 30 > $O/shard_stats.txt
python3 scripts/rocpd_syncs.py /tmp/sh/sh_results.db --marker row_pass_kernel --index 1 --show 40 > $O/shard_syncs.txt
head -12 $O/shard_stats.txt
head -50 $O/shard_syncs.txt
