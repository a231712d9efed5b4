# Config-2 f32: split vs plain screen
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-r4k}
mkdir -p $O
for sp in 1; do
  CML_KMEANS_SCREEN_SPLIT=$sp timeout -k 10 300 python3 bench.py --rows 10000000 --dim 128 --k 64 --dtype f32 --warmup 1 --steps 20 --breakdown > $O/cfg2_split$sp.json 2> $O/cfg2_split$sp.err || { tail -5 $O/cfg2_split$sp.err; exit 1; }
  tail -1 $O/cfg2_split$sp.json | python3 -c "
import json,sys; d=json.loads(sys.stdin.read()); e=d['extra']; b=e['breakdown']
print('split=$sp fit ms', e['fit_s']*1000, 'engine', e['engine_fit_ms'], 'init', b['init_ms'], 'first', b['iteration_ms'][0], 'steps', sum(b['iteration_ms'][1:]), 'rechecked', b.get('screen_rechecked_rank0'))"
done
timeout -k 10 300 rocprofv3 --kernel-trace -d /tmp/scr -o scr -- python3 bench.py --rows 10000000 --dim 128 --k 64 --dtype f32 --warmup 1 --steps 20 --no-overlap > $O/scr.log 2>&1 || { tail -5 $O/scr.log; exit 1; }
python3 scripts/rocpd_stats.py /tmp/scr/scr_results.db --top 14 > $O/cfg2_screen_stats.txt
cat $O/cfg2_screen_stats.txt
