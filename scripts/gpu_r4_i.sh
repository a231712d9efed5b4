# Pruned-step backoff + no pruned init at Dp 512: prune/init/API tests, overlap headline, config-5 pipeline
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-r4i}
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_kmeans_prune.py tests/test_kmeans_init_gpu.py tests/test_kmeans_api_gpu.py tests/test_distributed_gpu_gloo.py -v -m gpu --timeout 200 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1
rc=$?
tail -2 $O/pytest.log
grep -E "FAILED|Error" $O/pytest.log | head -20
[ $rc -le 1 ] || exit $rc
timeout -k 10 300 python3 bench.py --data overlap --warmup 1 --breakdown --no-overlap > $O/overlap.json 2> $O/overlap.err || { tail -5 $O/overlap.err; exit 1; }
tail -1 $O/overlap.json | python3 -c "
import json,sys; d=json.loads(sys.stdin.read()); e=d['extra']; b=e['breakdown']
print('overlap: fit ms', round(e['fit_s']*1000,1), 'init', b['init_ms'], 'steps', [round(t,1) for t in b['iteration_ms']], 'full', e.get('full_step_ms'), e.get('full_step_from_scratch_ms'))"
CML_TRACE=1 timeout -k 10 500 python3 bench.py --workload pipeline --steps 2 --warmup 1 > $O/pipe.json 2> $O/pipe.err || { tail -20 $O/pipe.err; exit 1; }
cut -c1-200 $O/pipe.json
grep -A10 "^range" $O/pipe.err
