# unique_rows kernels: the init GPU tests, the k-means GPU tests, then the 8-GPU shard fit on one rank
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
export PYTHONPATH=$GRAFT_REPO_ROOT
O=gpurun_out/${1:-uniq}
mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -p no:cacheprovider tests/test_kmeans_init_gpu.py tests/test_kmeans_kernels_gpu.py tests/test_kmeans_screen_gpu.py tests/test_distributed_gpu_gloo.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
for i in 1 2; do
CML_COMM_SELF=1 timeout -k 10 300 python3 bench.py --rows 12500000 --warmup 3 --no-overlap --breakdown > $O/shard$i.json 2> $O/shard$i.err || { tail -5 $O/shard$i.err; exit 1; }
tail -1 $O/shard$i.json | python3 -c "
import json,sys; d=json.loads(sys.stdin.read()); e=d['extra']; b=e['breakdown']
print('shard fit ms', e['fit_s']*1000, 'engine', e['engine_fit_ms'], 'init', b['init_ms'], 'its', b['iteration_ms'], 'steady', e.get('steady_state_ms_per_step'))"
done
