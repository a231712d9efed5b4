# One iteration of the shard work: init-table / gather / seed kernel tests, the sync audit of a fit, then
# the shard timeline (scripts/r5/gpu_shard_timeline.sh).
#   bash scripts/r5/gpu_shard_iter.sh OUTNAME
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp PYTHONPATH=$GRAFT_REPO_ROOT
O=gpurun_out/${1:-r5it}
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -p no:cacheprovider -m gpu tests/test_kmeans_init_gpu.py tests/test_kmeans_api_gpu.py tests/test_kmeans_prune.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
timeout -k 10 300 python3 scripts/r5/sync_audit.py --rows 2000000 > $O/sync_audit.txt 2>&1 || { tail -20 $O/sync_audit.txt; exit 1; }
head -40 $O/sync_audit.txt
bash scripts/r5/gpu_shard_timeline.sh ${1:-r5it}
