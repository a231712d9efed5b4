# Tree-model transforms of the reference workflow on one GPU (mb_tree_transform.py).
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${1:-tree}
mkdir -p $OUT
PYTHONPATH=. timeout -k 10 300 python -u scripts/mb_tree_transform.py > $OUT/tree_transform.log 2>&1
PYTHONPATH=. timeout -k 10 300 rocprofv3 --kernel-trace --runtime-trace -d /tmp/tt -o tt -- python3 scripts/mb_tree_transform.py > $OUT/prof.log 2>&1 || { tail -5 $OUT/prof.log; exit 1; }
python3 scripts/rocpd_longcalls.py /tmp/tt/tt_results.db --top 25 > $OUT/longcalls.txt
cat $OUT/longcalls.txt
