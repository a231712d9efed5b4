set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
PYTHONPATH=$GRAFT_REPO_ROOT timeout -k 10 400 python scripts/mb_trees.py > gpurun_out/mb_trees.log 2>&1; rc=$?
grep -v amdgpu.ids gpurun_out/mb_trees.log | tail -10
exit $rc
