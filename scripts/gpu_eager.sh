set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
PYTHONPATH=$GRAFT_REPO_ROOT timeout -k 10 300 python scripts/mb_eager_vs_graph.py > gpurun_out/mb_eager.log 2>&1; rc=$?
grep -v amdgpu.ids gpurun_out/mb_eager.log | tail -10
exit $rc
