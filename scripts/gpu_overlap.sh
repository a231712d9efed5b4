set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
PYTHONPATH=$GRAFT_REPO_ROOT timeout -k 10 300 python scripts/mb_overlap.py 25000000 > gpurun_out/mb_overlap.log 2>&1; rc=$?
grep -v amdgpu.ids gpurun_out/mb_overlap.log | tail -20
exit $rc
