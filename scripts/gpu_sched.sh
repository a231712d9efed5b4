set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
PYTHONPATH=$GRAFT_REPO_ROOT timeout -k 10 300 python scripts/mb_assign_sched.py ${MB_ARGS} > gpurun_out/mb_sched.log 2>&1; rc=$?
grep -v amdgpu.ids gpurun_out/mb_sched.log | tail -30
exit $rc
