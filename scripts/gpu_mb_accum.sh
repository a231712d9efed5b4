set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
PYTHONPATH=$GRAFT_REPO_ROOT timeout -k 10 400 python scripts/mb_accum.py > gpurun_out/mb_accum.log 2>&1; rc=$?
grep -v amdgpu.ids gpurun_out/mb_accum.log | tail -40
exit $rc
