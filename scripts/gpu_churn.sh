set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
PYTHONPATH=$GRAFT_REPO_ROOT timeout -k 10 300 python scripts/mb_label_churn.py 20000000 > gpurun_out/churn.log 2>&1; rc=$?
grep -v amdgpu.ids gpurun_out/churn.log | tail -30
exit $rc
