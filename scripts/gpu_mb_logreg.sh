set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/mb
PYTHONPATH=$GRAFT_REPO_ROOT timeout -k 10 400 python scripts/mb_logreg.py gpurun_out/mb/logreg.json > gpurun_out/mb/logreg.log 2>&1
rc=$?
grep -v amdgpu.ids gpurun_out/mb/logreg.log | tail -40
exit $rc
