# K9 assign A/B in one process (variant 0 = default build, 6 = per-sub-tile accumulator seeding)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
PYTHONPATH=$GRAFT_REPO_ROOT timeout -k 10 300 python scripts/mb_assign_ab.py 20000000 0,6 > gpurun_out/mb_ab.log 2>&1 || { tail -5 gpurun_out/mb_ab.log; exit 1; }
grep -v amdgpu.ids gpurun_out/mb_ab.log
