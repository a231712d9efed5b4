# K9 assign A/B in one process: variant 0 (default) vs 7 (PACK4 per-row key merge)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
PYTHONPATH=$GRAFT_REPO_ROOT timeout -k 10 300 python scripts/mb_assign_ab.py 20000000 0,7 > gpurun_out/mb_ab7.log 2>&1 || { tail -5 gpurun_out/mb_ab7.log; exit 1; }
PYTHONPATH=$GRAFT_REPO_ROOT timeout -k 10 300 python scripts/mb_assign_ab.py 20000000 0,7 256 256 fp8 > gpurun_out/mb_ab7_f8.log 2>&1 || { tail -5 gpurun_out/mb_ab7_f8.log; exit 1; }
PYTHONPATH=$GRAFT_REPO_ROOT timeout -k 10 300 python scripts/mb_assign_ab.py 20000000 0,7 128 64 > gpurun_out/mb_ab7_128.log 2>&1 || { tail -5 gpurun_out/mb_ab7_128.log; exit 1; }
grep -hv amdgpu.ids gpurun_out/mb_ab7.log gpurun_out/mb_ab7_f8.log gpurun_out/mb_ab7_128.log
