# Screen diagnostics (split vs plain), config-2 kernel profile (small outputs only)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
export PYTHONPATH=$GRAFT_REPO_ROOT
O=gpurun_out/${1:-r4g}
mkdir -p $O
timeout -k 10 300 python3 scripts/dbg_split.py > $O/dbg_split.log 2>&1 || { tail -20 $O/dbg_split.log; exit 1; }
grep -v amdgpu $O/dbg_split.log
