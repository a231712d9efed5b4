# Cold vs warm na.drop on a 4M-row upload batch, with trace ranges inside dropna / take_rows
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
export PYTHONPATH=$GRAFT_REPO_ROOT
O=gpurun_out/${1:-r4j}
mkdir -p $O
CML_TRACE=1 timeout -k 10 300 python3 scripts/mb_dropna.py > $O/mb_dropna.log 2>&1 || { tail -5 $O/mb_dropna.log; exit 1; }
grep -v amdgpu $O/mb_dropna.log | head -60
