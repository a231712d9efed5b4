# Cold vs warm na.drop on a 4M-row upload batch, with trace ranges inside dropna / take_rows
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
export PYTHONPATH=$GRAFT_REPO_ROOT
O=gpurun_out/${1:-r4j}
mkdir -p $O
CML_TRACE=1 timeout -k 10 300 python3 scripts/mb_dropna.py > $O/mb_dropna.log 2>&1 || { tail -5 $O/mb_dropna.log; exit 1; }
grep -v amdgpu $O/mb_dropna.log | head -60
python -c "
import sys; sys.path.insert(0, 'examples')
import hospital_resource_prediction as h
h.synth_uploads('/tmp/wfg/hospitals/incoming', n_files=4, rows=1000000)
" || exit 1
timeout -k 10 400 python examples/hospital_resource_prediction.py --master mi355x --out /tmp/wfg --trace > $O/workflow.log 2>&1 || { tail -20 $O/workflow.log; exit 1; }
grep -A12 "^range" $O/workflow.log
