set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONPATH=$GRAFT_REPO_ROOT
O=gpurun_out/${1:-r4e}
mkdir -p $O
timeout -k 10 200 python3 scripts/dbg_screen.py > $O/dbg_screen.log 2>&1; grep -v amdgpu $O/dbg_screen.log | tail -12
timeout -k 10 200 python3 scripts/mb_glm_fp8.py > $O/mb_glm_fp8.log 2>&1 || { tail -5 $O/mb_glm_fp8.log; exit 1; }
grep -v amdgpu $O/mb_glm_fp8.log
timeout -k 10 300 python3 scripts/mb_dropna.py > $O/mb_dropna.log 2>&1 || { tail -5 $O/mb_dropna.log; exit 1; }
head -10 $O/mb_dropna.log | grep -v amdgpu
python -c "
import sys; sys.path.insert(0, 'examples')
import hospital_resource_prediction as h
h.synth_uploads('/tmp/wfg/hospitals/incoming', n_files=4, rows=1000000)
" || exit 1
timeout -k 10 400 python examples/hospital_resource_prediction.py --master mi355x --out /tmp/wfg --trace > $O/workflow.log 2>&1 || { tail -20 $O/workflow.log; exit 1; }
grep -A24 "^range" $O/workflow.log
