# The reference workflow end to end on one MI355X (4M-row synthetic upload), with the phase trace.
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${1:-wf2}
mkdir -p $OUT
python -c "
import sys; sys.path.insert(0, 'examples')
import hospital_resource_prediction as h
h.synth_uploads('/tmp/wfg/hospitals/incoming', n_files=4, rows=1000000)
" || exit 1
timeout -k 10 600 python examples/hospital_resource_prediction.py --master mi355x --out /tmp/wfg --trace > $OUT/workflow.log 2>&1
rc=$?
tail -60 $OUT/workflow.log
exit $rc
