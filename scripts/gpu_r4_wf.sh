# The reference workflow on 4M uploaded rows (scripts/gpu_workflow2.sh) under cProfile: where the
# per-batch retrain (na.drop + assemble + LR) and the stream read spend host time.
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${1:-r4wf}
mkdir -p $OUT
python -c "
import sys; sys.path.insert(0, 'examples')
import hospital_resource_prediction as h
h.synth_uploads('/tmp/wfg/hospitals/incoming', n_files=4, rows=1000000)
" || exit 1
timeout -k 10 600 python -m cProfile -o $OUT/wf.prof examples/hospital_resource_prediction.py --master mi355x --out /tmp/wfg --trace > $OUT/workflow.log 2>&1
rc=$?
tail -32 $OUT/workflow.log
python -c "
import pstats; s = pstats.Stats('$OUT/wf.prof'); s.sort_stats('cumulative').print_stats(60)" > $OUT/prof_cum.txt
python -c "
import pstats; s = pstats.Stats('$OUT/wf.prof'); s.sort_stats('tottime').print_stats(40)" > $OUT/prof_tot.txt
exit $rc
