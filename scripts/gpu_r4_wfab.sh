# Reference workflow end to end (4M uploaded rows), session warm-up on / off, wall time of the process.
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${1:-wfab}
mkdir -p $OUT
python -c "
import sys; sys.path.insert(0, 'examples')
import hospital_resource_prediction as h
h.synth_uploads('/tmp/wfsrc/hospitals/incoming', n_files=4, rows=1000000)
" || exit 1
for i in 1 2 3 4; do
  w=$(( i == 4 ? 0 : 1 ))
  rm -rf /tmp/wf$i; mkdir -p /tmp/wf$i; cp -r /tmp/wfsrc/hospitals /tmp/wf$i/
  t0=$(date +%s.%N)
  CML_SINK_ASYNC=${SINK_ASYNC:-1} CML_SESSION_WARMUP=$w timeout -k 10 300 python examples/hospital_resource_prediction.py --master mi355x --out /tmp/wf$i --trace > $OUT/wf_$i.log 2>&1 || { tail -20 $OUT/wf_$i.log; exit 1; }
  t1=$(date +%s.%N)
  python -c "print('warmup=$w wall s', round($t1 - $t0, 3))" | tee -a $OUT/summary.txt
  grep -E "^stream.batch|^DataFrame.dropna|^frame.take_rows |fit  |transform  " $OUT/wf_$i.log | head -14 >> $OUT/summary.txt
done
cat $OUT/summary.txt
