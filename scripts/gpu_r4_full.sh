# Whole GPU test suite, smoke(), the headline bench and the reference workflow on one tree
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
export PYTHONPATH=$GRAFT_REPO_ROOT
O=gpurun_out/${1:-r4full}
mkdir -p $O
timeout -k 10 1000 python -u -m pytest tests -m gpu -q --timeout 200 --timeout-method thread -p no:cacheprovider > $O/pytest_gpu.log 2>&1
rc=$?
tail -3 $O/pytest_gpu.log
grep -E "FAILED|Error" $O/pytest_gpu.log | head -20
[ $rc -le 1 ] || exit $rc
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || { tail -5 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 400 python3 bench.py > $O/bench.json 2> $O/bench.err || { tail -5 $O/bench.err; exit 1; }
tail -1 $O/bench.json | cut -c1-400
python -c "
import sys; sys.path.insert(0, 'examples')
import hospital_resource_prediction as h
h.synth_uploads('/tmp/wfg/hospitals/incoming', n_files=4, rows=1000000)
" || exit 1
timeout -k 10 400 python examples/hospital_resource_prediction.py --master mi355x --out /tmp/wfg --trace > $O/workflow.log 2>&1 || { tail -20 $O/workflow.log; exit 1; }
grep -A8 "^range" $O/workflow.log
