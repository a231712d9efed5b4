# Tree transforms after K21b, then the reference workflow with its phase trace and the long host calls.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/${1:-tree2}
mkdir -p $OUT
timeout -k 10 200 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_glm_trees.py > $OUT/tests.log 2>&1 || { tail -20 $OUT/tests.log; exit 1; }
tail -2 $OUT/tests.log
PYTHONPATH=. timeout -k 10 300 python -u scripts/mb_tree_transform.py > $OUT/tree_transform.log 2>&1 || { tail -5 $OUT/tree_transform.log; exit 1; }
grep -E "transform|fit" $OUT/tree_transform.log | grep -v "  1 " 
python -c "
import sys; sys.path.insert(0, 'examples')
import hospital_resource_prediction as h
h.synth_uploads('/tmp/wfg/hospitals/incoming', n_files=4, rows=1000000)
" || exit 1
timeout -k 10 600 python examples/hospital_resource_prediction.py --master mi355x --out /tmp/wfg --trace > $OUT/workflow.log 2>&1 || { tail -20 $OUT/workflow.log; exit 1; }
tail -30 $OUT/workflow.log
rm -rf /tmp/wfg2; mkdir -p /tmp/wfg2; cp -r /tmp/wfg/hospitals /tmp/wfg2/
timeout -k 10 600 rocprofv3 --kernel-trace --runtime-trace -d /tmp/wp -o wp -- python3 examples/hospital_resource_prediction.py --master mi355x --out /tmp/wfg2 --trace > $OUT/workflow_prof.log 2>&1 || { tail -5 $OUT/workflow_prof.log; exit 1; }
python3 scripts/rocpd_longcalls.py /tmp/wp/wp_results.db --top 30 > $OUT/workflow_longcalls.txt
cat $OUT/workflow_longcalls.txt
