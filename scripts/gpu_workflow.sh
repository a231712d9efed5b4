set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/wf
python -c "import __graft_entry__ as g; g.build()" > gpurun_out/build.log 2>&1 || exit 1
python -c "
import sys; sys.path.insert(0, 'examples')
import hospital_resource_prediction as h
h.synth_uploads('/tmp/wfg/hospitals/incoming', n_files=4, rows=1000000)
" && \
timeout -k 10 600 python -m cProfile -s cumtime examples/hospital_resource_prediction.py --master mi355x --out /tmp/wfg --trace > gpurun_out/wf/profile.txt 2>&1; rc=$?
grep -B2 -A24 "^range " gpurun_out/wf/profile.txt | cut -c1-160
grep -A40 "Ordered by" gpurun_out/wf/profile.txt | cut -c1-160
exit $rc
