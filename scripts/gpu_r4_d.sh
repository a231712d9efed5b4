# Multi-rank device tests (fixed all-gather layout), screen tests, config-2 screen fit + kernel profile
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-r4d}
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_distributed_gpu_gloo.py tests/test_kmeans_screen_gpu.py tests/test_kmeans_exact_gpu.py tests/test_kmeans_api_gpu.py -v -m gpu --timeout 200 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1
rc=$?
tail -3 $O/pytest.log
grep -E "FAILED|ERROR" $O/pytest.log | head -20
[ $rc -le 1 ] || exit $rc
timeout -k 10 300 python3 bench.py --rows 10000000 --dim 128 --k 64 --dtype f32 --warmup 1 --steps 20 --breakdown > $O/cfg2_screen.json 2> $O/cfg2_screen.err || { tail -5 $O/cfg2_screen.err; exit 1; }
tail -1 $O/cfg2_screen.json | python3 -c "
import json,sys; d=json.loads(sys.stdin.read()); e=d['extra']
print('cfg2 f32 screen fit ms', e['fit_s']*1000, e['precision'], 'init', e['breakdown']['init_ms'], e['breakdown']['iteration_ms'][:5])"
timeout -k 10 300 rocprofv3 --kernel-trace -d $O/scr -o scr -- python3 bench.py --rows 10000000 --dim 128 --k 64 --dtype f32 --warmup 1 --steps 20 --no-overlap > $O/scr.log 2>&1 || { tail -5 $O/scr.log; exit 1; }
python3 scripts/rocpd_stats.py $O/scr/scr_results.db --marker to_bf16_err --index 1 --top 25
PYTHONPATH=$GRAFT_REPO_ROOT timeout -k 10 200 python3 scripts/mb_glm_fp8.py > $O/mb_glm_fp8.log 2>&1 || { tail -5 $O/mb_glm_fp8.log; exit 1; }
cat $O/mb_glm_fp8.log | grep -v amdgpu
timeout -k 10 300 python3 scripts/mb_dropna.py > $O/mb_dropna.log 2>&1 || { tail -5 $O/mb_dropna.log; exit 1; }
head -10 $O/mb_dropna.log | grep -v amdgpu
python -c "
import sys; sys.path.insert(0, 'examples')
import hospital_resource_prediction as h
h.synth_uploads('/tmp/wfg/hospitals/incoming', n_files=4, rows=1000000)
" || exit 1
timeout -k 10 400 python examples/hospital_resource_prediction.py --master mi355x --out /tmp/wfg --trace > $O/workflow.log 2>&1 || { tail -20 $O/workflow.log; exit 1; }
grep -A24 "^range" $O/workflow.log
