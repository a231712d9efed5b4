# Packed-f32 K13/K24: numerics tests, GLM microbench, logreg (config 4) and pipeline (config 5) benches.
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${1:-glmpk}
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_gpu_glm_trees.py tests/test_ml_more_gpu.py -x -q --timeout 200 --timeout-method thread -k "logreg or loss_grad or moments" > $OUT/pytest.log 2>&1 || { tail -20 $OUT/pytest.log; exit 1; }
tail -2 $OUT/pytest.log
PYTHONPATH=$GRAFT_REPO_ROOT timeout -k 10 300 python scripts/mb_glm.py > $OUT/glm.log 2>&1 || exit 1
grep -v amdgpu.ids $OUT/glm.log
timeout -k 10 300 python bench.py --workload logreg --steps 10 --warmup 2 > $OUT/logreg.json 2> $OUT/logreg.err || exit 1
cat $OUT/logreg.json
timeout -k 10 400 python bench.py --workload pipeline --steps 2 --warmup 1 > $OUT/pipeline.json 2> $OUT/pipeline.err || exit 1
cat $OUT/pipeline.json
