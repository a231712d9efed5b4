#!/bin/bash
# K13 fp8 (config-5 path): GLM kernel tests, then the GLM microbenchmark.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export PYTHONPATH="$GRAFT_REPO_ROOT${PYTHONPATH:+:$PYTHONPATH}"
mkdir -p gpurun_out/glm
timeout -k 10 300 python -u -m pytest tests/test_gpu_glm_trees.py tests/test_ml_more_gpu.py -x -q -m gpu --timeout 200 --timeout-method thread > gpurun_out/glm/tests.log 2>&1 || { tail -20 gpurun_out/glm/tests.log; exit 2; }
tail -2 gpurun_out/glm/tests.log
timeout -k 10 300 python -u scripts/mb_glm.py > gpurun_out/glm/mb.log 2>&1 || exit 3
grep logreg_grad gpurun_out/glm/mb.log
