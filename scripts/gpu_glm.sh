set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
python -c "import __graft_entry__ as g; g.build()" > gpurun_out/build.log 2>&1 || { tail -20 gpurun_out/build.log; exit 1; }
timeout -k 10 600 python -m pytest tests/test_gpu_glm_trees.py tests/test_gpu_frame_kernels.py -q -m gpu -x 2>&1 | tail -5 && \
PYTHONPATH=$GRAFT_REPO_ROOT timeout -k 10 300 python scripts/mb_glm.py 2>&1 | grep -v amdgpu.ids && \
CML_TRACE=1 timeout -k 10 600 python bench.py --workload pipeline --steps 1 --warmup 1 2>&1 | grep -v amdgpu.ids | tail -10 | cut -c1-200
