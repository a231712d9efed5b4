set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/prof
export TMPDIR=/tmp
python -c "import __graft_entry__ as g; g.build()" > gpurun_out/build.log 2>&1 || exit 1
timeout -k 10 300 python -m pytest tests/test_kmeans_kernels_gpu.py -x -q 2>&1 | tail -3
PYTHONPATH=$GRAFT_REPO_ROOT timeout -k 10 300 python scripts/mb_assign_ablate.py 2>&1 | grep -v amdgpu.ids
