set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
python -c "import __graft_entry__ as g; g.build()" > gpurun_out/build.log 2>&1 || { echo BUILD FAIL; tail -30 gpurun_out/build.log; exit 1; }
timeout -k 10 600 python -m pytest tests -q -m gpu --maxfail=15 > gpurun_out/pytest_gpu.log 2>&1; rc=$?; tail -5 gpurun_out/pytest_gpu.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" 2>&1 | grep -v amdgpu.ids | tail -3
timeout -k 10 400 python bench.py --steps 20 --warmup 3 2>&1 | grep -v amdgpu.ids | tail -2 | tee gpurun_out/bench_full.json
