set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
python -c "import __graft_entry__ as g; g.build()" > gpurun_out/build.log 2>&1 || { echo BUILD FAIL; tail -30 gpurun_out/build.log; exit 1; }
timeout -k 10 900 python -m pytest tests -q -m gpu --maxfail=20 ${PYTEST_ARGS} > gpurun_out/pytest_gpu.log 2>&1; rc=$?
grep -E "passed|failed|Error|error" gpurun_out/pytest_gpu.log | tail -30
exit $rc
