# Run selected GPU tests: TESTS env var (pytest node ids / files)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest ${TESTS} -x -v -m gpu --timeout 200 --timeout-method thread > gpurun_out/pytest_sel.log 2>&1; rc=$?
grep -E "PASS|FAIL|Error|error|assert" gpurun_out/pytest_sel.log | tail -40
tail -3 gpurun_out/pytest_sel.log
exit $rc
