# GPU tests of the given files (or all of tests/ with no arguments) in one pytest process.
#   bash scripts/r5/gpu_tests.sh OUTNAME [test files...]
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp PYTHONPATH=$GRAFT_REPO_ROOT
O=gpurun_out/${1:-r5tests}
shift || true
mkdir -p $O
T=${@:-tests}
timeout -k 10 1000 python -u -m pytest -x -v --timeout 120 --timeout-method thread -p no:cacheprovider -m gpu $T > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -3 $O/tests.log
