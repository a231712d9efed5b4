set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/mb
python -c "import __graft_entry__ as g; g.build()" > gpurun_out/build.log 2>&1 || exit 1
PYTHONPATH=$GRAFT_REPO_ROOT timeout -k 10 400 python scripts/mb_logreg.py gpurun_out/mb/logreg.json > gpurun_out/mb/logreg.log 2>&1
rc=$?
cat gpurun_out/mb/logreg.log | tail -30
exit $rc
