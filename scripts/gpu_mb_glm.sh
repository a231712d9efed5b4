set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/mb
python -c "import __graft_entry__ as g; g.build()" > gpurun_out/build.log 2>&1 || exit 1
PYTHONPATH=$GRAFT_REPO_ROOT timeout -k 10 400 python scripts/mb_glm.py > gpurun_out/mb/glm.log 2>&1
rc=$?
tail -30 gpurun_out/mb/glm.log
exit $rc
