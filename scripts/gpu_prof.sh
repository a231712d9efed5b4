set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/prof
export TMPDIR=/tmp
python -c "import __graft_entry__ as g; g.build()" > gpurun_out/build.log 2>&1 || exit 1
PYTHONPATH=$GRAFT_REPO_ROOT timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o mb -- python3 scripts/mb_accum.py > gpurun_out/prof/mb.log 2>&1
rc=$?; grep -v amdgpu.ids gpurun_out/prof/mb.log | tail -8
for f in $(find gpurun_out/prof -name "*kernel_stats.csv"); do cut -d, -f1-4 $f | head -14 | cut -c1-200; done
exit $rc
