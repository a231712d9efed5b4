set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/prof_sgd
python -c "import __graft_entry__ as g; g.build()" > gpurun_out/build.log 2>&1 || exit 1
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_sgd -o sgd -- python3 bench.py --workload logreg --solver sgd --steps 100 --warmup 5 --batch 131072 > gpurun_out/prof_sgd/bench.log 2>&1
rc=$?
find gpurun_out/prof_sgd -name '*kernel_stats.csv' -exec cat {} \; | cut -c1-220
exit $rc
