# Kernel trace + stats of the headline bench (API fit), no overlap fit
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/r4prof
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/r4prof/fit -o fit -- python3 bench.py --warmup 2 --no-overlap > gpurun_out/r4prof/fit.log 2>&1 || { tail -20 gpurun_out/r4prof/fit.log; exit 1; }
tail -1 gpurun_out/r4prof/fit.log | cut -c1-600
find gpurun_out/r4prof -name "*kernel_stats.csv" | head -3
f=$(find gpurun_out/r4prof -name "*kernel_stats.csv" | head -1)
python3 scripts/kstats.py "$f" 30
