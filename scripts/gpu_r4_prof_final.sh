# Kernel trace of the headline API fit on the final tree: per-kernel table of the timed fit window
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-r4proffinal}
mkdir -p $O
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d /tmp/pf -o pf -- python3 bench.py --warmup 2 --no-overlap > $O/fit.log 2>&1 || { tail -20 $O/fit.log; exit 1; }
tail -1 $O/fit.log | cut -c1-400
python3 scripts/rocpd_stats.py /tmp/pf/pf_results.db --marker row_pass_kernel --index 1 --top 40 > $O/kernel_stats_timed_fit.txt
head -25 $O/kernel_stats_timed_fit.txt
f=$(find /tmp/pf -name "*kernel_stats.csv" | head -1)
[ -n "$f" ] && cp "$f" $O/kernel_stats_whole_run.csv
true
