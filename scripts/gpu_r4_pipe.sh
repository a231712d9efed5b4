# Config-5 pipeline (125M x 512 per GPU, fp8 features): phase trace + kernel stats of the timed fits
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-r4pipe}
mkdir -p $O
CML_TRACE=1 timeout -k 10 500 python3 bench.py --workload pipeline --steps 2 --warmup 1 > $O/pipe.json 2> $O/pipe.err || { tail -20 $O/pipe.err; exit 1; }
cut -c1-400 $O/pipe.json
grep -A30 "^range" $O/pipe.err
timeout -k 10 500 rocprofv3 --kernel-trace -d $O/tr -o tr -- python3 bench.py --workload pipeline --steps 1 --warmup 1 > $O/tr.log 2>&1 || { tail -5 $O/tr.log; exit 1; }
python3 scripts/rocpd_stats.py $O/tr/tr_results.db --top 40 > $O/kernel_stats.txt
head -45 $O/kernel_stats.txt
