# Round-2 GPU check: full GPU test suite, headline bench, rocprofv3 kernel stats of the bench.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r2}
mkdir -p $OUT/prof
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1
rc=$?; tail -3 $OUT/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $OUT/bench.json 2> $OUT/bench.err || exit 1
cat $OUT/bench.json
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o bench -- python3 bench.py --steps 10 --warmup 2 > $OUT/prof/bench.log 2>&1 || exit 1
for f in $(find $OUT/prof -name "*kernel_stats.csv"); do python3 scripts/kstats.py $f 12; done
