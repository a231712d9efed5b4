set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${1:-r2g}
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_kmeans_kernels_gpu.py -x -q --timeout 120 --timeout-method thread > $OUT/pytest_km.log 2>&1
rc=$?; tail -3 $OUT/pytest_km.log; [ $rc -eq 0 ] || exit $rc
CML_TRACE=1 timeout -k 10 400 python bench.py --workload pipeline --steps 2 --warmup 1 > $OUT/pipeline.json 2> $OUT/pipeline.err || exit 1
cat $OUT/pipeline.json; grep -A12 "^range" $OUT/pipeline.err
