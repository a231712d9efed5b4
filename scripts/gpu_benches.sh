set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/benches
python -c "import __graft_entry__ as g; g.build()" > gpurun_out/build.log 2>&1 || exit 1
timeout -k 10 300 python bench.py --steps 20 --warmup 3 2>&1 | grep '^{' > gpurun_out/benches/kmeans_100Mx256_k256.json && \
timeout -k 10 300 python bench.py --rows 10000000 --dim 128 --k 64 --steps 50 --warmup 5 2>&1 | grep '^{' > gpurun_out/benches/kmeans_10Mx128_k64.json && \
timeout -k 10 400 python bench.py --workload logreg --steps 10 --warmup 2 2>&1 | grep '^{' > gpurun_out/benches/logreg_100Mx256.json
rc=$?
cat gpurun_out/benches/*.json | cut -c1-330
exit $rc
