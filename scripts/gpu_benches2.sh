set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/benches
python -c "import __graft_entry__ as g; g.build()" > gpurun_out/build.log 2>&1 || exit 1
timeout -k 10 400 python bench.py --workload logreg --solver sgd --steps 200 --warmup 10 --batch 1048576 2>&1 | grep '^{' > gpurun_out/benches/logreg_sgd_100Mx256.json && \
timeout -k 10 400 python bench.py --workload logreg --solver sgd --steps 200 --warmup 10 --batch 131072 2>&1 | grep '^{' > gpurun_out/benches/logreg_sgd_100Mx256_b128k.json && \
timeout -k 10 400 python bench.py --workload logreg --steps 10 --warmup 2 2>&1 | grep "^{" > gpurun_out/benches/logreg_100Mx256.json
rc=$?
cat gpurun_out/benches/logreg*.json | cut -c1-400
exit $rc
