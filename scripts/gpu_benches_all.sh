# All bench.py workloads on one GPU (JSON lines under gpurun_out/benches)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/benches
timeout -k 10 300 python bench.py --steps 20 --warmup 3 > gpurun_out/benches/kmeans.json 2> gpurun_out/benches/kmeans.err || exit 1
timeout -k 10 300 python bench.py --rows 10000000 --dim 128 --k 64 --steps 50 --warmup 5 > gpurun_out/benches/kmeans_10Mx128.json 2> gpurun_out/benches/k2.err || exit 1
timeout -k 10 300 python bench.py --workload logreg --steps 10 --warmup 2 > gpurun_out/benches/logreg.json 2> gpurun_out/benches/logreg.err || exit 1
timeout -k 10 300 python bench.py --workload logreg --solver sgd --steps 200 --warmup 20 > gpurun_out/benches/logreg_sgd.json 2> gpurun_out/benches/sgd.err || exit 1
timeout -k 10 300 python bench.py --workload logreg --solver sgd --batch 131072 --steps 500 --warmup 50 > gpurun_out/benches/logreg_sgd_128k.json 2> gpurun_out/benches/sgd2.err || exit 1
timeout -k 10 600 python bench.py --workload pipeline --steps 2 --warmup 1 > gpurun_out/benches/pipeline.json 2> gpurun_out/benches/pipe.err || exit 1
for f in gpurun_out/benches/*.json; do python -c "import json,sys;d=json.load(open('$f'));print('$f', d['value'], d['ms_per_step'])"; done
