# headline bench, incremental-sums cap 1/16 vs 1/4, alternating processes
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/benches
for cap in 0.0625 0.25 0.0625 0.25; do
  CML_KMEANS_DELTA_CAP=$cap timeout -k 10 300 python bench.py --steps 20 --warmup 3 > gpurun_out/benches/bench_cap_$cap.json 2>/dev/null || exit 1
  python -c "import json;d=json.load(open('gpurun_out/benches/bench_cap_$cap.json'));print('cap $cap', round(d['ms_per_step'],3), d['extra']['full_accumulate_ms_per_step'])"
done
