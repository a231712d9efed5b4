# incremental-sums cap (CML_KMEANS_DELTA_CAP, fraction of rows) on the pipeline and the headline
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/benches
for cap in 0.0625 0.25 0.0625 0.25; do
  CML_KMEANS_DELTA_CAP=$cap CML_TRACE=1 timeout -k 10 300 python bench.py --workload pipeline --steps 2 --warmup 1 > gpurun_out/benches/pipe_cap_$cap.log 2>&1 || { tail -20 gpurun_out/benches/pipe_cap_$cap.log; exit 1; }
  echo "cap $cap"; grep -E "Pipeline.fit|KMeans.fit|kmeans.step " gpurun_out/benches/pipe_cap_$cap.log
done
CML_KMEANS_DELTA_CAP=0.25 timeout -k 10 300 python bench.py --steps 20 --warmup 3 > gpurun_out/benches/bench_cap25.json 2>/dev/null || exit 1
cut -c1-400 gpurun_out/benches/bench_cap25.json
