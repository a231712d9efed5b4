# segacc slices from the filled count: KMeans GPU tests, then headline (cap 1/16 vs 1/4) and pipeline (1/4)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/benches
timeout -k 10 300 python -u -m pytest tests/test_kmeans_incremental_gpu.py tests/test_kmeans_kernels_gpu.py tests/test_distributed_gpu_gloo.py -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/pytest_km.log 2>&1 || { grep -E "FAIL|Error|assert" gpurun_out/pytest_km.log | head -20; tail -20 gpurun_out/pytest_km.log; exit 1; }
tail -1 gpurun_out/pytest_km.log
for cap in 0.0625 0.25 0.0625 0.25; do
  CML_KMEANS_DELTA_CAP=$cap timeout -k 10 300 python bench.py --steps 20 --warmup 3 > gpurun_out/benches/bench_cap_$cap.json 2>/dev/null || exit 1
  python -c "import json;d=json.load(open('gpurun_out/benches/bench_cap_$cap.json'));print('cap $cap', round(d['ms_per_step'],3), d['extra']['full_accumulate_ms_per_step'], d['extra']['training_cost'])"
done
for cap in 0.0625 0.25; do
  CML_KMEANS_DELTA_CAP=$cap CML_TRACE=1 timeout -k 10 300 python bench.py --workload pipeline --steps 2 --warmup 1 > gpurun_out/benches/pipe_cap_$cap.log 2>&1 || { tail -20 gpurun_out/benches/pipe_cap_$cap.log; exit 1; }
  echo "pipeline cap $cap"; grep -E "Pipeline.fit|KMeans.fit|kmeans.step " gpurun_out/benches/pipe_cap_$cap.log
done
