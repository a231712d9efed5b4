#!/bin/bash
# Offset-form (read-only) pruning bounds: pruning/init/incremental GPU tests, then the headline bench with
# the offset form on and off.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export PYTHONPATH="$GRAFT_REPO_ROOT${PYTHONPATH:+:$PYTHONPATH}"
out=gpurun_out/lazy; mkdir -p $out
timeout -k 10 600 python -u -m pytest tests/test_kmeans_prune.py tests/test_kmeans_init_gpu.py tests/test_kmeans_incremental_gpu.py tests/test_kmeans_kernels_gpu.py tests/test_distributed_gpu_gloo.py -x -q -m gpu --timeout 200 --timeout-method thread > $out/tests.log 2>&1
rc=$?; tail -3 $out/tests.log; [ $rc -eq 0 ] || exit $rc
for l in 1 0 1; do
  CML_KMEANS_LAZY_BOUNDS=$l timeout -k 10 200 python -u bench.py --breakdown > $out/bench_lazy$l.log 2>&1 || exit 4
  tail -1 $out/bench_lazy$l.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); e=d['extra']; print($l, d['value'], e['fit_s'], e['init_s'], e['breakdown']['iteration_ms'][:4], e['steady_state_ms_per_step'], e['training_cost'])"
done
