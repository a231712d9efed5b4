# A/B of the k-means|| first-round size (CML_KMEANS_INIT_FIRST) on the headline bench: fit, init and first steps per value
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp PYTHONPATH=$PWD
mkdir -p gpurun_out/r6k
for F in 320 256 192 128 64; do
  CML_KMEANS_INIT_FIRST=$F timeout -k 10 300 python3 bench.py --breakdown --no-overlap --warmup 2 > gpurun_out/r6k/first_$F.json 2> gpurun_out/r6k/first_$F.err || exit 1
  tail -1 gpurun_out/r6k/first_$F.json | python3 -c "
import json,sys;d=json.loads(sys.stdin.read());e=d['extra'];b=e['breakdown'];print('$F', e['fit_s'], b['init_ms'], b['iteration_ms'][:2], b.get('init_pruned_rounds_rank0'), e['training_cost_hex'])"
done
