# A/B of two kernel-library builds on the same box, interleaved (A B A B): the headline and the 8-GPU shard.
#   build each variant here, copy them to ab/libA.so and ab/libB.so, then on the box:
#   bash scripts/ab_libs.sh OUT [rounds] [h|s|hs]      (headline, shard or both; default both)
# Every run swaps the in-tree library and imports it with CML_NO_AUTOBUILD=1 (no rebuild on the box).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp PYTHONPATH=$PWD CML_NO_AUTOBUILD=1
O=gpurun_out/${1:-ab}
R=${2:-2}
W=${3:-hs}
L=clustermachinelearningforhospitalnetworks_apache_spark_amd/_native/libcml_kernels.so
mkdir -p "$O"
cp "$L" "$O/.orig.so"
for i in $(seq 1 "$R"); do
  for v in A B; do
    cp "ab/lib$v.so" "$L"
    if [[ $W == *h* ]]; then
      timeout -k 10 300 python3 bench.py --no-overlap > "$O/h_${v}_$i.json" 2> "$O/h_${v}_$i.err" \
        || { tail -5 "$O/h_${v}_$i.err"; exit 1; }
    fi
    if [[ $W == *s* ]]; then
      CML_COMM_SELF=1 timeout -k 10 300 python3 bench.py --rows 12500000 --warmup 3 --no-overlap \
        > "$O/s_${v}_$i.json" 2> "$O/s_${v}_$i.err" || { tail -5 "$O/s_${v}_$i.err"; exit 1; }
    fi
    python3 - "$O" "$v" "$i" "$W" <<'PY'
import json, sys
o, v, i, w = sys.argv[1:5]
for tag in [t for t in ("h", "s") if t in w]:
    d = json.loads(open(f"{o}/{tag}_{v}_{i}.json").read().strip().splitlines()[-1])
    e = d["extra"]
    print(f"{v} round {i} {'headline' if tag == 'h' else 'shard   '}: fit {1e3 * e['fit_s']:.2f} ms, engine {e['engine_fit_ms']} ms, "
          f"steady {e.get('steady_state_ms_per_step'):.4f} ms", flush=True)
PY
  done
done
cp "$O/.orig.so" "$L"
