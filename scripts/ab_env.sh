# A/B of an environment knob on the same box, interleaved: the headline and/or the 8-GPU shard.
#   bash scripts/ab_env.sh OUT VAR "VALUE_A VALUE_B" [rounds] [h|s|hs]
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp PYTHONPATH=$PWD
O=gpurun_out/${1:?out}
VAR=${2:?var}
VALS=${3:?values}
R=${4:-2}
W=${5:-hs}
mkdir -p "$O"
for i in $(seq 1 "$R"); do
  for v in $VALS; do
    if [[ $W == *h* ]]; then
      env "$VAR=$v" timeout -k 10 300 python3 bench.py --no-overlap > "$O/h_${v}_$i.json" 2> "$O/h_${v}_$i.err" \
        || { tail -5 "$O/h_${v}_$i.err"; exit 1; }
    fi
    if [[ $W == *s* ]]; then
      env "$VAR=$v" CML_COMM_SELF=1 timeout -k 10 300 python3 bench.py --rows 12500000 --warmup 3 --no-overlap \
        > "$O/s_${v}_$i.json" 2> "$O/s_${v}_$i.err" || { tail -5 "$O/s_${v}_$i.err"; exit 1; }
    fi
    python3 - "$O" "$v" "$i" "$W" "$VAR" <<'PY'
import json, sys
o, v, i, w, var = sys.argv[1:6]
for tag in [t for t in ("h", "s") if t in w]:
    d = json.loads(open(f"{o}/{tag}_{v}_{i}.json").read().strip().splitlines()[-1])
    e = d["extra"]
    print(f"{var}={v} round {i} {'headline' if tag == 'h' else 'shard   '}: fit {1e3 * e['fit_s']:.2f} ms, "
          f"engine {e['engine_fit_ms']} ms, steady {e.get('steady_state_ms_per_step'):.4f} ms", flush=True)
PY
  done
done
