# Strong-scaling emulation on one GPU: the per-rank shard of an N-GPU headline run (100M/N rows),
# through the multi-rank launch path (eager steps, 2 row chunks) and the 1-rank graph path.
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${1:-strong}
mkdir -p $OUT
for n in 50000000 25000000 12500000; do
  CML_KMEANS_GRAPH=0 timeout -k 10 240 python bench.py --rows $n --chunks 2 --steps 30 --warmup 5 > $OUT/eager_c2_$n.json 2> $OUT/eager_c2_$n.err || exit 1
  timeout -k 10 240 python bench.py --rows $n --steps 30 --warmup 5 > $OUT/graph_c1_$n.json 2> $OUT/graph_c1_$n.err || exit 1
  python3 - $OUT $n <<'PY'
import json, sys
out, n = sys.argv[1], sys.argv[2]
for tag in ("eager_c2", "graph_c1"):
    r = json.load(open(f"{out}/{tag}_{n}.json"))
    print(f"{tag} rows={n}: {r['ms_per_step']:.3f} ms/step  full={r['extra'].get('full_accumulate_ms_per_step', 0):.3f}")
PY
done
