"""In-process A/B of K9 (variant 0) vs K9r (variant 8: register-resident centres + LDS-DMA X ring).

usage: python scripts/mb_assign_rr.py N D K [variants] [fp8]   (variant 9 = K9 with the K9r default off)
Alternates variants round by round (DVFS drift hits both); reports the full assign pass and the
compute-only pass (every row aliases row 0: no HBM stream)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

import bench  # noqa: E402
from clustermachinelearningforhospitalnetworks_apache_spark_amd.models.kmeans import LloydEngine
from clustermachinelearningforhospitalnetworks_apache_spark_amd.ops import kmeans_ops as K

n = int(sys.argv[1]) if len(sys.argv) > 1 else 20_000_000
D = int(sys.argv[2]) if len(sys.argv) > 2 else 256
KC = int(sys.argv[3]) if len(sys.argv) > 3 else 256
variants = [int(v) for v in sys.argv[4].split(",")] if len(sys.argv) > 4 else [0, 8]
FP8 = len(sys.argv) > 5 and sys.argv[5] == "fp8"
x = bench.make_blobs(n, D, KC, seed=1000, device=torch.device("cuda"))
if FP8:
    x = x.to(torch.float8_e4m3fn)
eng = LloydEngine(x, D, KC, use_graph=False)
eng.set_centers(x[:KC].to(torch.float32).double().cpu().numpy())
print(f"n={n} d={D} (padded {eng.dp}) k={KC} {'fp8' if FP8 else 'bf16'}", flush=True)
x0 = torch.as_strided(eng.x, (n, eng.dp), (0, 1))
plans = {}
for v in variants:
    K.set_assign_variant(0 if v == 9 else v)
    K.set_rr_default(v != 9)
    plans[v] = K.plan_assign(n, eng.dp, KC, fp8=FP8)
K.set_assign_variant(0)
K.set_rr_default(True)


def run(v, xx):
    p = plans[v]
    K.assign_bf16(xx, n, eng.dp, eng.cb, eng.cnorm, p, eng.labels, None, eng.cost_part, eng.hist, eng.rank,
                  xnorm=eng.xnorm)


def timed(v, xx, reps=5):
    ts = []
    for _ in range(reps):
        a, b = torch.cuda.Event(True), torch.cuda.Event(True)
        a.record()
        run(v, xx)
        b.record()
        torch.cuda.synchronize()
        ts.append(a.elapsed_time(b))
    return ts


labels = {}
res = {(v, m): [] for v in variants for m in ("full", "compute")}
for rnd in range(5):
    for v in variants:
        eng.labels.fill_(-1)
        run(v, eng.x)
        torch.cuda.synchronize()
        if rnd == 0:
            labels[v] = eng.labels.clone()
        res[(v, "full")] += timed(v, eng.x)
        res[(v, "compute")] += timed(v, x0)
    print(f"round {rnd} done", flush=True)
for v in variants:
    same = float((labels[v] == labels[variants[0]]).float().mean())
    for m in ("full", "compute"):
        ts = sorted(res[(v, m)])
        t = ts[len(ts) // 2]
        print(f"variant {v} (grid {plans[v].grid}, rr_ct {plans[v].rr_ct}) {m:8s}: median {t:.3f} ms (min {ts[0]:.3f})"
              f" -> {2 * n * D * KC / t / 1e9:.0f} TF/s, {n * eng.dp * eng.x.element_size() / t / 1e9:.2f} TB/s;"
              f" label agreement with variant {variants[0]}: {same:.6f}", flush=True)
