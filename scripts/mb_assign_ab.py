"""In-process A/B of two K9 assign variants (kmeans_ops.set_assign_variant), 20M x 256, k = 256.

Alternates the variants round by round so clock/DVFS drift hits both equally; reports the full pass and the
compute-only pass (every row aliases row 0, no HBM stream)."""
import sys
import torch
import bench
from clustermachinelearningforhospitalnetworks_apache_spark_amd.models.kmeans import LloydEngine
from clustermachinelearningforhospitalnetworks_apache_spark_amd.ops import kmeans_ops as K

n = int(sys.argv[1]) if len(sys.argv) > 1 else 20_000_000
variants = [int(v) for v in sys.argv[2].split(",")] if len(sys.argv) > 2 else [0, 6]
D = int(sys.argv[3]) if len(sys.argv) > 3 else 256
KC = int(sys.argv[4]) if len(sys.argv) > 4 else 256
FP8 = len(sys.argv) > 5 and sys.argv[5] == "fp8"
x = bench.make_blobs(n, D, KC, seed=1000, device=torch.device("cuda"))
if FP8:
    x = x.to(torch.float8_e4m3fn)
eng = LloydEngine(x, D, KC, use_graph=False)
eng.set_centers(x[:KC].to(torch.float32).double().cpu().numpy())
print(f"n={n} d={D} (padded {eng.dp}) k={KC} {'fp8' if FP8 else 'bf16'}", flush=True)
eng.step()
x0 = torch.as_strided(eng.x, (n, eng.dp), (0, 1))


def run(xx):
    K.assign_bf16(xx, n, eng.dp, eng.cb, eng.cnorm, eng.aplan, eng.labels, None, eng.cost_part, eng.hist,
                  eng.rank, xnorm=eng.xnorm)


def timed(xx, reps=5):
    ts = []
    for _ in range(reps):
        a, b = torch.cuda.Event(True), torch.cuda.Event(True)
        a.record()
        run(xx)
        b.record()
        torch.cuda.synchronize()
        ts.append(a.elapsed_time(b))
    return ts


labels = {}
res = {(v, m): [] for v in variants for m in ("full", "compute")}
for rnd in range(6):
    for v in variants:
        K.set_assign_variant(v)
        run(eng.x)
        torch.cuda.synchronize()
        if rnd == 0:
            labels[v] = eng.labels.clone()
        res[(v, "full")] += timed(eng.x)
        res[(v, "compute")] += timed(x0)
K.set_assign_variant(0)
for v in variants:
    same = bool(torch.equal(labels[v], labels[variants[0]]))
    for m in ("full", "compute"):
        ts = sorted(res[(v, m)])
        t = ts[len(ts) // 2]
        print(f"variant {v} {m:8s}: median {t:.3f} ms (min {ts[0]:.3f}) -> {2 * n * D * KC / t / 1e9:.0f} TF/s"
              f"  labels equal to variant {variants[0]}: {same}", flush=True)
