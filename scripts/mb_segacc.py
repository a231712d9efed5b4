"""Sort-regime accumulate (K10: counting sort + segmented f64 sums, kmeans_segacc) on its own: cuda-event time
of one full accumulate of N x 256 bf16 rows over k = 256 labels, plain and with the seeded step's upper-bound
side output (UB), and the HBM rate of the gathered row reads.

    python scripts/mb_segacc.py [--rows N] [--reps R]
"""
import argparse

import torch

import bench
from clustermachinelearningforhospitalnetworks_apache_spark_amd.models.kmeans import LloydEngine
from clustermachinelearningforhospitalnetworks_apache_spark_amd.ops import kmeans_ops as K

ap = argparse.ArgumentParser()
ap.add_argument("--rows", type=int, default=50_000_000)
ap.add_argument("--reps", type=int, default=5)
a = ap.parse_args()
n, d, k = a.rows, 256, 256
dev = torch.device("cuda", 0)
x = bench.make_blobs(n, d, k, seed=1, device=dev)
eng = LloydEngine(x, d, k, prune=False, use_graph=False)
eng.set_centers(x[:k].double().cpu().numpy())
eng.step()  # labels, ranks and histograms of a full K9r pass
torch.cuda.synchronize()
msg = torch.zeros_like(eng.msgs[0])
ub = torch.empty(n, dtype=torch.float32, device=dev)
gb = n * d * 2 / 1e9
print(f"sum grid scale {eng._qscale!r} (0: plain f64 sums)")


def run(with_ub: bool):
    K.accumulate_sort(x, n, eng.dp, d, eng.labels, eng.rank, eng.hist, eng.aplan, k, eng.cost_part, eng.off,
                      eng.seg, eng.perm, eng.cplan, msg, eng.slots, ub_centres=eng.cb if with_ub else None,
                      ub=ub if with_ub else None, qscale=eng._qscale)


for with_ub in (False, True):
    run(with_ub)
    torch.cuda.synchronize()
    ts = []
    for _ in range(a.reps):
        s, e = torch.cuda.Event(True), torch.cuda.Event(True)
        s.record()
        run(with_ub)
        e.record()
        torch.cuda.synchronize()
        ts.append(s.elapsed_time(e))
    t = min(ts)
    print(f"accumulate_sort n={n} d={d} k={k} ub={with_ub}: best {t:.3f} ms, median {sorted(ts)[len(ts) // 2]:.3f} ms"
          f" ({gb / t:.2f} TB/s of rows)", flush=True)
