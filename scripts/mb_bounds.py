"""K9p bounds pass on its own (offset-form bounds, the pruned step's read-only pass): cuda-event time of one
launch over N rows with a given candidate fraction, against a plain device copy of the same 12 B/row.

    python scripts/mb_bounds.py [--rows N] [--cand FRACTION] [--k K] [--reps R]
"""
import argparse

import torch

from clustermachinelearningforhospitalnetworks_apache_spark_amd.ops import kmeans_ops as K

ap = argparse.ArgumentParser()
ap.add_argument("--rows", type=int, default=12_500_000)
ap.add_argument("--cand", type=float, default=0.03)
ap.add_argument("--k", type=int, default=256)
ap.add_argument("--reps", type=int, default=20)
a = ap.parse_args()
n, k, dev = a.rows, a.k, torch.device("cuda", 0)
g = torch.Generator(device=dev).manual_seed(3)
lab = torch.randint(0, k, (n,), generator=g, device=dev, dtype=torch.int32)
# offset-form bounds: ub - cu[label], lb + cl[label] with zero drifts; a row is proven when ub <= thr[label]
thr = torch.full((k,), 1.0, device=dev)
ub = torch.where(torch.rand(n, generator=g, device=dev) < a.cand, 2.0, 0.5).to(torch.float32)
lb = torch.full((n,), 0.1, device=dev)
drift = torch.zeros(k, device=dev)
dmax = torch.zeros(3, device=dev)
cum = torch.zeros(2 * k, device=dev)
c2 = torch.full((1,), 1e-3, device=dev)
cap = n
cand = torch.zeros(cap + 1024, dtype=torch.int32, device=dev)
cand_lab = torch.zeros_like(cand)
cand_xn = torch.zeros(cap + 1024, device=dev)
xn = torch.rand(n, generator=g, device=dev)
count = torch.zeros(1, dtype=torch.int32, device=dev)


def run():
    K.prune_bounds(lab, ub, lb, drift, dmax, thr, c2, k, cand, count, xn=xn, cand_lab=cand_lab, cand_xn=cand_xn,
                   cum=cum)


def timed(fn):
    fn()
    torch.cuda.synchronize()
    ts = []
    for _ in range(a.reps):
        s, e = torch.cuda.Event(True), torch.cuda.Event(True)
        s.record()
        fn()
        e.record()
        torch.cuda.synchronize()
        ts.append(s.elapsed_time(e))
    return sorted(ts)[len(ts) // 2]


t = timed(run)
src = torch.empty(3 * n, dtype=torch.int32, device=dev)
dst = torch.empty_like(src)
tc = timed(lambda: dst.copy_(src))
print(f"bounds pass n={n} k={k} candidates {int(count.item())} ({a.cand:.0%}): {1e3 * t:.1f} us "
      f"({12 * n / t / 1e9:.2f} TB/s of bounds); copy of 12 B/row: {1e3 * tc:.1f} us "
      f"({24 * n / tc / 1e9:.2f} TB/s read+write)", flush=True)
m = int(count.item())
rows = cand[:m].long()
want = torch.nonzero(ub > 1.0).flatten()
ok = (torch.equal(torch.sort(rows).values, want) and torch.equal(cand_lab[:m], lab[rows])
      and torch.equal(cand_xn[:m], xn[rows]))
print(f"candidate list (rows, labels, norms) correct: {ok}", flush=True)
if not ok:
    raise SystemExit(1)
