"""Microbenchmark of the K9r modes (kmeans_rr.h): mode 0 (plain assign + counting-sort ranks), mode 1
(top-2 bounds, the pruned full pass) and mode 2 (candidate positions) on n x d bf16 rows, k centres.
Also the fused row pass. Prints ms per launch (median of reps)."""
import sys
import time

import torch

from clustermachinelearningforhospitalnetworks_apache_spark_amd.models.kmeans import LloydEngine, to_device_matrix
from clustermachinelearningforhospitalnetworks_apache_spark_amd.ops import kmeans_ops as K

n = int(sys.argv[1]) if len(sys.argv) > 1 else 20_000_000
d = int(sys.argv[2]) if len(sys.argv) > 2 else 256
k = int(sys.argv[3]) if len(sys.argv) > 3 else 256
reps = 7
g = torch.Generator(device="cuda").manual_seed(0)
x = torch.empty((n, d), dtype=torch.bfloat16, device="cuda")
cen = torch.randn(k, d, device="cuda", generator=g) * 4
for s in range(0, n, 1 << 22):
    m = min(1 << 22, n - s)
    x[s:s + m] = (cen[torch.randint(0, k, (m,), device="cuda", generator=g)] +
                  torch.randn(m, d, device="cuda", generator=g)).to(torch.bfloat16)
x = to_device_matrix(x, d)
dp = x.shape[1]
kp = -(-k // 32) * 32
cb = torch.zeros((kp, dp), dtype=torch.bfloat16, device="cuda")
cn = torch.zeros(kp, device="cuda")
K.update_centers(None, k, d, cen.double().clone(), cb, dp, kp, cn, None)
xn = torch.empty(n, device="cuda")


def timeit(fn):
    fn()
    torch.cuda.synchronize()
    ts = []
    for _ in range(reps):
        t = time.perf_counter()
        fn()
        torch.cuda.synchronize()
        ts.append(time.perf_counter() - t)
    ts.sort()
    return 1000 * ts[len(ts) // 2]


c0 = cb[0].float().contiguous()
cost = torch.empty(n, device="cuda")
near = torch.empty(n, dtype=torch.int32, device="cuda")
mx = torch.zeros(1, device="cuda")
er = torch.tensor([2 ** 31 - 1, -1], dtype=torch.int32, device="cuda")
t = timeit(lambda: K.row_pass(x, n, dp, xn))
print(f"row pass (norms)            {t:8.3f} ms  {n * dp * 2 / t / 1e9:6.2f} TB/s")
t = timeit(lambda: K.row_pass(x, n, dp, xn, c0, float(cn[0]), cost, near, xn_max=mx, erange=er))
print(f"row pass (fused init)       {t:8.3f} ms  {n * dp * 2 / t / 1e9:6.2f} TB/s")
plan = K.plan_assign(n, dp, k)
lab = torch.zeros(n, dtype=torch.int32, device="cuda")
cp = torch.zeros(plan.grid, dtype=torch.float64, device="cuda")
hist = torch.zeros(plan.grid * plan.kp, dtype=torch.int32, device="cuda")
rank = torch.zeros(n, dtype=torch.int32, device="cuda")
t0 = timeit(lambda: K.assign_bf16(x, n, dp, cb, cn, plan, lab, None, cp, hist, rank, xnorm=xn))
print(f"K9r mode 0 (+ranks)         {t0:8.3f} ms")
ub = torch.zeros(n, device="cuda")
lb = torch.zeros(n, device="cuda")
mc = torch.tensor([float(cn[:k].max())], device="cuda")
tau = LloydEngine.prune_tau(dp)
t1 = timeit(lambda: K.assign_rr_ext(1, x, n, dp, cb, cn, plan, xn, lab, cp, ub, lb, mc, tau, hist=hist, rank=rank))
print(f"K9r mode 1 (top-2, +ranks)  {t1:8.3f} ms  ({100 * (t1 / t0 - 1):+.1f} %)")
t1b = timeit(lambda: K.assign_rr_ext(1, x, n, dp, cb, cn, plan, xn, lab, cp, ub, lb, mc, tau))
print(f"K9r mode 1 (top-2, no ranks){t1b:8.3f} ms")
for frac in (0.02, 0.05, 0.2):
    m = int(n * frac)
    tr = plan.round_rows
    cand = torch.sort(torch.randperm(n, device="cuda", generator=g)[:m]).values.to(torch.int32)
    pad = -(-m // tr) * tr + tr
    idx = torch.zeros(pad, dtype=torch.int32, device="cuda")
    idx[:m] = cand
    cl = torch.zeros(pad, dtype=torch.int32, device="cuda")
    cl[:m] = lab[cand.long()]
    cx = torch.zeros(pad, device="cuda")
    cx[:m] = xn[cand.long()]
    cnt = torch.tensor([m], dtype=torch.int32, device="cuda")
    t2 = timeit(lambda: K.assign_rr_ext(2, x, m, dp, cb, cn, plan, cx, lab, cp, ub, lb, mc, tau, idx=idx, n_dev=cnt,
                                        lab_in=cl))
    print(f"K9r mode 2, {100 * frac:4.1f} % rows     {t2:8.3f} ms  ({m * dp * 2 / t2 / 1e9:5.2f} TB/s of candidate rows;"
          f" full-pass share {t2 / t0:.3f})")

# centre tiles per wave: the k-means|| candidate chunk sizes
for kk in (64, 128, 192, 256, 320):
    kpp_ = -(-kk // 32) * 32
    cbk = torch.zeros((kpp_, dp), dtype=torch.bfloat16, device="cuda")
    cnk = torch.zeros(kpp_, device="cuda")
    cen2 = torch.randn(kk, d, device="cuda", generator=g).double() * 4
    K.update_centers(None, kk, d, cen2.clone(), cbk, dp, kpp_, cnk, None)
    pl = K.plan_assign(n, dp, kk)
    bst = torch.empty(n, device="cuda")
    t = timeit(lambda: K.assign_bf16(x, n, dp, cbk, cnk, pl, lab, bst, None, xnorm=xn))
    print(f"K9r mode 0, k={kk:3d} (CT={pl.rr_ct})     {t:8.3f} ms")
