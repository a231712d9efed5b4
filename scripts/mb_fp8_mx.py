"""fp8 rows: the K9r assign with MX-scaled fp8 MFMAs (kmeans_rr.h compute_mx, default) against the bf16
widening pass (K.set_fp8_mx(False)), on config-5 shaped data (32 Gaussian blobs, standardised, e4m3, k = 128):
one full assign pass, and device pruned Lloyd steps of a fresh engine each way. Labels of the two arithmetics
may differ inside the rounding band only (tests/test_kmeans_mx_gpu.py).

    python scripts/mb_fp8_mx.py [--rows N] [--dim D] [--k K] [--steps S]
"""
import argparse
import time

import torch

ap = argparse.ArgumentParser()
ap.add_argument("--rows", type=int, default=20_000_000)
ap.add_argument("--dim", type=int, default=512)
ap.add_argument("--k", type=int, default=128)
ap.add_argument("--steps", type=int, default=8)
a = ap.parse_args()

from clustermachinelearningforhospitalnetworks_apache_spark_amd.models.kmeans import LloydEngine  # noqa: E402
from clustermachinelearningforhospitalnetworks_apache_spark_amd.ops import kmeans_ops as K  # noqa: E402

dev = torch.device("cuda", 0)
g = torch.Generator(device=dev)
g.manual_seed(7)
n, d, k = a.rows, a.dim, a.k
cen = torch.randn(32, d, generator=g, device=dev) * 3
x8 = torch.empty((n, d), dtype=torch.float8_e4m3fn, device=dev)
for s0 in range(0, n, 1 << 21):
    m = min(1 << 21, n - s0)
    z = cen[torch.randint(0, 32, (m,), generator=g, device=dev)] + torch.randn((m, d), generator=g, device=dev)
    x8[s0:s0 + m] = (z / 3.2).clamp(-440, 440).to(torch.float8_e4m3fn)
    del z
init = x8[torch.randperm(n, generator=torch.Generator().manual_seed(1))[:k].to(dev)].float().double().cpu().numpy()
torch.cuda.synchronize()


def ms(fn, reps=5):
    fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        fn()
    torch.cuda.synchronize()
    return 1e3 * (time.perf_counter() - t0) / reps


labels = {}
for mx in (True, False):
    K.set_fp8_mx(mx)
    eng = LloydEngine(x8, d, k, prune=True, use_graph=False)
    eng.set_centers(init)
    eng.step()  # first step (norms, state)
    lab = torch.empty(n, dtype=torch.int32, device=dev)
    best = torch.empty(n, dtype=torch.float32, device=dev)
    t_pass = ms(lambda: K.assign_bf16(x8, n, eng.dp, eng.cb, eng.cnorm, eng.aplan, lab, best, None,
                                      xnorm=eng.xnorm))
    times, full = [], []
    for _ in range(a.steps):
        t0 = time.perf_counter()
        eng.step()
        torch.cuda.synchronize()
        times.append(1e3 * (time.perf_counter() - t0))
        full.append(eng.prune_stats()["full"])
    labels[mx] = eng.labels[:n].clone()
    print(f"mx={mx}: K9r pass {t_pass:.2f} ms ({n * k * d * 2 / t_pass / 1e9:.0f} TFLOP/s); pruned steps ms "
          f"{[round(t, 2) for t in times]} full {full}", flush=True)
    del eng
    torch.cuda.empty_cache()
K.set_fp8_mx(True)
print("labels differing after the steps:", int((labels[True] != labels[False]).sum().item()), "of", n)
