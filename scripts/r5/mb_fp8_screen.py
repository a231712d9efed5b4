"""fp8 rows, device pruned Lloyd steps with the MX screen (kmeans_rr.h MODE 3) against the bf16 widening pass
(CML_KMEANS_FP8_SCREEN=0): per-step time and the rows the screen leaves to the bf16 re-check, on config-5
shaped data (32 Gaussian blobs, standardised, e4m3, k = 128).

    python scripts/r5/mb_fp8_screen.py [--rows N] [--dim D] [--k K] [--steps S]
"""
import argparse
import os
import time

import torch

ap = argparse.ArgumentParser()
ap.add_argument("--rows", type=int, default=20_000_000)
ap.add_argument("--dim", type=int, default=512)
ap.add_argument("--k", type=int, default=128)
ap.add_argument("--steps", type=int, default=8)
a = ap.parse_args()

from clustermachinelearningforhospitalnetworks_apache_spark_amd.models.kmeans import LloydEngine  # noqa: E402

dev = torch.device("cuda", 0)
g = torch.Generator(device=dev)
g.manual_seed(7)
n, d, k = a.rows, a.dim, a.k
cen = torch.randn(32, d, generator=g, device=dev) * 3
spread = torch.rand(d, generator=g, device=dev) * 4 + 0.25
x8 = torch.empty((n, d), dtype=torch.float8_e4m3fn, device=dev)
for s0 in range(0, n, 1 << 21):
    m = min(1 << 21, n - s0)
    z = (cen[torch.randint(0, 32, (m,), generator=g, device=dev)] + torch.randn((m, d), generator=g, device=dev))
    z = z * spread
    x8[s0:s0 + m] = (z / (3.2 * spread)).clamp(-440, 440).to(torch.float8_e4m3fn)
    del z
init = x8[torch.randperm(n, generator=torch.Generator().manual_seed(1))[:k].to(dev)].float().double().cpu().numpy()
torch.cuda.synchronize()

labels = {}
for screen in ("1", "0"):
    os.environ["CML_KMEANS_FP8_SCREEN"] = screen
    eng = LloydEngine(x8, d, k, prune=True, use_graph=False)
    eng.set_centers(init)
    eng.step()  # first step (norms, state)
    torch.cuda.synchronize()
    times, stats = [], []
    for _ in range(a.steps):
        t0 = time.perf_counter()
        eng.step()
        torch.cuda.synchronize()
        times.append(1e3 * (time.perf_counter() - t0))
        stats.append(eng.prune_stats())
    labels[screen] = eng.labels[:n].clone()
    print(f"screen={screen}: step ms {[round(t, 2) for t in times]}", flush=True)
    print(f"  stats {[(s['full'], s.get('screen_rechecked')) for s in stats]}", flush=True)
    del eng
    torch.cuda.empty_cache()
print("same labels:", bool(torch.equal(labels["1"], labels["0"])))
