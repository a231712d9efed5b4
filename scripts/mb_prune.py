"""Pruned Lloyd step breakdown: per-phase wall time (device-synchronised trace ranges) and the
candidate count of every step, on the bench's data (100M x 256 bf16, k = 256 by default)."""
import argparse
import sys
import time

import torch

sys.path.insert(0, ".")
from bench import make_blobs  # noqa: E402
from clustermachinelearningforhospitalnetworks_apache_spark_amd.models.kmeans import LloydEngine  # noqa: E402
from clustermachinelearningforhospitalnetworks_apache_spark_amd.utils.trace import TRACER  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--rows", type=int, default=100_000_000)
ap.add_argument("--dim", type=int, default=256)
ap.add_argument("--k", type=int, default=256)
ap.add_argument("--steps", type=int, default=10)
ap.add_argument("--warmup", type=int, default=3)
a = ap.parse_args()
x = make_blobs(a.rows, a.dim, a.k, seed=1000, device=torch.device("cuda", 0))
eng = LloydEngine(x, a.dim, a.k, prune=True)
eng.set_centers(eng.init_kmeans_parallel(seed=42))
for i in range(a.warmup):
    eng.step()
    print("warmup", i, eng.prune_stats(), flush=True)
torch.cuda.synchronize()
t0 = time.perf_counter()
for i in range(a.steps):
    eng.step()
torch.cuda.synchronize()
print(f"untraced: {1e3 * (time.perf_counter() - t0) / a.steps:.3f} ms/step", flush=True)
TRACER.enable(sync=True)
TRACER.reset()
for i in range(a.steps):
    eng.step()
    print("step", i, eng.prune_stats(), flush=True)
print(TRACER.report())
