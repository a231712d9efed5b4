"""Host-side (Python) time of a KMeans fit on the GPU: cProfile of the timed public-API fit after a warm-up,
top functions by own time and by cumulative time. The GPU work is asynchronous, so what this shows is the
launch path and the host work between the fit's synchronising reads (scripts/sync_audit.py lists those).

    CML_COMM_SELF=1 python scripts/prof_host.py [--rows N] [--dim D] [--k K] [--iters I] [--top T]
"""
import argparse
import cProfile
import io
import pstats
import time

import torch

ap = argparse.ArgumentParser()
ap.add_argument("--rows", type=int, default=12_500_000)
ap.add_argument("--dim", type=int, default=256)
ap.add_argument("--k", type=int, default=256)
ap.add_argument("--iters", type=int, default=20)
ap.add_argument("--top", type=int, default=45)
a = ap.parse_args()

import bench  # noqa: E402
from clustermachinelearningforhospitalnetworks_apache_spark_amd.ml.clustering import KMeans  # noqa: E402
from clustermachinelearningforhospitalnetworks_apache_spark_amd.sql import SparkSession  # noqa: E402

spark = SparkSession.builder.master("mi355x").getOrCreate()
x = bench.make_blobs(a.rows, a.dim, a.k, seed=1, device=torch.device("cuda", 0))
df = spark.createDataFrameFromTensors({"features": x})
for _ in range(2):
    KMeans(k=a.k, maxIter=a.iters, tol=0.0, seed=42).fit(df)  # warm-up (kernel loads, allocator, norms)
torch.cuda.synchronize()
pr = cProfile.Profile()
t0 = time.perf_counter()
pr.enable()
KMeans(k=a.k, maxIter=a.iters, tol=0.0, seed=42).fit(df)
torch.cuda.synchronize()
pr.disable()
print(f"fit wall {1e3 * (time.perf_counter() - t0):.2f} ms (under cProfile)")
for key in ("tottime", "cumulative"):
    s = io.StringIO()
    pstats.Stats(pr, stream=s).sort_stats(key).print_stats(a.top)
    print(f"=== by {key}")
    print("\n".join(line for line in s.getvalue().splitlines() if line.strip())[:20000])
