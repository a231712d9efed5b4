"""Where the KMeans fit synchronises with the device: torch's sync debug mode reports every synchronising
torch call (blocking copies, .item(), nonzero, ...) of one public-API fit, with the Python stack that made it.

    python scripts/sync_audit.py [--rows N] [--dim D] [--k K]
"""
import argparse
import collections
import traceback
import warnings

import torch

ap = argparse.ArgumentParser()
ap.add_argument("--rows", type=int, default=2_000_000)
ap.add_argument("--dim", type=int, default=256)
ap.add_argument("--k", type=int, default=256)
ap.add_argument("--iters", type=int, default=20)
a = ap.parse_args()

import bench  # noqa: E402
from clustermachinelearningforhospitalnetworks_apache_spark_amd.ml.clustering import KMeans  # noqa: E402
from clustermachinelearningforhospitalnetworks_apache_spark_amd.sql import SparkSession  # noqa: E402

spark = SparkSession.builder.master("mi355x").getOrCreate()
x = bench.make_blobs(a.rows, a.dim, a.k, seed=1, device=torch.device("cuda", 0))
df = spark.createDataFrameFromTensors({"features": x})
KMeans(k=a.k, maxIter=3, tol=0.0, seed=7).fit(df)  # warm-up (kernel loads, allocator)
bench._drop_norm_cache(x)
torch.cuda.synchronize()

sites = collections.Counter()


def show(message, category, filename, lineno, file=None, line=None):
    st = [f for f in traceback.extract_stack()[:-2] if "clustermachinelearning" in f.filename or "bench" in f.filename]
    key = " <- ".join(f"{f.filename.split('/')[-1]}:{f.lineno} {f.name}" for f in st[-4:][::-1])
    sites[key] += 1


warnings.showwarning = show
warnings.simplefilter("always")
torch.cuda.set_sync_debug_mode("warn")
KMeans(k=a.k, maxIter=a.iters, tol=0.0, seed=42).fit(df)
torch.cuda.set_sync_debug_mode(0)
print(f"synchronising calls in one fit: {sum(sites.values())}")
for k, v in sites.most_common():
    print(f"{v:4d}  {k}")
