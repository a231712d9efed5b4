"""Certified f32 path (BASELINE config-2 shape, 10M x 128 f32, k = 64): public-API fit time and the time of
KMeansModel.transform's prediction column (certified screen, exact f64 labels) and computeCost, each against
exact_assign (labels and cost must match bit for bit).

    python scripts/mb_cert.py [--rows N] [--dim D] [--k K] [--reps R]
"""
import argparse
import time

import numpy as np
import torch

ap = argparse.ArgumentParser()
ap.add_argument("--rows", type=int, default=10_000_000)
ap.add_argument("--dim", type=int, default=128)
ap.add_argument("--k", type=int, default=64)
ap.add_argument("--reps", type=int, default=3)
a = ap.parse_args()

import bench  # noqa: E402
from clustermachinelearningforhospitalnetworks_apache_spark_amd.ml.clustering import KMeans  # noqa: E402
from clustermachinelearningforhospitalnetworks_apache_spark_amd.ops import kmeans_ops as K  # noqa: E402
from clustermachinelearningforhospitalnetworks_apache_spark_amd.sql import SparkSession  # noqa: E402

dev = torch.device("cuda", 0)
spark = SparkSession.builder.master("mi355x").getOrCreate()
x = bench.make_blobs(a.rows, a.dim, a.k, seed=1, device=dev).to(torch.float32)
df = spark.createDataFrameFromTensors({"features": x})
km = KMeans(k=a.k, maxIter=20, tol=0.0, seed=42)
km.fit(df)  # warm-up
fits = []
for _ in range(a.reps):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    model = km.fit(df)
    torch.cuda.synchronize()
    fits.append(1e3 * (time.perf_counter() - t0))
print(f"fit ms {[round(t, 2) for t in fits]}", flush=True)
tr = []
for _ in range(a.reps + 1):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    pred = model.transform(df)._column_data("prediction").values
    torch.cuda.synchronize()
    tr.append(1e3 * (time.perf_counter() - t0))
print(f"transform (prediction column materialised) ms {[round(t, 2) for t in tr]}", flush=True)
t0 = time.perf_counter()
cost = model.computeCost(df)
torch.cuda.synchronize()
print(f"computeCost {cost} in {1e3 * (time.perf_counter() - t0):.2f} ms", flush=True)
cen = torch.as_tensor(np.stack(model.clusterCenters()), dtype=torch.float64, device=dev)
t0 = time.perf_counter()
lab_ex, d_ex = K.exact_assign(x, cen)
torch.cuda.synchronize()
print(f"exact_assign {1e3 * (time.perf_counter() - t0):.2f} ms; labels equal: "
      f"{bool(torch.equal(lab_ex.long(), pred.long()))}; cost equal: {cost == float(d_ex.sum().item())}", flush=True)
