"""Tree model transforms of the reference workflow (ref.py:130-160) on one GPU: the workflow trace showed
RandomForestRegressionModel.transform at 766 ms against 1-9 ms for the other tree transforms. Each call
is bracketed by device syncs; the first RF-regression transform also runs under cProfile."""
import cProfile
import io
import os
import pstats
import sys
import time

import torch

from clustermachinelearningforhospitalnetworks_apache_spark_amd.ml.classification import (  # noqa: E402
    DecisionTreeClassifier, RandomForestClassifier)
from clustermachinelearningforhospitalnetworks_apache_spark_amd.ml.feature import VectorAssembler  # noqa: E402
from clustermachinelearningforhospitalnetworks_apache_spark_amd.ml.regression import (  # noqa: E402
    DecisionTreeRegressor, RandomForestRegressor)
from clustermachinelearningforhospitalnetworks_apache_spark_amd.sql import SparkSession  # noqa: E402

ROWS = int(os.environ.get("MB_ROWS", 2_000_000))
spark = SparkSession.builder.master("mi355x" if torch.cuda.is_available() else "local[4]").getOrCreate()
dev = spark._device
g = torch.Generator(device=dev).manual_seed(0)
cols = {c: torch.randint(0, 100, (ROWS,), generator=g, device=dev).to(torch.int32)
        for c in ("admission_count", "current_occupancy", "emergency_visits")}
cols["seasonality_index"] = torch.rand(ROWS, generator=g, device=dev, dtype=torch.float64)
los = (cols["admission_count"].double() * 0.05 + cols["seasonality_index"] * 3
       + torch.rand(ROWS, generator=g, device=dev, dtype=torch.float64))
cols["length_of_stay"] = los
cols["LOS_binary"] = (los > 5.0).to(torch.int32)
df = spark.createDataFrameFromTensors(cols)
feats = ["admission_count", "current_occupancy", "emergency_visits", "seasonality_index"]


def sync():
    if torch.cuda.is_available():
        torch.cuda.synchronize()


def timed(name, fn):
    sync()
    t = time.perf_counter()
    out = fn()
    sync()
    print(f"{name:36s} {1000 * (time.perf_counter() - t):9.2f} ms", flush=True)
    return out


data = VectorAssembler(inputCols=feats, outputCol="features").transform(df).select("features", "length_of_stay")
tr, te = data.randomSplit([0.7, 0.3], seed=42)
dt = timed("DecisionTreeRegressor.fit", lambda: DecisionTreeRegressor(featuresCol="features",
                                                                      labelCol="length_of_stay").fit(tr))
timed("DecisionTreeRegressionModel.transform", lambda: dt.transform(te))
rf = timed("RandomForestRegressor.fit", lambda: RandomForestRegressor(featuresCol="features",
                                                                      labelCol="length_of_stay").fit(tr))
print("rf trees", len(rf._trees), "nodes", rf.totalNumNodes, "depths", [rf.trees[i].depth for i in range(3)])
pr = cProfile.Profile()
sync()
pr.enable()
timed("RandomForestRegressionModel.transform", lambda: rf.transform(te))
pr.disable()
s = io.StringIO()
pstats.Stats(pr, stream=s).sort_stats("cumulative").print_stats(25)
print(s.getvalue())
for rep in range(2):
    timed("RandomForestRegressionModel.transform", lambda: rf.transform(te))
cdata = VectorAssembler(inputCols=feats, outputCol="features").transform(df).select("features", "LOS_binary")
ctr, cte = cdata.randomSplit([0.7, 0.3], seed=42)
rfc = timed("RandomForestClassifier.fit", lambda: RandomForestClassifier(featuresCol="features",
                                                                          labelCol="LOS_binary").fit(ctr))
timed("RandomForestClassificationModel.transform", lambda: rfc.transform(cte))
dtc = timed("DecisionTreeClassifier.fit", lambda: DecisionTreeClassifier(featuresCol="features",
                                                                          labelCol="LOS_binary").fit(ctr))
timed("DecisionTreeClassificationModel.transform", lambda: dtc.transform(cte))
sys.stdout.flush()
