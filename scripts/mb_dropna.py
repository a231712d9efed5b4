"""Per-batch retrain pieces of the reference workflow on one GPU: a 4M-row upload
batch read through the streaming CSV path's reader, then na.drop / VectorAssembler / LinearRegression
timed cold (first call: allocator growth) and warm, each phase bracketed by device syncs."""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "examples"))
import hospital_resource_prediction as h  # noqa: E402

from clustermachinelearningforhospitalnetworks_apache_spark_amd.io.csv import read_csv_files  # noqa: E402
from clustermachinelearningforhospitalnetworks_apache_spark_amd.ml.feature import VectorAssembler  # noqa: E402
from clustermachinelearningforhospitalnetworks_apache_spark_amd.ml.regression import LinearRegression  # noqa: E402
from clustermachinelearningforhospitalnetworks_apache_spark_amd.sql import SparkSession  # noqa: E402
from clustermachinelearningforhospitalnetworks_apache_spark_amd.sql import functions as F  # noqa: E402
from clustermachinelearningforhospitalnetworks_apache_spark_amd.sql import types as T  # noqa: E402

ROWS = int(os.environ.get("MB_ROWS", 1_000_000))
d = "/tmp/mb_dropna/in"
if not os.path.isdir(d):
    h.synth_uploads(d, n_files=4, rows=ROWS)
files = sorted(os.path.join(d, f) for f in os.listdir(d))
spark = SparkSession.builder.master("mi355x" if torch.cuda.is_available() else "local[4]").getOrCreate()
schema = T.StructType([T.StructField("hospital_id", T.StringType()), T.StructField("event_time", T.TimestampType()),
                       T.StructField("admission_count", T.IntegerType()),
                       T.StructField("current_occupancy", T.IntegerType()),
                       T.StructField("emergency_visits", T.IntegerType()),
                       T.StructField("seasonality_index", T.DoubleType()),
                       T.StructField("length_of_stay", T.DoubleType())])
feats = ["admission_count", "current_occupancy", "emergency_visits", "seasonality_index"]


def sync():
    if torch.cuda.is_available():
        torch.cuda.synchronize()


def timed(name, fn):
    sync()
    t = time.perf_counter()
    out = fn()
    sync()
    print(f"{name:28s} {1000 * (time.perf_counter() - t):9.2f} ms", flush=True)
    return out


for rep in range(3):
    print(f"--- rep {rep}")
    df = timed("read_csv_files (4 files)", lambda: read_csv_files(spark, files, schema, True))
    df = df.withColumn("ingest_time", F.current_timestamp())
    clean = timed("na.drop", lambda: df.na.drop())
    data = timed("VectorAssembler", lambda: VectorAssembler(inputCols=feats, outputCol="features").transform(clean))
    timed("count", lambda: data.count())
    m = timed("LinearRegression.fit", lambda: LinearRegression(featuresCol="features",
                                                               labelCol="length_of_stay").fit(data))
    timed("summary.rmse", lambda: m.summary.rootMeanSquaredError)
    w = timed("sql BETWEEN window", lambda: df.filter(
        "event_time BETWEEN '2025-03-31 22:00:00' AND '2025-03-31 23:00:00'"))
    print("rows", df.count(), "clean", clean.count(), "window", w.count(), flush=True)

if os.environ.get("CML_TRACE") == "1":
    from clustermachinelearningforhospitalnetworks_apache_spark_amd.utils.trace import TRACER
    print(TRACER.report(), flush=True)
