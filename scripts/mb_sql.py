"""DataFrame / SQL-layer microbenchmarks: one driver, one subcommand per experiment.

    python scripts/mb_sql.py frame [--rows 100000000] [--reps 10]
        bandwidth of the frame kernels (K2 assemble, K3 compact, K5 split / counter uniform, K22 Poisson, K6 binarize,
        K23 metric sums / confusion, K7 moments, K8 scale, K4 absmax / fp8 quantise) against the torch expression of
        the same op; bytes are the compulsory HBM traffic, the ceiling ~8 TB/s (GPU only)
    python scripts/mb_sql.py groupby [--rows 10000000] [--master mi355x]
        groupBy().agg() wall time: the columnar merge (sql/aggregate_fast.py) against the Python-tuple merge of the
        same partials, at hospital and patient cardinality
    python scripts/mb_sql.py groupby-once [N]
        one low-cardinality groupBy().agg() after a warm-up, for a kernel trace
    python scripts/mb_sql.py relational [--rows 10000000] [--host-rows 200000] [--master mi355x]
        orderBy / dropDuplicates / join on the device path (sql/relational_fast.py) against the row loop
    python scripts/mb_sql.py window [--rows 10000000] [--host-rows 1000000] [--master mi355x]
        row_number, lag and a running sum per hospital: device (sql/window_fast.py) vs host (sql/window.py)
    python scripts/mb_sql.py dropna [--rows 1000000] [--reps 3]
        the reference workflow's per-batch pieces on 4 upload files: CSV read, na.drop, VectorAssembler, count,
        LinearRegression fit, summary, a BETWEEN window; each phase between device syncs (CML_TRACE=1: stage table)

Every subcommand runs on the CPU as well (``--master local[4]``) except ``frame``.
"""
import argparse
import json
import os
import sys
import time

import numpy as np
import pandas as pd
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from clustermachinelearningforhospitalnetworks_apache_spark_amd.sql import SparkSession, Window  # noqa: E402
from clustermachinelearningforhospitalnetworks_apache_spark_amd.sql import functions as F  # noqa: E402


def sync():
    if torch.cuda.is_available():
        torch.cuda.synchronize()


def wall_s(fn):
    sync()
    t = time.perf_counter()
    out = fn()
    sync()
    return time.perf_counter() - t, out


def default_master():
    return "mi355x" if torch.cuda.is_available() else "local[4]"


def session(master):
    return SparkSession.builder.master(master).getOrCreate()


def cmd_frame(argv):
    from clustermachinelearningforhospitalnetworks_apache_spark_amd.ops import frame_ops, glm_ops
    ap = argparse.ArgumentParser(prog="mb_sql.py frame")
    ap.add_argument("--rows", type=int, default=100_000_000)
    ap.add_argument("--reps", type=int, default=10)
    a = ap.parse_args(argv)
    n, reps, dev = a.rows, a.reps, torch.device("cuda")
    g = torch.Generator(device=dev).manual_seed(0)
    out = []

    def timed(fn):
        fn()
        torch.cuda.synchronize()
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        for _ in range(reps):
            fn()
        e.record()
        torch.cuda.synchronize()
        return s.elapsed_time(e) / reps

    def rec(name, fn, nbytes, ref=None):
        ms = timed(fn)
        r = {"kernel": name, "ms": round(ms, 4), "GB": round(nbytes / 1e9, 3), "TB_s": round(nbytes / ms / 1e9, 3)}
        if ref is not None:
            tms = timed(ref)
            r.update(torch_ms=round(tms, 4), speedup_vs_torch=round(tms / ms, 2))
        out.append(r)
        print(json.dumps(r), flush=True)

    # K2 assemble: the reference's 4 feature columns (3 int32 + 1 float64) -> [n, 4] float64
    c1 = torch.randint(0, 100, (n,), device=dev, dtype=torch.int32, generator=g)
    c2 = torch.randint(0, 500, (n,), device=dev, dtype=torch.int32, generator=g)
    c3 = torch.randint(0, 50, (n,), device=dev, dtype=torch.int32, generator=g)
    c4 = torch.rand(n, device=dev, dtype=torch.float64, generator=g)
    parts = [(c1, None), (c2, None), (c3, None), (c4, None)]
    rec("K2 assemble 3xi32+f64 -> [n,4] f64", lambda: frame_ops.assemble(parts), n * (12 + 8 + 32 + 1),
        lambda: torch.stack([c1.double(), c2.double(), c3.double(), c4], 1))
    del c1, c2, c3
    mask = torch.rand(n, device=dev, generator=g) < 0.5
    rec("K3 compact 50% of n", lambda: frame_ops.compact(mask), n + 8 * int(mask.sum()),
        lambda: torch.nonzero(mask).flatten())
    del mask
    rows = torch.arange(n, device=dev, dtype=torch.int64)
    rec("K5 counter_uniform", lambda: frame_ops.counter_uniform(rows, 12345), n * 16)
    rec("K5 split_buckets 70/30", lambda: frame_ops.split_buckets(rows, 12345, [0.0, 0.7, 1.0]), n * 9)
    cdf = [0.36787944117144233, 0.7357588823428847, 0.9196986029286058, 0.9810118431238462]  # Poisson(1)
    rec("K22 poisson1 -> int32", lambda: frame_ops.poisson1(rows, 12345, cdf, torch.int32), n * 12)
    del rows
    rec("K6 binarize f64", lambda: frame_ops.binarize(c4, 0.5), n * 16, lambda: (c4 > 0.5).to(torch.float64))
    p = torch.rand(n, device=dev, dtype=torch.float64, generator=g)
    rec("K23 reg_metric_sums", lambda: frame_ops.reg_metric_sums(c4, p), n * 16,
        lambda: torch.stack([((c4 - p) ** 2).sum(), (c4 - p).abs().sum(), c4.sum(), (c4 * c4).sum(), p.sum(),
                             (p * p).sum()]))
    yl, pl = (c4 > 0.5).to(torch.int64), (p > 0.5).to(torch.int64)
    rec("K23 confusion 2x2 (int64 labels)", lambda: frame_ops.confusion(yl, pl, 2), n * 16)
    del p, yl, pl, c4
    m = n // 4  # K7 moments, K8 scale, K4 absmax / fp8 quantise on [m, 256] bf16
    X = torch.randn((m, 256), device=dev, dtype=torch.bfloat16, generator=g)
    rec(f"K7 moments [{m},256] bf16", lambda: glm_ops.moments(X, 256), m * 512,
        lambda: (X.float().mean(0), X.float().var(0)))
    mean = torch.zeros(256, device=dev, dtype=torch.float64)
    inv = torch.ones(256, device=dev, dtype=torch.float64)
    rec(f"K8 scale_apply [{m},256] bf16 -> bf16",
        lambda: glm_ops.scale_apply(X, 256, mean, inv, True, out_dtype=torch.bfloat16), m * 1024)
    rec(f"K4 col_absmax [{m},256] bf16", lambda: frame_ops.col_absmax(X, 256), m * 512, lambda: X.abs().amax(0))
    sc = torch.ones(256, device=dev, dtype=torch.float32)
    rec(f"K4 quant_fp8 [{m},256] bf16 -> e4m3", lambda: frame_ops.quant_fp8(X, 256, sc), m * 768,
        lambda: (X.float() * sc).to(torch.float8_e4m3fn))
    print(json.dumps({"rows": n, "results": out}))


def cmd_groupby(argv):
    from clustermachinelearningforhospitalnetworks_apache_spark_amd.sql import aggregate_fast as AF
    ap = argparse.ArgumentParser(prog="mb_sql.py groupby")
    ap.add_argument("--rows", type=int, default=10_000_000)
    ap.add_argument("--master", default=default_master())
    a = ap.parse_args(argv)
    spark, n = session(a.master), a.rows
    rs = np.random.RandomState(0)
    df = spark.createDataFrame(pd.DataFrame({
        "hospital_id": rs.randint(0, 500, n).astype(np.int32), "patient_id": rs.randint(0, max(1, n // 10), n),
        "los": rs.gamma(2.0, 3.0, n), "age": rs.randint(0, 100, n).astype(np.int32)}))
    out = []
    for key in ("hospital_id", "patient_id"):
        def q():
            return df.groupBy(key).agg(F.count("*"), F.avg("los"), F.max("age"), F.stddev("los")).count()
        for path in ("columnar", "python-merge"):
            AF.ENABLED = path == "columnar"
            q()
            s, _ = wall_s(q)
            r = {"key": key, "rows": n, "path": path, "s": round(s, 4), "Mrows_s": round(n / s / 1e6, 2)}
            out.append(r)
            print(json.dumps(r), flush=True)
        AF.ENABLED = True
    print(json.dumps({"device": str(spark._device), "results": out}))


def cmd_groupby_once(argv):
    n = int(argv[0]) if argv else 10_000_000
    spark = session(default_master())
    rs = np.random.RandomState(0)
    df = spark.createDataFrame(pd.DataFrame({"hospital_id": rs.randint(0, 500, n).astype(np.int32),
                                             "los": rs.gamma(2.0, 3.0, n),
                                             "age": rs.randint(0, 100, n).astype(np.int32)}))
    for _ in range(2):
        df.groupBy("hospital_id").agg(F.count("*"), F.avg("los"), F.max("age"), F.stddev("los")).count()
    sync()


def cmd_relational(argv):
    from clustermachinelearningforhospitalnetworks_apache_spark_amd.sql import relational_fast as RF
    ap = argparse.ArgumentParser(prog="mb_sql.py relational")
    ap.add_argument("--rows", type=int, default=10_000_000)
    ap.add_argument("--host-rows", type=int, default=200_000)
    ap.add_argument("--master", default=default_master())
    a = ap.parse_args(argv)
    spark = session(a.master)
    dim = spark.createDataFrame(pd.DataFrame({"hospital_id": np.arange(0, 500, dtype=np.int32),
                                              "region": [f"r{i % 17}" for i in range(500)]}))
    ops = {
        "orderBy(ward desc, los)": lambda d: d.orderBy(F.col("ward").desc(), "los").count(),
        "orderBy(hospital_id, age desc, rid)": lambda d: d.orderBy("hospital_id", F.col("age").desc(), "rid").count(),
        "dropDuplicates(hospital_id, ward, age)": lambda d: d.dropDuplicates(["hospital_id", "ward", "age"]).count(),
        "join(dim, hospital_id) inner": lambda d: d.join(dim, "hospital_id").count(),
        "join(dim, hospital_id) leftanti": lambda d: d.join(dim, "hospital_id", "leftanti").count(),
    }
    out = []
    for n, paths in ((a.rows, ("device",)), (a.host_rows, ("device", "row-loop"))):
        rs = np.random.RandomState(0)
        df = spark.createDataFrame(pd.DataFrame({
            "hospital_id": rs.randint(0, 500, n).astype(np.int32),
            "ward": np.array(["icu", "er", "gen", "ped", "onc"], dtype=object)[rs.randint(0, 5, n)],
            "los": rs.gamma(2.0, 3.0, n), "age": rs.randint(0, 100, n).astype(np.int32),
            "rid": np.arange(n, dtype=np.int64)}))
        for name, fn in ops.items():
            for p in paths:
                RF.ENABLED = p == "device"
                fn(df)  # warm
                s, _ = wall_s(lambda: fn(df))
                r = {"op": name, "rows": n, "path": p, "s": round(s, 4), "Mrows_s": round(n / s / 1e6, 2)}
                out.append(r)
                print(json.dumps(r), flush=True)
        RF.ENABLED = True
    print(json.dumps({"device": str(spark._device), "results": out}))


def cmd_window(argv):
    from clustermachinelearningforhospitalnetworks_apache_spark_amd.sql import window as W
    ap = argparse.ArgumentParser(prog="mb_sql.py window")
    ap.add_argument("--rows", type=int, default=10_000_000)
    ap.add_argument("--host-rows", type=int, default=1_000_000)
    ap.add_argument("--master", default=default_master())
    a = ap.parse_args(argv)
    spark = session(a.master)

    def run(n, device):
        rs = np.random.RandomState(0)
        df = spark.createDataFrame(pd.DataFrame({"h": rs.randint(0, 50, n), "t": rs.randint(0, 10 ** 9, n),
                                                 "los": rs.rand(n) * 10}))
        spec = Window.partitionBy("h").orderBy("t")
        W.DEVICE_WINDOWS = device

        def q():
            return df.select(F.row_number().over(spec).alias("rn"), F.lag("los", 1).over(spec).alias("prev"),
                             F.sum("los").over(spec).alias("run")).count()
        q()
        return wall_s(q)[0]

    dev_s = run(a.rows, True)
    host_s = run(a.host_rows, False)
    dev_small = run(a.host_rows, True)
    W.DEVICE_WINDOWS = True
    print(json.dumps({"device_rows": a.rows, "device_s": round(dev_s, 4), "device_rows_per_s": a.rows / dev_s,
                      "host_rows": a.host_rows, "host_s": round(host_s, 3), "device_s_same_rows": round(dev_small, 4),
                      "speedup_same_rows": round(host_s / dev_small, 1)}))


def cmd_dropna(argv):
    sys.path.insert(0, os.path.join(ROOT, "examples"))
    import hospital_resource_prediction as h

    from clustermachinelearningforhospitalnetworks_apache_spark_amd.io.csv import read_csv_files
    from clustermachinelearningforhospitalnetworks_apache_spark_amd.ml.feature import VectorAssembler
    from clustermachinelearningforhospitalnetworks_apache_spark_amd.ml.regression import LinearRegression
    from clustermachinelearningforhospitalnetworks_apache_spark_amd.sql import types as T
    ap = argparse.ArgumentParser(prog="mb_sql.py dropna")
    ap.add_argument("--rows", type=int, default=int(os.environ.get("MB_ROWS", 1_000_000)), help="rows per file")
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--dir", default="/tmp/mb_dropna/in")
    a = ap.parse_args(argv)
    if not os.path.isdir(a.dir):
        h.synth_uploads(a.dir, n_files=4, rows=a.rows)
    files = sorted(os.path.join(a.dir, f) for f in os.listdir(a.dir))
    spark = session(default_master())
    schema = T.StructType([T.StructField("hospital_id", T.StringType()),
                           T.StructField("event_time", T.TimestampType()),
                           T.StructField("admission_count", T.IntegerType()),
                           T.StructField("current_occupancy", T.IntegerType()),
                           T.StructField("emergency_visits", T.IntegerType()),
                           T.StructField("seasonality_index", T.DoubleType()),
                           T.StructField("length_of_stay", T.DoubleType())])
    feats = ["admission_count", "current_occupancy", "emergency_visits", "seasonality_index"]

    def timed(name, fn):
        s, out = wall_s(fn)
        print(f"{name:28s} {1000 * s:9.2f} ms", flush=True)
        return out

    for rep in range(a.reps):
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


COMMANDS = {"frame": cmd_frame, "groupby": cmd_groupby, "groupby-once": cmd_groupby_once,
            "relational": cmd_relational, "window": cmd_window, "dropna": cmd_dropna}

if __name__ == "__main__":
    if len(sys.argv) < 2 or sys.argv[1] not in COMMANDS:
        print(__doc__)
        sys.exit(2)
    COMMANDS[sys.argv[1]](sys.argv[2:])
