"""Shared fixtures: a local-mode session and the reference's hospital schema (ref.py:64-72)."""
import datetime as dt
import os

import numpy as np
import pandas as pd

PKG = "clustermachinelearningforhospitalnetworks_apache_spark_amd"


def session():
    """The shared local session, with the temp views of earlier tests dropped (a view shadows a
    table of the same name, as in Spark, so leftovers would leak between test modules)."""
    from clustermachinelearningforhospitalnetworks_apache_spark_amd.sql import SparkSession
    s = SparkSession.builder.appName("tests").master("local[2]").getOrCreate()
    for v in list(s.catalog._views):
        s.catalog.dropTempView(v)
    return s


def hospital_schema():
    from clustermachinelearningforhospitalnetworks_apache_spark_amd.sql.types import (DoubleType, IntegerType,
                                                                                        StringType, StructField,
                                                                                        StructType, TimestampType)
    return StructType([
        StructField("hospital_id", StringType(), True),
        StructField("event_time", TimestampType(), True),
        StructField("admission_count", IntegerType(), True),
        StructField("current_occupancy", IntegerType(), True),
        StructField("emergency_visits", IntegerType(), True),
        StructField("seasonality_index", DoubleType(), True),
        StructField("length_of_stay", DoubleType(), True),
    ])


def hospital_frame(n=500, seed=0, start="2025-03-31 21:30:00", minutes=120, null_frac=0.0):
    rs = np.random.RandomState(seed)
    t0 = pd.Timestamp(start)
    ts = [t0 + pd.Timedelta(seconds=int(s)) for s in rs.randint(0, minutes * 60, n)]
    adm = rs.randint(0, 60, n)
    occ = rs.randint(50, 400, n)
    er = rs.randint(0, 40, n)
    season = rs.rand(n)
    los = 1.5 + 0.04 * adm + 0.008 * occ + 0.06 * er + 2.5 * season + rs.randn(n) * 0.4
    df = pd.DataFrame({"hospital_id": [f"H{i % 7}" for i in range(n)], "event_time": ts, "admission_count": adm,
                       "current_occupancy": occ, "emergency_visits": er, "seasonality_index": season,
                       "length_of_stay": los})
    if null_frac:
        m = rs.rand(n) < null_frac
        df = df.astype({"admission_count": "object"})
        df.loc[m, "admission_count"] = None
    return df


def write_csv_files(pdf, d, nfiles=3, prefix="upload"):
    os.makedirs(d, exist_ok=True)
    paths = []
    for i, part in enumerate(np.array_split(pdf, nfiles)):
        p = os.path.join(d, f"{prefix}_{i}.csv")
        out = part.copy()
        out["event_time"] = out["event_time"].dt.strftime("%Y-%m-%d %H:%M:%S")
        out.to_csv(p, index=False)
        paths.append(p)
    return paths
