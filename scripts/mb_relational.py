"""Wall time of the relational operators (orderBy, dropDuplicates, join) on the device path
(sql/relational_fast.py) against the row-loop path, on a synthetic hospital-records frame.

    python scripts/mb_relational.py [--rows 10000000] [--host-rows 200000] [--master mi355x]
"""
import argparse
import json
import sys
import time

import numpy as np
import pandas as pd
import torch

sys.path.insert(0, ".")
from clustermachinelearningforhospitalnetworks_apache_spark_amd.sql import SparkSession  # noqa: E402
from clustermachinelearningforhospitalnetworks_apache_spark_amd.sql import functions as F  # noqa: E402
from clustermachinelearningforhospitalnetworks_apache_spark_amd.sql import relational_fast as RF  # noqa: E402


def frame(spark, n):
    rs = np.random.RandomState(0)
    pdf = pd.DataFrame({"hospital_id": rs.randint(0, 500, n).astype(np.int32),
                        "ward": np.array(["icu", "er", "gen", "ped", "onc"], dtype=object)[rs.randint(0, 5, n)],
                        "los": rs.gamma(2.0, 3.0, n), "age": rs.randint(0, 100, n).astype(np.int32),
                        "rid": np.arange(n, dtype=np.int64)})
    return spark.createDataFrame(pdf)


def timed(fn):
    if torch.cuda.is_available():
        torch.cuda.synchronize()
    t = time.perf_counter()
    fn()
    if torch.cuda.is_available():
        torch.cuda.synchronize()
    return time.perf_counter() - t


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=10_000_000)
    ap.add_argument("--host-rows", type=int, default=200_000)
    ap.add_argument("--master", default="mi355x")
    a = ap.parse_args()
    spark = SparkSession.builder.master(a.master).getOrCreate()
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
        df = frame(spark, n)
        for name, fn in ops.items():
            for p in paths:
                RF.ENABLED = p == "device"
                fn(df)  # warm
                s = timed(lambda: fn(df))
                r = {"op": name, "rows": n, "path": p, "s": round(s, 4), "Mrows_s": round(n / s / 1e6, 2)}
                out.append(r)
                print(json.dumps(r), flush=True)
        RF.ENABLED = True
    print(json.dumps({"device": str(spark._device), "results": out}))


if __name__ == "__main__":
    main()
