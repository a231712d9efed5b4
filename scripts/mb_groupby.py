"""groupBy().agg() wall time on one device: the columnar merge (sql/aggregate_fast.py) against the
Python-tuple merge of the same device partials, at low (hospital) and high (patient) cardinality.

    python scripts/mb_groupby.py [--rows 10000000] [--master mi355x]
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
from clustermachinelearningforhospitalnetworks_apache_spark_amd.sql import aggregate_fast as AF  # noqa: E402
from clustermachinelearningforhospitalnetworks_apache_spark_amd.sql import functions as F  # noqa: E402


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
    ap.add_argument("--master", default="mi355x")
    a = ap.parse_args()
    spark = SparkSession.builder.master(a.master).getOrCreate()
    n = a.rows
    rs = np.random.RandomState(0)
    pdf = pd.DataFrame({"hospital_id": rs.randint(0, 500, n).astype(np.int32),
                        "patient_id": rs.randint(0, n // 10, n).astype(np.int64),
                        "los": rs.gamma(2.0, 3.0, n), "age": rs.randint(0, 100, n).astype(np.int32)})
    df = spark.createDataFrame(pdf)
    out = []
    for key in ("hospital_id", "patient_id"):
        q = lambda: df.groupBy(key).agg(F.count("*"), F.avg("los"), F.max("age"), F.stddev("los")).count()  # noqa
        for path in ("columnar", "python-merge"):
            AF.ENABLED = path == "columnar"
            q()
            s = timed(q)
            r = {"key": key, "rows": n, "path": path, "s": round(s, 4), "Mrows_s": round(n / s / 1e6, 2)}
            out.append(r)
            print(json.dumps(r), flush=True)
        AF.ENABLED = True
    print(json.dumps({"device": str(spark._device), "results": out}))


if __name__ == "__main__":
    main()
