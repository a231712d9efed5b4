"""Window functions on the device vs the host path (sql/window_fast.py vs sql/window.py):
row_number, lag and a running sum per hospital ordered by event time.

    python scripts/mb_window.py [--rows 10000000] [--host-rows 1000000]
"""
import argparse
import json
import sys
import time

import numpy as np
import torch

sys.path.insert(0, ".")
from clustermachinelearningforhospitalnetworks_apache_spark_amd.sql import SparkSession, Window  # noqa: E402
from clustermachinelearningforhospitalnetworks_apache_spark_amd.sql import functions as F  # noqa: E402
from clustermachinelearningforhospitalnetworks_apache_spark_amd.sql import window as W  # noqa: E402


def run(spark, n, device):
    rs = np.random.RandomState(0)
    import pandas as pd
    pdf = pd.DataFrame({"h": rs.randint(0, 50, n), "t": rs.randint(0, 10 ** 9, n).astype(np.int64),
                        "los": rs.rand(n) * 10})
    df = spark.createDataFrame(pdf)
    spec = Window.partitionBy("h").orderBy("t")
    W.DEVICE_WINDOWS = device
    out = df.select(F.row_number().over(spec).alias("rn"), F.lag("los", 1).over(spec).alias("prev"),
                    F.sum("los").over(spec).alias("run"))
    out.count()
    if torch.cuda.is_available():
        torch.cuda.synchronize()
    t0 = time.time()
    out = df.select(F.row_number().over(spec).alias("rn"), F.lag("los", 1).over(spec).alias("prev"),
                    F.sum("los").over(spec).alias("run"))
    out.count()
    if torch.cuda.is_available():
        torch.cuda.synchronize()
    return time.time() - t0


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=10_000_000)
    ap.add_argument("--host-rows", type=int, default=1_000_000)
    a = ap.parse_args()
    spark = SparkSession.builder.appName("mbw").master("mi355x" if torch.cuda.is_available() else "local[1]") \
        .getOrCreate()
    dev_s = run(spark, a.rows, True)
    host_s = run(spark, a.host_rows, False)
    dev_small = run(spark, a.host_rows, True)
    print(json.dumps({"device_rows": a.rows, "device_s": round(dev_s, 4), "device_rows_per_s": a.rows / dev_s,
                      "host_rows": a.host_rows, "host_s": round(host_s, 3), "device_s_same_rows": round(dev_small, 4),
                      "speedup_same_rows": round(host_s / dev_small, 1)}))
    spark.stop()


if __name__ == "__main__":
    main()
