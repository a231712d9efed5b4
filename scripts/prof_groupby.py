"""One low-cardinality groupBy().agg() for kernel profiling (rocprofv3 --kernel-trace --stats)."""
import sys

import numpy as np
import pandas as pd
import torch

sys.path.insert(0, ".")
from clustermachinelearningforhospitalnetworks_apache_spark_amd.sql import SparkSession  # noqa: E402
from clustermachinelearningforhospitalnetworks_apache_spark_amd.sql import functions as F  # noqa: E402

spark = SparkSession.builder.master("mi355x").getOrCreate()
n = int(sys.argv[1]) if len(sys.argv) > 1 else 10_000_000
rs = np.random.RandomState(0)
pdf = pd.DataFrame({"hospital_id": rs.randint(0, 500, n).astype(np.int32), "los": rs.gamma(2.0, 3.0, n),
                    "age": rs.randint(0, 100, n).astype(np.int32)})
df = spark.createDataFrame(pdf)
for _ in range(2):
    df.groupBy("hospital_id").agg(F.count("*"), F.avg("los"), F.max("age"), F.stddev("los")).count()
torch.cuda.synchronize()
