"""JSON round trip of non-finite doubles: Spark writes NaN / Infinity / -Infinity as quoted strings and
reads them back (allowNonNumericNumbers); a null stays a missing field."""
import math

import pandas as pd

from clustermachinelearningforhospitalnetworks_apache_spark_amd.sql import SparkSession
from clustermachinelearningforhospitalnetworks_apache_spark_amd.sql import types as T


def test_json_nan_inf_round_trip(tmp_path):
    spark = SparkSession.builder.master("local[1]").getOrCreate()
    schema = T.StructType([T.StructField("id", T.IntegerType()), T.StructField("v", T.DoubleType())])
    rows = [(1, 1.5), (2, float("nan")), (3, float("inf")), (4, float("-inf")), (5, None)]
    df = spark.createDataFrame(rows, schema)
    path = str(tmp_path / "j")
    df.write.mode("overwrite").json(path)
    text = "".join(open(f).read() for f in sorted((tmp_path / "j").glob("*.json")))
    assert '"v":"NaN"' in text and '"v":"Infinity"' in text and '"v":"-Infinity"' in text
    for back in (spark.read.schema(schema).json(path), spark.read.json(path)):
        got = {r["id"]: r["v"] for r in back.collect()}
        assert got[1] == 1.5 and math.isnan(got[2]) and got[3] == math.inf and got[4] == -math.inf
        assert got[5] is None
