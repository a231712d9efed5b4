"""na.drop skips the per-row work of columns that cannot hold a null (round 4): dictionary strings
without a -1 code, integer device columns; a -1 code or a NaN still drops the row."""
import numpy as np
import torch

from clustermachinelearningforhospitalnetworks_apache_spark_amd.sql import types as T
from clustermachinelearningforhospitalnetworks_apache_spark_amd.sql.column import ColumnData, DictColumnData
from clustermachinelearningforhospitalnetworks_apache_spark_amd.sql.dataframe import _never_null, _non_null_mask


def test_never_null_rules():
    d = np.array(["a", "b", None], dtype=object)
    full = DictColumnData(np.array([0, 1, 0, 1]), d, None, T.StringType())
    holes = DictColumnData(np.array([0, -1, 1, 0]), d, None, T.StringType())
    assert _never_null(full) and not _never_null(holes)
    assert list(_non_null_mask(holes).numpy()) == [True, False, True, True]
    masked = DictColumnData(np.array([0, 1]), d, np.array([True, False]), T.StringType())
    assert not _never_null(masked)
    ints = ColumnData(torch.arange(4), None, T.IntegerType())
    floats = ColumnData(torch.tensor([1.0, float("nan")]), None, T.DoubleType())
    host = ColumnData(np.array([1, 2]), None, T.IntegerType())
    assert _never_null(ints) and not _never_null(floats) and not _never_null(host)


def test_dropna_drops_null_codes():
    from clustermachinelearningforhospitalnetworks_apache_spark_amd.sql import SparkSession
    import pandas as pd
    spark = SparkSession.builder.master("local[1]").getOrCreate()
    df = spark.createDataFrame(pd.DataFrame({"s": ["x", None, "y", "x"], "v": [1.0, 2.0, float("nan"), 4.0]}))
    out = df.na.drop().toPandas()
    assert out["s"].tolist() == ["x", "x"] and out["v"].tolist() == [1.0, 4.0]
