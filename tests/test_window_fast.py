"""Device window functions (sql/window_fast.py) against the host implementation of sql/window.py:
ranking, ntile, lag/lead (numeric and string), count/sum/avg/first/last over default, ROWS and
RANGE frames, whole-partition min/max; nulls, NaN, descending orders and nulls-last placement."""
import math

import numpy as np
import pandas as pd
import pytest

from clustermachinelearningforhospitalnetworks_apache_spark_amd.sql import SparkSession, Window
from clustermachinelearningforhospitalnetworks_apache_spark_amd.sql import functions as F
from clustermachinelearningforhospitalnetworks_apache_spark_amd.sql import window as W


def _frame(spark, n=700, seed=0):
    rs = np.random.RandomState(seed)
    g = rs.randint(0, 6, n)
    t = rs.randint(0, 40, n).astype(float)
    # (no NaN in the ordering key here: the host path orders NaN inconsistently, see the NaN test)
    v = rs.randint(-50, 50, n)
    x = rs.normal(size=n)
    rows = []
    for i in range(n):
        rows.append((int(g[i]) if rs.rand() > 0.03 else None, float(t[i]), int(v[i]) if rs.rand() > 0.05 else None,
                     float(x[i]), ["icu", "er", "gen"][i % 3]))
    return spark.createDataFrame(rows, "g int, t double, v int, x double, w string")


def _cols(spec):
    return [F.row_number().over(spec), F.rank().over(spec), F.dense_rank().over(spec), F.percent_rank().over(spec),
            F.cume_dist().over(spec), F.ntile(4).over(spec), F.lag("v", 1).over(spec), F.lead("x", 2, -1.0).over(spec),
            F.lag("w", 1).over(spec), F.count("v").over(spec), F.sum("v").over(spec), F.avg("x").over(spec),
            F.first("v").over(spec), F.last("w").over(spec)]


SPECS = [
    lambda: Window.partitionBy("g").orderBy("t"),
    lambda: Window.partitionBy("g").orderBy(F.col("t").desc(), "v"),
    lambda: Window.partitionBy("g", "w").orderBy(F.col("v").asc_nulls_last()),
    lambda: Window.partitionBy("g").orderBy("t").rowsBetween(-2, 1),
    lambda: Window.partitionBy("g").orderBy("t").rowsBetween(Window.unboundedPreceding, Window.currentRow),
    lambda: Window.partitionBy("g").orderBy("t").rangeBetween(Window.currentRow, Window.unboundedFollowing),
    lambda: Window.orderBy("x"),
]


def _same(a, b):
    assert len(a) == len(b)
    for ra, rb in zip(a, b):
        for u, v in zip(ra, rb):
            if isinstance(u, float) or isinstance(v, float):
                if u is None or v is None:
                    assert u is None and v is None
                elif math.isnan(u) or math.isnan(v):
                    assert math.isnan(u) and math.isnan(v)
                else:
                    assert u == pytest.approx(v, rel=1e-10, abs=1e-12)
            else:
                assert u == v, (ra, rb)


@pytest.fixture(scope="module")
def spark():
    s = SparkSession.builder.appName("wfast").master("local[1]").getOrCreate()
    yield s
    s.stop()


@pytest.mark.parametrize("si", range(len(SPECS)))
def test_device_window_equals_host(spark, si):
    df = _frame(spark)
    spec = SPECS[si]()
    cols = _cols(spec)
    W.DEVICE_WINDOWS = True
    fast = [tuple(r) for r in df.select(*cols).collect()]
    W.DEVICE_WINDOWS = False
    try:
        slow = [tuple(r) for r in df.select(*cols).collect()]
    finally:
        W.DEVICE_WINDOWS = True
    _same(fast, slow)


def test_device_window_min_max_whole_partition(spark):
    df = _frame(spark)
    spec = Window.partitionBy("g")
    cols = [F.min("v").over(spec), F.max("x").over(spec), F.count("*").over(spec), F.sum("x").over(spec)]
    W.DEVICE_WINDOWS = True
    fast = [tuple(r) for r in df.select(*cols).collect()]
    W.DEVICE_WINDOWS = False
    try:
        slow = [tuple(r) for r in df.select(*cols).collect()]
    finally:
        W.DEVICE_WINDOWS = True
    _same(fast, slow)


def test_device_window_nan_orders_last_as_peers(spark):
    df = spark.createDataFrame([(1, 2.0), (1, float("nan")), (1, 1.0), (1, float("nan"))], "g int, t double")
    out = df.select("t", F.rank().over(Window.partitionBy("g").orderBy("t")).alias("r")).collect()
    got = sorted((r.r, "nan" if math.isnan(r.t) else r.t) for r in out)
    assert got == [(1, 1.0), (2, 2.0), (3, "nan"), (3, "nan")]


@pytest.mark.gpu
def test_device_window_gpu_equals_host():
    s = SparkSession.builder.appName("wfast_gpu").master("mi355x").getOrCreate()
    try:
        df = _frame(s, n=5000, seed=2)
        assert df._device.type == "cuda"
        for mk in SPECS:
            cols = _cols(mk())
            W.DEVICE_WINDOWS = True
            fast = [tuple(r) for r in df.select(*cols).collect()]
            W.DEVICE_WINDOWS = False
            try:
                slow = [tuple(r) for r in df.select(*cols).collect()]
            finally:
                W.DEVICE_WINDOWS = True
            _same(fast, slow)
    finally:
        s.stop()
