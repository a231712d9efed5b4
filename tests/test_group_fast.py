"""Device group-by (sql/group_fast.py) against the row-loop path of sql/group.py: same groups,
same first-appearance order, same values — with nulls, NaN, -0.0, dictionary-encoded and plain
string keys, tumbling and sliding windows, first/last, the custom Summarizer aggregate and
global aggregates. Also checks the native CSV dictionary encoder end to end."""
import datetime as dt
import math

import numpy as np
import pandas as pd
import pytest

from clustermachinelearningforhospitalnetworks_apache_spark_amd.sql import SparkSession
from clustermachinelearningforhospitalnetworks_apache_spark_amd.sql import functions as F
from clustermachinelearningforhospitalnetworks_apache_spark_amd.sql import group_fast


def _frame(spark, n=3000, seed=0):
    rs = np.random.RandomState(seed)
    ward = np.array(["icu", "er", "gen", None], dtype=object)[rs.randint(0, 4, n)]
    x = rs.normal(size=n)
    x[rs.rand(n) < 0.05] = np.nan
    x[rs.rand(n) < 0.05] = -0.0
    k = rs.randint(0, 7, n).astype(float)
    k[rs.rand(n) < 0.03] = np.nan
    k[k == 3] = -0.0
    los = rs.randint(0, 30, n)
    t0 = dt.datetime(2024, 1, 1)
    ts = [t0 + dt.timedelta(seconds=int(s)) for s in rs.randint(0, 7200, n)]
    pdf = pd.DataFrame({"ward": ward, "x": x, "k": k, "los": los, "ts": ts,
                        "h": rs.randint(0, 5, n).astype(np.int64)})
    df = spark.createDataFrame(pdf)
    # some nulls in a numeric column
    return df.withColumn("xn", F.when(F.col("los") % 7 == 0, None).otherwise(F.col("x")))


def _rows(df):
    out = []
    for r in df.collect():
        out.append(tuple(r))
    return out


def _same(a, b):
    assert len(a) == len(b)
    for ra, rb in zip(a, b):
        assert len(ra) == len(rb)
        for u, v in zip(ra, rb):
            if isinstance(u, float) and isinstance(v, float):
                if math.isnan(u) or math.isnan(v):
                    assert math.isnan(u) and math.isnan(v)
                else:
                    assert u == pytest.approx(v, rel=1e-12, abs=1e-12)
            elif hasattr(u, "toArray"):
                np.testing.assert_allclose(u.toArray(), v.toArray(), rtol=1e-12, atol=1e-12)
            else:
                assert u == v, (ra, rb)


QUERIES = [
    lambda df: df.groupBy("ward").agg(F.count("*"), F.count("xn"), F.sum("los"), F.avg("x"), F.max("los"),
                                      F.min("x"), F.stddev("xn"), F.variance("x"), F.var_pop("los"),
                                      F.stddev_pop("x")),
    lambda df: df.groupBy("k").agg(F.count("*").alias("c"), F.sum("x"), F.first("xn"), F.last("xn"),
                                   F.first("ward"), F.count("ward")),
    lambda df: df.groupBy("ward", "h").agg(F.sum("x"), F.avg("los"), F.min("ts"), F.max("ts")),
    lambda df: df.groupBy(F.window("ts", "10 minutes")).agg(F.count("*"), F.avg("x")),
    lambda df: df.groupBy(F.window("ts", "10 minutes", "4 minutes"), "ward").agg(F.count("*"), F.sum("los")),
    lambda df: df.agg(F.count("*"), F.sum("los"), F.avg("xn"), F.max("x"), F.min("k")),
    lambda df: df.groupBy((F.col("los") % 4).alias("b")).agg(F.count("*"), F.sum("xn")),
    lambda df: df.groupBy("ward").count(),
]


@pytest.fixture(scope="module")
def spark():
    s = SparkSession.builder.appName("gfast").master("local[1]").getOrCreate()
    yield s
    s.stop()


@pytest.mark.parametrize("qi", range(len(QUERIES)))
def test_fast_equals_row_loop(spark, qi):
    df = _frame(spark)
    q = QUERIES[qi]
    group_fast.ENABLED = True
    fast = _rows(q(df))
    group_fast.ENABLED = False
    try:
        slow = _rows(q(df))
    finally:
        group_fast.ENABLED = True
    if qi == 1:
        # the row loop keys NaN by object identity (one group per NaN row); Spark and the device
        # path put all NaN keys in one group — compare the non-NaN groups
        fast = [r for r in fast if not (isinstance(r[0], float) and math.isnan(r[0]))]
        slow = [r for r in slow if not (isinstance(r[0], float) and math.isnan(r[0]))]
    _same(fast, slow)


def test_fast_nan_keys_one_group(spark):
    df = _frame(spark)
    rows = df.groupBy("k").count().collect()
    nan_rows = [r for r in rows if isinstance(r[0], float) and math.isnan(r[0])]
    assert len(nan_rows) == 1
    assert sum(r[1] for r in rows) == 3000
    zero = [r for r in rows if r[0] == 0.0]
    assert len(zero) == 1  # 0.0 and -0.0 group together


def test_fast_summarizer(spark):
    from clustermachinelearningforhospitalnetworks_apache_spark_amd.ml.feature import VectorAssembler
    from clustermachinelearningforhospitalnetworks_apache_spark_amd.ml.stat import Summarizer
    df = VectorAssembler(inputCols=["los", "h"], outputCol="f").transform(_frame(spark))
    q = lambda d: d.groupBy("ward").agg(Summarizer.mean(F.col("f")).alias("m"), F.count("*"))
    group_fast.ENABLED = True
    fast = _rows(q(df))
    group_fast.ENABLED = False
    try:
        slow = _rows(q(df))
    finally:
        group_fast.ENABLED = True
    _same(fast, slow)


def test_csv_dictionary_codes(tmp_path, spark):
    rs = np.random.RandomState(3)
    n = 70000
    wards = np.array(["icu", "er", 'a "q" b', "", "gen"])
    w = wards[rs.randint(0, 5, n)]
    p = tmp_path / "a.csv"
    with open(p, "w") as fh:
        fh.write("ward,los\n")
        for i in range(n):
            s = w[i]
            fh.write(('"' + s.replace('"', '""') + '"' if '"' in s else s) + f",{i % 11}\n")
    df = spark.read.csv(str(p), header=True, inferSchema=True)
    cd = df._cols["ward"]
    assert cd.codes is not None and cd.codes.dtype == np.int32
    vals = df.select("ward").toPandas()["ward"].tolist()
    expect = [None if s == "" else s for s in w]
    assert vals == expect
    got = {r[0]: r[1] for r in df.groupBy("ward").agg(F.sum("los")).collect()}
    los = np.arange(n) % 11
    for k in ("icu", "er", 'a "q" b', "gen", None):
        assert got[k] == int(sum(l for e, l in zip(expect, los) if e == k))
    # row subsets keep the codes aligned with the values
    sub = df.filter(F.col("los") > 5)
    assert sub._cols["ward"].codes is not None
    dic = {}
    for c, v in zip(sub._cols["ward"].codes, sub._cols["ward"].values):
        assert dic.setdefault(int(c), v) == v


@pytest.mark.gpu
def test_fast_equals_row_loop_gpu():
    s = SparkSession.builder.appName("gfast_gpu").master("mi355x").getOrCreate()
    try:
        df = _frame(s, n=20000, seed=4)
        assert df._device.type == "cuda"
        for qi, q in enumerate(QUERIES):
            group_fast.ENABLED = True
            fast = _rows(q(df))
            group_fast.ENABLED = False
            try:
                slow = _rows(q(df))
            finally:
                group_fast.ENABLED = True
            if qi == 1:
                fast = [r for r in fast if not (isinstance(r[0], float) and math.isnan(r[0]))]
                slow = [r for r in slow if not (isinstance(r[0], float) and math.isnan(r[0]))]
            _same(fast, slow)
    finally:
        s.stop()


@pytest.mark.parametrize("qi", [0, 1, 2, 5, 6, 7])
def test_columnar_merge_bitwise_equals_python_merge(spark, qi):
    """aggregate_fast (device merge of the tensor partials) against group.gather_partials /
    final_row over the same partials: identical values, bit for bit, and identical order."""
    from clustermachinelearningforhospitalnetworks_apache_spark_amd.sql import aggregate_fast
    df = _frame(spark)
    q = QUERIES[qi]
    dev = _rows(q(df))
    aggregate_fast.ENABLED = False
    try:
        py = _rows(q(df))
    finally:
        aggregate_fast.ENABLED = True
    assert len(dev) == len(py)
    for a, b in zip(dev, py):
        for u, v in zip(a, b):
            if isinstance(u, float) and isinstance(v, float) and math.isnan(u):
                assert math.isnan(v)
            else:
                assert u == v and type(u) is type(v), (a, b)


def test_high_cardinality_groupby(spark):
    import numpy as np
    import pandas as pd
    n = 50000
    rs = np.random.RandomState(1)
    pdf = pd.DataFrame({"pid": rs.randint(0, 20000, n), "v": rs.rand(n)})
    got = spark.createDataFrame(pdf).groupBy("pid").agg(F.count("*").alias("c"), F.sum("v").alias("s"),
                                                         F.max("v").alias("m"))
    from clustermachinelearningforhospitalnetworks_apache_spark_amd.sql.column import ColumnData
    assert all(not c.is_host for c in got._cols.values())  # device columns, no per-group Python rows
    ref = pdf.groupby("pid").v.agg(["size", "sum", "max"])
    rows = got.collect()
    assert len(rows) == len(ref)
    for r in rows[:500]:
        assert r.c == ref.loc[r.pid, "size"] and abs(r.s - ref.loc[r.pid, "sum"]) < 1e-9 and r.m == ref.loc[r.pid, "max"]
