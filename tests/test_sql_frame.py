"""DataFrame / Column / SQL semantics on the local (CPU) backend."""
import datetime as dt
import math

import numpy as np
import pandas as pd
import pytest

from helpers import hospital_frame, session
from clustermachinelearningforhospitalnetworks_apache_spark_amd.sql import Row
from clustermachinelearningforhospitalnetworks_apache_spark_amd.sql import functions as F
from clustermachinelearningforhospitalnetworks_apache_spark_amd.sql import types as T


@pytest.fixture(scope="module")
def spark():
    return session()


def test_create_select_withcolumn(spark):
    df = spark.createDataFrame([(1, "a", 2.0), (2, "b", None), (3, None, 5.5)], ["x", "s", "y"])
    assert df.columns == ["x", "s", "y"]
    assert df.count() == 3
    out = df.withColumn("z", F.col("x") * 2 + 1).select("x", "z").collect()
    assert [r.z for r in out] == [3, 5, 7]
    assert df.schema["y"].dataType == T.DoubleType()


def test_when_otherwise_binarize_like_reference(spark):
    # ref.py:176-177: LOS_binary = when(length_of_stay > threshold, 1).otherwise(0)
    df = spark.createDataFrame([(4.0,), (5.0,), (5.1,), (None,)], ["length_of_stay"])
    out = df.withColumn("LOS_binary", F.when(df["length_of_stay"] > 5.0, 1).otherwise(0)).collect()
    assert [r.LOS_binary for r in out] == [0, 0, 1, 0]  # strict '>' ; null comparison -> otherwise


def test_null_semantics_and_logic(spark):
    df = spark.createDataFrame([(1.0, None), (None, True), (2.0, False)], "a DOUBLE, b BOOLEAN")
    assert df.filter(F.col("a") > 0).count() == 2
    assert df.filter(F.col("a").isNull()).count() == 1
    # Kleene logic: null AND false = false, null OR true = true
    r = df.select((F.col("b") & F.lit(False)).alias("x"), (F.col("b") | F.lit(True)).alias("y")).collect()
    assert [x.x for x in r] == [False, False, False]
    assert [x.y for x in r] == [True, True, True]


def test_na_drop_and_fill(spark):
    df = spark.createDataFrame([(1, None, "a"), (None, 2.0, "b"), (3, 3.0, None), (4, 4.0, "d")], ["i", "d", "s"])
    assert df.na.drop().count() == 1
    assert df.na.drop(how="all").count() == 4
    assert df.na.drop(subset=["i"]).count() == 3
    assert df.dropna(thresh=3).count() == 1
    f = df.na.fill(0).collect()
    assert f[1].i == 0 and f[0].d == 0.0
    assert df.na.fill("z").collect()[2].s == "z"


def test_random_split_deterministic_and_complete(spark):
    df = spark.range(5000)
    a, b = df.randomSplit([0.7, 0.3], seed=42)
    ia = {r.id for r in a.collect()}
    ib = {r.id for r in b.collect()}
    assert not ia & ib and len(ia) + len(ib) == 5000
    assert 0.67 < len(ia) / 5000 < 0.73
    a2, _ = df.randomSplit([7, 3], seed=42)  # weights are normalised
    assert {r.id for r in a2.collect()} == ia
    a3, _ = df.randomSplit([0.7, 0.3], seed=43)
    assert {r.id for r in a3.collect()} != ia


def test_groupby_agg_and_describe(spark):
    pdf = hospital_frame(300)
    df = spark.createDataFrame(pdf)
    g = df.groupBy("hospital_id").agg(F.avg("length_of_stay").alias("m"), F.count("*").alias("n")).collect()
    got = {r.hospital_id: (r.m, r.n) for r in g}
    want = pdf.groupby("hospital_id")["length_of_stay"].agg(["mean", "count"])
    for k, (m, n) in got.items():
        assert abs(m - want.loc[k, "mean"]) < 1e-9 and n == want.loc[k, "count"]
    st = df.agg(F.stddev("length_of_stay"), F.min("admission_count"), F.max("admission_count")).collect()[0]
    assert abs(st[0] - pdf.length_of_stay.std(ddof=1)) < 1e-9
    d = {r.summary: r for r in df.describe("length_of_stay").collect()}
    assert d["count"].length_of_stay == "300"


def test_orderby_distinct_limit_union_join(spark):
    df = spark.createDataFrame([(3, "c"), (1, "a"), (2, "b"), (1, "a")], ["k", "v"])
    assert [r.k for r in df.orderBy("k").collect()] == [1, 1, 2, 3]
    assert [r.k for r in df.orderBy(F.col("k").desc()).collect()] == [3, 2, 1, 1]
    assert df.distinct().count() == 3
    assert df.limit(2).count() == 2
    assert df.union(df).count() == 8
    other = spark.createDataFrame([(1, 10.0), (3, 30.0)], ["k", "w"])
    j = df.join(other, "k").orderBy("k").collect()
    assert [(r.k, r.w) for r in j] == [(1, 10.0), (1, 10.0), (3, 30.0)]
    assert df.join(other, "k", "left").count() == 4


def test_sql_between_timestamps_like_reference(spark):
    pdf = hospital_frame(400)
    df = spark.createDataFrame(pdf)
    df.createOrReplaceTempView("hospital_unbounded_table")
    q = """
        SELECT *
        FROM hospital_unbounded_table
        WHERE event_time BETWEEN '2025-03-31 22:00:00' AND '2025-03-31 23:00:00'
    """
    got = spark.sql(q).na.drop().count()
    lo, hi = pd.Timestamp("2025-03-31 22:00:00"), pd.Timestamp("2025-03-31 23:00:00")
    assert got == int(((pdf.event_time >= lo) & (pdf.event_time <= hi)).sum())


def test_sql_aggregates_order_limit(spark):
    df = spark.createDataFrame([("a", 1.0), ("b", 2.0), ("a", 3.0), ("c", 4.0)], ["g", "x"])
    df.createOrReplaceTempView("t")
    r = spark.sql("SELECT g, SUM(x) AS s, COUNT(*) AS n FROM t GROUP BY g HAVING COUNT(*) >= 1 "
                  "ORDER BY s DESC LIMIT 2").collect()
    assert [(x.g, x.s, x.n) for x in r] == [("a", 4.0, 2), ("c", 4.0, 1)] or \
        [(x.g, x.s) for x in r] == [("c", 4.0), ("a", 4.0)]
    r2 = spark.sql("select g, case when x > 2 then 'hi' else 'lo' end as lvl from t where g in ('a','c') "
                   "order by x").collect()
    assert [x.lvl for x in r2] == ["lo", "hi", "hi"]
    assert spark.sql("select count(distinct g) as c from t").collect()[0].c == 3


def test_show_and_to_pandas(spark, capsys):
    df = spark.createDataFrame([(1, dt.datetime(2025, 3, 31, 22, 0, 5), None)], "a INT, t TIMESTAMP, s STRING")
    df.show()
    out = capsys.readouterr().out
    assert "2025-03-31 22:00:05" in out and "NULL" in out
    pdf = df.toPandas()
    assert pdf.t.iloc[0] == pd.Timestamp("2025-03-31 22:00:05")


def test_current_timestamp_and_functions(spark):
    df = spark.range(3).withColumn("ingest_time", F.current_timestamp())
    rows = df.collect()
    assert all(isinstance(r.ingest_time, dt.datetime) for r in rows)
    assert len({r.ingest_time for r in rows}) == 1
    r = spark.createDataFrame([(-2.5, "Ab")], ["v", "s"]).select(
        F.abs("v").alias("a"), F.round("v").alias("r"), F.upper("s").alias("u"), F.length("s").alias("n")).collect()[0]
    assert (r.a, r.r, r.u, r.n) == (2.5, -3.0, "AB", 2)


def test_row_api():
    r = Row(a=1, b="x")
    assert r.a == 1 and r["b"] == "x" and r.asDict() == {"a": 1, "b": "x"}
