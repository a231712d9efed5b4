"""first / last with and without ignoreNulls, and try_sum's overflow-to-null, against a plain Python
model of Spark's semantics (functions.first(col, ignorenulls=False) picks the group's first ROW, null
included; try_sum is null when an integral total leaves the LongType range, while sum wraps as
Spark's non-ANSI LongType arithmetic does). Property-tested on random null patterns with the device
group-by on and off, and on W=2 gloo ranks (row order across shards = rank order)."""
import json
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp
from hypothesis import given, settings
from hypothesis import strategies as st

from clustermachinelearningforhospitalnetworks_apache_spark_amd.sql import SparkSession
from clustermachinelearningforhospitalnetworks_apache_spark_amd.sql import functions as F
from clustermachinelearningforhospitalnetworks_apache_spark_amd.sql import functions_tail as FT
from clustermachinelearningforhospitalnetworks_apache_spark_amd.sql import group_fast
from clustermachinelearningforhospitalnetworks_apache_spark_amd.sql import types as T

SCHEMA = T.StructType([T.StructField("g", T.IntegerType()), T.StructField("v", T.LongType()),
                       T.StructField("x", T.DoubleType())])


def _wrap(s):
    return (s + 2 ** 63) % 2 ** 64 - 2 ** 63


def _model(rows):
    out = {}
    for g, v, x in rows:
        out.setdefault(g, []).append((v, x))
    res = {}
    for g, vals in out.items():
        vs = [v for v, _ in vals]
        nn = [v for v in vs if v is not None]
        xs = [x for _, x in vals]
        xnn = [x for x in xs if x is not None]
        tot = sum(nn)
        res[g] = {"f": vs[0], "l": vs[-1], "fi": nn[0] if nn else None, "li": nn[-1] if nn else None,
                  "fx": xs[0], "lxi": xnn[-1] if xnn else None,
                  "sum": _wrap(tot) if nn else None,
                  "try_sum": (tot if -2 ** 63 <= tot < 2 ** 63 else None) if nn else None,
                  "try_avg": (sum(float(v) for v in nn) / len(nn)) if nn else None}
    return res


def _query(df):
    return df.groupBy("g").agg(
        F.first("v").alias("f"), F.last("v").alias("l"),
        F.first("v", ignorenulls=True).alias("fi"), FT.last_value("v", True).alias("li"),
        FT.first_value("x").alias("fx"), F.last("x", True).alias("lxi"),
        F.sum("v").alias("sum"), FT.try_sum("v").alias("try_sum"), FT.try_avg("v").alias("try_avg"))


def _collect(df):
    return {r["g"]: {k: r[k] for k in ("f", "l", "fi", "li", "fx", "lxi", "sum", "try_sum", "try_avg")}
            for r in _query(df).collect()}


def _check(got, want):
    assert set(got) == set(want)
    for g in want:
        for k, w in want[g].items():
            v = got[g][k]
            if k == "try_avg" and w is not None:
                assert v == pytest.approx(w, rel=1e-12), (g, k)
            else:
                assert v == w, (g, k, v, w)


_val = st.one_of(st.none(), st.integers(-5, 5),
                 st.sampled_from([2 ** 62, 2 ** 62 + 7, -(2 ** 62), 2 ** 63 - 1, -(2 ** 63)]))
_row = st.tuples(st.integers(0, 3), _val, st.one_of(st.none(), st.floats(-9, 9, allow_nan=False)))


@pytest.fixture(scope="module")
def spark():
    s = SparkSession.builder.master("local[1]").getOrCreate()
    yield s


@settings(max_examples=40, deadline=None)
@given(rows=st.lists(_row, min_size=1, max_size=24))
def test_first_last_try_sum_property(spark, rows):
    df = spark.createDataFrame(rows, SCHEMA)
    want = _model(rows)
    _check(_collect(df), want)
    old = group_fast.ENABLED
    group_fast.ENABLED = False
    try:
        _check(_collect(df), want)
    finally:
        group_fast.ENABLED = old


def test_first_defaults_to_row_semantics(spark):
    df = spark.createDataFrame([(1, None, 1.0), (1, 5, None), (1, None, 2.0)], SCHEMA)
    r = _query(df).collect()[0]
    assert r["f"] is None and r["l"] is None and r["fi"] == 5 and r["li"] == 5
    assert r["fx"] == 1.0 and r["lxi"] == 2.0
    # without nulls the device path runs and agrees
    df2 = spark.createDataFrame([(1, 3, 1.0), (1, 4, 2.0)], SCHEMA)
    r2 = _query(df2).collect()[0]
    assert (r2["f"], r2["l"], r2["fi"], r2["li"]) == (3, 4, 3, 4)


def test_try_sum_overflow_is_null_sum_wraps(spark):
    big = 2 ** 63 - 1
    df = spark.createDataFrame([(0, big, 0.0), (0, 1, 0.0), (1, big, 0.0), (1, -1, 0.0)], SCHEMA)
    got = {r["g"]: r for r in _query(df).collect()}
    assert got[0]["try_sum"] is None and got[0]["sum"] == -(2 ** 63)
    assert got[1]["try_sum"] == big - 1 == got[1]["sum"]


# ---------------------------------------------------------------- W=2: first/last follow rank order

_ROWS = [(0, None, 1.0), (0, 7, None), (1, 2 ** 63 - 1, 3.0), (0, 8, 4.0), (1, 5, None), (0, None, None)]


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _rank_main(rank, world, port, out_path):
    os.environ.update({"RANK": str(rank), "WORLD_SIZE": str(world), "LOCAL_RANK": str(rank),
                       "MASTER_ADDR": "127.0.0.1", "MASTER_PORT": str(port), "CML_FORCE_CPU": "1"})
    import torch
    torch.set_num_threads(1)
    spark = SparkSession.builder.master("local[1]").getOrCreate()
    got = _collect(spark.createDataFrame(_ROWS, SCHEMA))
    if rank == 0:
        with open(out_path, "w") as fh:
            json.dump({str(k): v for k, v in got.items()}, fh)
    spark.stop()


def test_first_last_two_ranks(tmp_path):
    out = str(tmp_path / "w2.json")
    mp.start_processes(_rank_main, args=(2, _free_port(), out), nprocs=2, join=True, start_method="spawn")
    with open(out) as fh:
        got = {int(k): v for k, v in json.load(fh).items()}
    _check(got, _model(_ROWS))


def test_window_first_last_ignore_nulls_and_try_sum(spark):
    from clustermachinelearningforhospitalnetworks_apache_spark_amd.sql.window import Window
    rows = [(0, None, 1.0), (0, 4, 2.0), (0, None, 3.0), (0, 2 ** 63 - 1, 4.0), (1, None, 1.0)]
    df = spark.createDataFrame(rows, SCHEMA)
    w = Window.partitionBy("g").orderBy("x").rowsBetween(Window.unboundedPreceding, Window.currentRow)
    out = df.select("g", "x", F.first("v").over(w).alias("f"), F.first("v", True).over(w).alias("fi"),
                    F.last("v", True).over(w).alias("li"), FT.try_sum("v").over(w).alias("ts"),
                    F.sum("v").over(w).alias("s")).orderBy("g", "x").collect()
    assert [r["f"] for r in out] == [None, None, None, None, None]
    assert [r["fi"] for r in out] == [None, 4, 4, 4, None]
    assert [r["li"] for r in out] == [None, 4, 4, 2 ** 63 - 1, None]
    assert [r["ts"] for r in out] == [None, 4, 4, None, None]
    assert [r["s"] for r in out] == [None, 4, 4, -(2 ** 63) + 3, None]
