"""Device relational operators (sql/relational_fast.py) against the row-loop implementations of
sql/group.py / sql/sqlparse.py: orderBy with mixed directions and null placement over numeric,
string, date and boolean keys; dropDuplicates (subset, nulls, -0.0); DataFrame.join for every join
type with string / multi-column keys, null keys and clashing names; SQL joins; repartition."""
import datetime as dt
import math

import numpy as np
import pytest

from clustermachinelearningforhospitalnetworks_apache_spark_amd.sql import SparkSession
from clustermachinelearningforhospitalnetworks_apache_spark_amd.sql import functions as F
from clustermachinelearningforhospitalnetworks_apache_spark_amd.sql import relational_fast as RF


def _frame(spark, n=600, seed=0):
    rs = np.random.RandomState(seed)
    rows = []
    for i in range(n):
        rows.append((int(rs.randint(0, 7)) if rs.rand() > 0.05 else None,
                     ["icu", "er", "gen", "ped", None][rs.randint(0, 5)],
                     float(rs.randint(-20, 20)) if rs.rand() > 0.05 else None,
                     dt.date(2024, 1, 1) + dt.timedelta(days=int(rs.randint(0, 30))),
                     bool(rs.rand() > 0.5), i))
    return spark.createDataFrame(rows, "g int, w string, x double, d date, b boolean, id long")


def _both(fn):
    RF.ENABLED = False
    try:
        host = fn()
    finally:
        RF.ENABLED = True
    return fn(), host


def _rows(df):
    return [tuple(r) for r in df.collect()]


@pytest.fixture(scope="module")
def spark():
    s = SparkSession.builder.master("local[1]").getOrCreate()
    yield s


ORDERS = [
    lambda: ["g", "x", "id"],
    lambda: [F.col("w").desc(), F.col("x").asc_nulls_last(), "id"],
    lambda: [F.col("d").desc(), F.col("b"), F.col("g").desc_nulls_last(), "id"],
    lambda: [F.col("x") * 2 + F.col("g"), "id"],
]


@pytest.mark.parametrize("k", range(len(ORDERS)))
def test_sort_matches_row_loop(spark, k):
    df = _frame(spark)
    dev, host = _both(lambda: _rows(df.orderBy(*ORDERS[k]())))
    assert dev == host


def test_sort_stable_and_ids(spark):
    df = _frame(spark)
    out = df.orderBy("g")
    ids = [r.id for r in out.collect()]
    gs = [r.g for r in out.collect()]
    # nulls first, stable within equal keys
    for a, b, ga, gb in zip(ids, ids[1:], gs, gs[1:]):
        if ga == gb:
            assert a < b
    assert gs[0] is None


def test_sort_nan_largest(spark):
    df = spark.createDataFrame([(1.0,), (float("nan"),), (None,), (-3.0,), (float("inf"),)], "x double")
    got = [r.x for r in df.orderBy("x").collect()]
    assert got[0] is None and got[1:3] == [-3.0, 1.0] and got[3] == float("inf") and math.isnan(got[4])
    got = [r.x for r in df.orderBy(F.col("x").desc()).collect()]
    assert math.isnan(got[0]) and got[-1] is None


@pytest.mark.parametrize("subset", [None, ["g"], ["w", "b"], ["g", "w"]])
def test_dedup_matches_row_loop(spark, subset):
    df = _frame(spark).drop("id")
    dev, host = _both(lambda: _rows(df.dropDuplicates(subset)))
    assert dev == host


def test_dedup_zero_and_nan(spark):
    df = spark.createDataFrame([(0.0,), (-0.0,), (float("nan"),), (float("nan"),), (None,), (None,)], "x double")
    got = [r.x for r in df.distinct().collect()]
    assert len(got) == 3 and got[0] == 0.0 and math.isnan(got[1]) and got[2] is None


HOWS = ["inner", "left", "right", "full", "leftsemi", "leftanti", "cross"]


@pytest.mark.parametrize("how", HOWS)
def test_join_matches_row_loop(spark, how):
    left = _frame(spark, 200)
    right = spark.createDataFrame([(g, w, float(g or 0) * 10, f"r{j}") for j, (g, w) in enumerate(
        [(0, "icu"), (1, "er"), (1, "er"), (3, None), (None, "gen"), (9, "icu"), (2, "ped"), (4, "gen")])],
        "g int, w string, x double, tag string")
    on = ["g", "w"] if how != "cross" else None
    fn = (lambda: _rows(left.crossJoin(right))) if how == "cross" else (lambda: _rows(left.join(right, on, how)))
    dev, host = _both(fn)
    assert dev == host
    if how != "cross":
        assert left.join(right, on, how).columns[-2:] == (["x_r", "tag"] if how not in ("leftsemi", "leftanti")
                                                          else left.columns[-2:])


def test_join_null_keys_never_match(spark):
    a = spark.createDataFrame([(None, 1), (1, 2)], "k int, v int")
    b = spark.createDataFrame([(None, "x"), (1, "y")], "k int, s string")
    assert [tuple(r) for r in a.join(b, "k").collect()] == [(1, 2, "y")]
    assert [tuple(r) for r in a.join(b, "k", "leftanti").collect()] == [(None, 1)]
    full = sorted([tuple(r) for r in a.join(b, "k", "full").collect()], key=str)
    assert full == sorted([(None, 1, None), (1, 2, "y"), (None, None, "x")], key=str)


def test_join_mixed_numeric_key_types(spark):
    a = spark.createDataFrame([(1,), (2,), (3,)], "k int")
    b = spark.createDataFrame([(1.0, "a"), (3.0, "c")], "k double, s string")
    assert [tuple(r) for r in a.join(b, "k").collect()] == [(1, "a"), (3, "c")]


def test_sql_join_matches_row_loop(spark):
    left = _frame(spark, 300)
    right = spark.createDataFrame([(i, f"name{i}", i * 1.5) for i in range(0, 8, 2)], "g int, name string, x double")
    left.createOrReplaceTempView("lt")
    right.createOrReplaceTempView("rt")
    qs = ["SELECT lt.id, rt.name, rt.x FROM lt JOIN rt ON lt.g = rt.g",
          "SELECT * FROM lt LEFT JOIN rt USING (g)",
          "SELECT * FROM lt FULL OUTER JOIN rt ON lt.g = rt.g AND lt.x = rt.x",
          "SELECT lt.id FROM lt LEFT ANTI JOIN rt ON lt.g = rt.g"]
    for q in qs:
        dev, host = _both(lambda: _rows(spark.sql(q)))
        assert dev == host, q


def test_repartition_keeps_rows(spark):
    df = _frame(spark)
    assert _rows(df.repartition(3)) == _rows(df)


@pytest.mark.gpu
def test_relational_gpu_matches_row_loop():
    s = SparkSession.builder.master("mi355x").getOrCreate()
    df = _frame(s, 5000, seed=3)
    assert df._device.type == "cuda"
    for order in ORDERS:
        dev, host = _both(lambda: _rows(df.orderBy(*order())))
        assert dev == host
    dev, host = _both(lambda: _rows(df.drop("id").dropDuplicates(["g", "w", "b"])))
    assert dev == host
    right = s.createDataFrame([(g, f"t{g}") for g in range(0, 7, 2)], "g int, tag string")
    for how in ("inner", "left", "full", "leftanti"):
        dev, host = _both(lambda: _rows(df.join(right, "g", how)))
        assert dev == host


def test_device_paths_do_not_gather_rows(spark, monkeypatch):
    """The device operators never fall back to the row loop for supported keys."""
    from clustermachinelearningforhospitalnetworks_apache_spark_amd.sql.dataframe import DataFrame

    def boom(self):
        raise AssertionError("row-loop path taken")
    df = _frame(spark)
    right = spark.createDataFrame([(1, "a")], "g int, tag string")
    monkeypatch.setattr(DataFrame, "_gather_host", boom)
    df.orderBy(F.col("w").desc(), "x").count()
    df.dropDuplicates(["g", "w"]).count()
    df.join(right, "g", "full").count()
    df.repartition(2).count()


@pytest.mark.parametrize("op", ["intersect", "intersectAll", "subtract", "exceptAll"])
def test_set_ops_match_row_loop(spark, op):
    a = _frame(spark, 400, seed=1).select("g", "w", "b")
    b = _frame(spark, 300, seed=2).select("g", "w", "b")
    dev, host = _both(lambda: _rows(getattr(a, op)(b)))
    assert dev == host and len(dev) > 0


def test_dictionary_encoded_strings_match_row_loop(spark, monkeypatch):
    """String columns dictionary-encoded at creation (codes + distinct strings) go through the
    same sort / dedup / join / set-operation results as plain object columns."""
    from clustermachinelearningforhospitalnetworks_apache_spark_amd.sql import builder
    from clustermachinelearningforhospitalnetworks_apache_spark_amd.sql.column import DictColumnData
    monkeypatch.setattr(builder, "DICT_MIN_ROWS", 16)
    df = _frame(spark, 500, seed=5)
    assert isinstance(df._cols["w"], DictColumnData)
    right = spark.createDataFrame([(w, f"t{j}") for j, w in enumerate(["icu", "er", "er", None, "onc"] * 5)],
                                  "w string, tag string")
    other = _frame(spark, 300, seed=6).select("w", "g")
    cases = [lambda: _rows(df.orderBy(F.col("w").desc_nulls_last(), "id")),
             lambda: _rows(df.dropDuplicates(["w", "b"])),
             lambda: _rows(df.join(right, "w", "full")),
             lambda: _rows(df.select("w", "g").exceptAll(other)),
             lambda: _rows(df.orderBy("w", "id").join(right, "w", "leftanti"))]
    for fn in cases:
        dev, host = _both(fn)
        assert dev == host
    out = df.orderBy("w")
    assert isinstance(out._cols["w"], DictColumnData)
