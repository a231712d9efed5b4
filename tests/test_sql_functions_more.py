"""Statistical aggregates (vs numpy / scipy), math / date / string scalars, arrays, structs and the
explode generators of sql.functions_more."""
import datetime as dt

import numpy as np
import pytest

from helpers import session
from clustermachinelearningforhospitalnetworks_apache_spark_amd.sql import functions as F


@pytest.fixture(scope="module")
def spark():
    return session()


def test_stat_aggregates_match_numpy(spark):
    from scipy import stats
    rs = np.random.RandomState(0)
    n = 500
    x = rs.gamma(2.0, size=n)
    y = 0.5 * x + rs.normal(size=n)
    g = rs.randint(0, 3, n)
    df = spark.createDataFrame([(float(a), float(b), int(c)) for a, b, c in zip(x, y, g)],
                               "x DOUBLE, y DOUBLE, g INT")
    r = df.select(F.skewness("x"), F.kurtosis("x"), F.corr("x", "y"), F.covar_pop("x", "y"),
                  F.covar_samp("x", "y"), F.median("x"), F.percentile("x", [0.1, 0.9]),
                  F.count_if(F.col("x") > 2), F.max_by("y", "x"), F.min_by("g", "x")).collect()[0]
    assert r[0] == pytest.approx(stats.skew(x), rel=1e-10)
    assert r[1] == pytest.approx(stats.kurtosis(x), rel=1e-10)
    assert r[2] == pytest.approx(np.corrcoef(x, y)[0, 1], rel=1e-10)
    assert r[3] == pytest.approx(np.cov(x, y, ddof=0)[0, 1], rel=1e-10)
    assert r[4] == pytest.approx(np.cov(x, y, ddof=1)[0, 1], rel=1e-10)
    assert r[5] == pytest.approx(np.median(x))
    np.testing.assert_allclose(r[6], np.percentile(x, [10, 90]))
    assert r[7] == int((x > 2).sum())
    assert r[8] == pytest.approx(y[np.argmax(x)]) and r[9] == g[np.argmin(x)]
    # grouped: the merge formulas per group
    grp = {row[0]: row[1:] for row in df.groupBy("g").agg(F.skewness("x"), F.corr("x", "y"),
                                                           F.mode("g"), F.product(F.lit(1.0))).collect()}
    for c in range(3):
        m = g == c
        assert grp[c][0] == pytest.approx(stats.skew(x[m]), rel=1e-9)
        assert grp[c][1] == pytest.approx(np.corrcoef(x[m], y[m])[0, 1], rel=1e-9)
        assert grp[c][2] == c and grp[c][3] == 1.0


def test_moment_merge_is_exact():
    from clustermachinelearningforhospitalnetworks_apache_spark_amd.sql.functions_more import (_merge_moments4,
                                                                                             _moments4)
    import torch
    rs = np.random.RandomState(1)
    x = rs.normal(3, 2, 1000) ** 3
    whole = _moments4(torch.as_tensor(x))
    parts = [_moments4(torch.as_tensor(p)) for p in np.array_split(x, 7)]
    merged = _merge_moments4(parts)
    np.testing.assert_allclose(merged[1:], whole[1:], rtol=1e-9)
    assert merged[0] == whole[0]


def test_math_and_string_scalars(spark):
    df = spark.createDataFrame([(2.0, 3.0, "hello world", float("nan")), (-8.0, 0.5, "ab", 1.0)],
                               "a DOUBLE, b DOUBLE, s STRING, c DOUBLE")
    r = df.select(F.pow("a", "b"), F.atan2("a", "b"), F.cbrt("a"), F.bround(F.lit(2.5)), F.nanvl("c", "a"),
                  F.initcap("s"), F.instr("s", "o"), F.translate("s", "lo", "01"), F.md5("s"), F.sha2("s", 256),
                  F.reverse("s"), F.repeat("s", 2)).collect()
    assert r[0][0] == 8.0 and r[0][1] == pytest.approx(np.arctan2(2, 3))
    assert r[1][2] == pytest.approx(-2.0) and r[0][3] == 2.0
    assert r[0][4] == 2.0 and r[1][4] == 1.0
    assert r[0][5] == "Hello World" and r[0][6] == 5 and r[0][7] == "he001 w1r0d"
    import hashlib
    assert r[0][8] == hashlib.md5(b"hello world").hexdigest()
    assert r[0][9] == hashlib.sha256(b"hello world").hexdigest()
    assert r[1][10] == "ba" and r[1][11] == "abab"


def test_date_functions(spark):
    df = spark.createDataFrame([(dt.datetime(2024, 1, 31, 10, 30), dt.datetime(2023, 11, 30, 0, 0))],
                               "t TIMESTAMP, u TIMESTAMP")
    r = df.select(F.dayofyear("t"), F.weekofyear("t"), F.quarter("t"), F.last_day("t"), F.add_months("t", 1),
                  F.months_between("t", "u"), F.date_trunc("month", "t"), F.trunc("t", "year")).collect()[0]
    assert r[0] == 31 and r[1] == 5 and r[2] == 1
    assert r[3] == dt.date(2024, 1, 31)
    assert r[4] == dt.date(2024, 2, 29)  # month end -> month end
    assert r[5] == 2.0  # both month ends
    assert r[6] == dt.datetime(2024, 1, 1) and r[7] == dt.date(2024, 1, 1)


def test_arrays_structs_explode(spark):
    df = spark.createDataFrame([(1, "a,b,c"), (2, ""), (3, None)], "id INT, s STRING")
    arr = df.withColumn("parts", F.split("s", ","))
    sizes = [r[0] for r in arr.select(F.size("parts")).collect()]
    assert sizes == [3, 1, -1]
    ex = arr.select("id", F.explode("parts").alias("p"))
    assert [(r.id, r.p) for r in ex.collect()] == [(1, "a"), (1, "b"), (1, "c"), (2, "")]
    pe = arr.select("id", F.posexplode("parts").alias("i", "v"))
    assert pe.columns == ["id", "i", "v"] and [tuple(r) for r in pe.collect()][:2] == [(1, 0, "a"), (1, 1, "b")]
    eo = arr.select("id", F.explode_outer("parts"))
    assert eo.count() == 5 and eo.columns == ["id", "col"]
    wc = arr.withColumn("p", F.explode("parts"))
    assert wc.count() == 4 and wc.columns[-1] == "p"
    nums = spark.createDataFrame([(1.0, 5.0, 3.0), (2.0, 2.0, 9.0)], "a DOUBLE, b DOUBLE, c DOUBLE")
    a = nums.select(F.array("a", "b", "c").alias("v"))
    r = a.select(F.array_max("v"), F.array_min("v"), F.sort_array("v", False), F.element_at("v", -1),
                 F.array_contains("v", 9.0), F.array_join("v", "|")).collect()
    assert r[0][0] == 5.0 and r[1][1] == 2.0 and r[0][2] == [5.0, 3.0, 1.0] and r[1][3] == 9.0
    assert r[1][4] is True and r[0][5] == "1.0|5.0|3.0"
    st = nums.select(F.struct("a", "b").alias("s")).collect()
    assert st[0].s.a == 1.0 and st[1].s.b == 2.0
    # exploded rows get fresh global row ids
    assert ex._row_ids.tolist() == [0, 1, 2, 3]
