"""Spark 3.4/3.5 function additions (sql/functions_tail.py): regression aggregates against numpy,
discrete percentiles, string / bitwise aggregation, try_* overflow, regex / URL / string helpers,
number formatting and timestamp arithmetic (values from Spark's function documentation where it
gives them)."""
import datetime as dt

import numpy as np
import pytest

from clustermachinelearningforhospitalnetworks_apache_spark_amd.sql import SparkSession
from clustermachinelearningforhospitalnetworks_apache_spark_amd.sql import functions as F


@pytest.fixture(scope="module")
def spark():
    s = SparkSession.builder.appName("ft").master("local[1]").getOrCreate()
    yield s
    s.stop()


def test_regr_aggregates(spark):
    rs = np.random.RandomState(0)
    x = rs.normal(size=500)
    y = 2.5 * x - 1.0 + rs.normal(size=500) * 0.3
    rows = [(float(a), float(b), int(i % 3)) for i, (a, b) in enumerate(zip(y, x))]
    rows.append((None, 1.0, 0))
    df = spark.createDataFrame(rows, "y double, x double, g int")
    r = df.select(F.regr_count("y", "x"), F.regr_slope("y", "x"), F.regr_intercept("y", "x"), F.regr_r2("y", "x"),
                  F.regr_avgx("y", "x"), F.regr_avgy("y", "x"), F.regr_sxx("y", "x"), F.regr_syy("y", "x"),
                  F.regr_sxy("y", "x")).collect()[0]
    slope, icpt = np.polyfit(x, y, 1)
    r2 = np.corrcoef(x, y)[0, 1] ** 2
    assert r[0] == 500
    np.testing.assert_allclose(list(r[1:]), [slope, icpt, r2, x.mean(), y.mean(), ((x - x.mean()) ** 2).sum(),
                                             ((y - y.mean()) ** 2).sum(), ((x - x.mean()) * (y - y.mean())).sum()],
                               rtol=1e-9)
    per = {row.g: row.s for row in df.groupBy("g").agg(F.regr_slope("y", "x").alias("s")).collect()}
    for gg in range(3):
        m = np.arange(500) % 3 == gg
        assert per[gg] == pytest.approx(np.polyfit(x[m], y[m], 1)[0], rel=1e-9)


def test_percentiles_string_and_bit_aggs(spark):
    df = spark.createDataFrame([(i, f"w{i}", i * 3) for i in [1, 2, 3, 4, 10]], "v int, s string, b long")
    r = df.select(F.percentile_disc("v", 0.5), F.percentile_cont("v", 0.5), F.percentile_disc("v", 0.9),
                  F.string_agg("s", ","), F.bit_and("b"), F.bit_or("b"), F.bit_xor("b"), F.std("v"),
                  F.any_value("v")).collect()[0]
    assert r[0] == 3.0 and r[1] == 3.0 and r[2] == 10.0
    assert r[3] == "w1,w2,w3,w4,w10"
    b = [3, 6, 9, 12, 30]
    assert r[4] == (3 & 6 & 9 & 12 & 30) and r[5] == (3 | 6 | 9 | 12 | 30) and r[6] == (3 ^ 6 ^ 9 ^ 12 ^ 30)
    assert r[7] == pytest.approx(np.std([1, 2, 3, 4, 10], ddof=1))


def test_try_and_null_safe(spark):
    df = spark.createDataFrame([(2 ** 62, 2, None), (-5, 3, 1)], "a long, b long, c int")
    r = df.select(F.try_multiply("a", "b"), F.try_subtract("a", "b"), F.equal_null("c", F.lit(None)),
                  F.zeroifnull("c"), F.nullifzero(F.lit(0)), F.pmod("a", "b"), F.try_element_at(F.array(F.lit(1)), 5)
                  ).collect()
    assert r[0][0] is None and r[0][1] == 2 ** 62 - 2 and r[0][2] is True and r[0][3] == 0 and r[0][4] is None
    assert r[1][0] == -15 and r[1][5] == 1 and r[1][2] is False and r[1][6] is None
    big = spark.createDataFrame([(2 ** 31 - 1, 1)], "a int, b int").select(F.try_multiply("a", "b"),
                                                                        F.try_subtract(F.lit(-2 ** 31), "b")).collect()
    assert big[0][0] == 2 ** 31 - 1 and big[0][1] is None


def test_string_helpers(spark):
    df = spark.createDataFrame([("11.12.13", "Spark SQL", "AbCD123-@$#")], "a string, s string, m string")
    r = df.select(F.split_part("a", F.lit("."), F.lit(3)), F.split_part("a", F.lit("."), F.lit(-1)),
                  F.split_part("a", F.lit("."), F.lit(9)), F.regexp_count("s", r"[a-z]"), F.regexp_substr("s", r"S\w+"),
                  F.regexp_instr("s", "SQL"), F.regexp_like("s", "^Sp"), F.startswith("s", "Spa"),
                  F.endswith("s", "QL"), F.contains("s", "k S"), F.left("s", 3), F.right("s", 3), F.btrim(F.lit("  x ")),
                  F.chr(F.lit(65)), F.mask("m"), F.url_encode(F.lit("a b&c")), F.url_decode(F.lit("a+b%26c")),
                  F.parse_url(F.lit("http://spark.apache.org/path?query=1#frag"), "HOST"),
                  F.parse_url(F.lit("http://spark.apache.org/path?query=1"), "QUERY", "query"),
                  F.to_char(F.lit(454.0), "999.00"), F.to_char(F.lit(-12454.8), "99,999.9MI"),
                  F.width_bucket(F.lit(5.3), F.lit(0.2), F.lit(10.6), 5), F.log(F.lit(2.0), F.lit(8.0)),
                  F.bit_count(F.lit(7)), F.bit_get(F.lit(5), 2), F.e(), F.pi()).collect()[0]
    assert list(r[:19]) == ["13", "13", "", 4, "Spark", 7, True, True, True, True, "Spa", "SQL", "x", "A",
                            "XxXXnnn-@$#", "a+b%26c", "a b&c", "spark.apache.org", "1"]
    assert r[19] == "454.00" and r[20] == "12,454.8-" and r[21] == 3 and r[22] == pytest.approx(3.0)
    assert r[23] == 3 and r[24] == 1 and r[25] == pytest.approx(np.e) and r[26] == pytest.approx(np.pi)


def test_timestamp_arithmetic(spark):
    df = spark.createDataFrame([(dt.datetime(2016, 3, 11, 9, 0, 7), dt.datetime(2024, 4, 1, 11, 0, 0))],
                               "a timestamp, b timestamp")
    r = df.select(F.timestampadd("YEAR", 1, "a"), F.timestampadd("SECOND", -10, "a"), F.timestampdiff("DAY", "a", "b"),
                  F.timestampdiff("MONTH", "a", "b"), F.dayname("a"), F.monthname("a"), F.weekday("a"), F.day("a"),
                  F.convert_timezone(F.lit("Europe/Brussels"), F.lit("America/Los_Angeles"), "a"),
                  F.date_diff("b", "a")).collect()[0]
    assert r[0] == dt.datetime(2017, 3, 11, 9, 0, 7) and r[1] == dt.datetime(2016, 3, 11, 8, 59, 57)
    assert r[2] == (dt.datetime(2024, 4, 1, 11) - dt.datetime(2016, 3, 11, 9, 0, 7)).days
    assert r[3] == 96 and r[4] == "Fri" and r[5] == "Mar" and r[6] == 4 and r[7] == 11
    assert r[8] == dt.datetime(2016, 3, 11, 0, 0, 7)
    assert r[9] == (dt.date(2024, 4, 1) - dt.date(2016, 3, 11)).days
    assert len(spark.range(3).select(F.uuid()).collect()[0][0]) == 36


def test_string_functions_per_distinct_on_dictionary_columns(monkeypatch):
    """Row functions over a dictionary-encoded column run once per distinct value and give the
    same rows as the per-row evaluation."""
    from clustermachinelearningforhospitalnetworks_apache_spark_amd.sql import SparkSession, builder
    from clustermachinelearningforhospitalnetworks_apache_spark_amd.sql import functions as F
    from clustermachinelearningforhospitalnetworks_apache_spark_amd.sql import functions as Fm
    from clustermachinelearningforhospitalnetworks_apache_spark_amd.sql.column import DictColumnData
    s = SparkSession.builder.master("local[1]").getOrCreate()
    rows = [(["icu-a", "er-b", None, "gen-c", "icu-d"][i % 5], i) for i in range(3000)]
    monkeypatch.setattr(Fm, "_DISTINCT_MIN_ROWS", 16)
    monkeypatch.setattr(builder, "DICT_MIN_ROWS", 16)
    dd = s.createDataFrame(rows, "w string, i int")
    assert isinstance(dd._cols["w"], DictColumnData)
    monkeypatch.setattr(builder, "DICT_MIN_ROWS", 1 << 30)
    plain = s.createDataFrame(rows, "w string, i int")
    q = lambda d: [tuple(r) for r in d.select(F.upper("w"), F.col("w").startswith("icu"), F.length("w"),  # noqa
                                                F.regexp_replace("w", "-", "_"), F.col("w").like("%-_"),
                                                F.substring("w", 2, 3)).collect()]
    assert q(dd) == q(plain)
    out = dd.select(F.regexp_replace("w", "-", "_").alias("u"))
    assert isinstance(out._cols["u"], DictColumnData)
    assert dd.filter(F.col("w").contains("icu")).count() == 1200
