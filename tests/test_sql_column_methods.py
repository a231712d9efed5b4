"""pyspark Column methods (string predicates, LIKE / ILIKE / RLIKE, substr and slicing, getItem /
getField / [], eqNullSafe, bitwise operators, ** and reflected %, withField / dropFields) and the
remaining pyspark.sql.functions (find_in_set, elt, get, position, replace, regexp_extract_all,
str_to_map, to_csv / from_csv, partition transforms, histogram_numeric, nth_value, call_function)."""
import datetime as dt

import pytest

from clustermachinelearningforhospitalnetworks_apache_spark_amd.sql import SparkSession, Window
from clustermachinelearningforhospitalnetworks_apache_spark_amd.sql import functions as F
from clustermachinelearningforhospitalnetworks_apache_spark_amd.sql.types import Row


@pytest.fixture(scope="module")
def df():
    s = SparkSession.builder.master("local[1]").getOrCreate()
    return s.createDataFrame([("icu", 1, None, {"a": 1}), ("er", 2, 3.5, {"a": 2}), ("icu", 3, 4.0, None),
                              ("gen_x", 4, 1.0, {"a": 5})], "w string, x int, y double, m map<string,int>")


def test_string_predicates(df):
    c = F.col("w")
    assert df.filter(c.startswith("ic")).count() == 2
    assert df.filter(c.endswith("x")).count() == 1
    assert df.filter(c.contains("c")).count() == 2
    assert df.filter(c.like("%c_")).count() == 2
    assert df.filter(c.like("gen\\_%")).count() == 1 and df.filter(c.like("ge__%")).count() == 1
    assert df.filter(c.ilike("ICU")).count() == 2
    assert df.filter(c.rlike("^e")).count() == 1


def test_substr_items_fields(df):
    r = df.select(F.col("w").substr(2, 2).alias("a"), F.col("w")[1:2].alias("b"), F.col("m")["a"].alias("c"),
                  F.col("m").getItem("a").alias("d")).collect()
    assert [(x.a, x.b, x.c, x.d) for x in r] == [("cu", "ic", 1, 1), ("r", "er", 2, 2), ("cu", "ic", None, None),
                                                 ("en", "ge", 5, 5)]
    st = df.select(F.struct("w", "x").alias("s"))
    got = st.select(F.col("s").withField("z", F.lit(1)).alias("a"), F.col("s").dropFields("w").alias("b"),
                    F.col("s")["x"].alias("c"), F.col("s").getField("w").alias("d")).collect()[0]
    assert got.a == Row(w="icu", x=1, z=1) and got.b == Row(x=1) and got.c == 1 and got.d == "icu"


def test_operators(df):
    r = df.select(F.col("x").bitwiseAND(2).alias("a"), F.col("x").bitwiseOR(8).alias("b"),
                  F.col("x").bitwiseXOR(1).alias("c"), (F.col("x") ** 2).alias("d"), (7 % F.col("x")).alias("e"),
                  F.col("y").eqNullSafe(None).alias("f"), F.col("y").isNaN().alias("g")).collect()
    assert [x.a for x in r] == [0, 2, 2, 0] and [x.b for x in r] == [9, 10, 11, 12]
    assert [x.c for x in r] == [0, 3, 2, 5] and [x.d for x in r] == [1.0, 4.0, 9.0, 16.0]
    assert [x.e for x in r] == [0, 1, 1, 3] and [x.f for x in r] == [True, False, False, False]
    assert str(F.col("x").bitwiseAND(2)._expr) == "(x & 2)"


def test_more_functions(df):
    r = df.select(F.find_in_set(F.lit("b"), F.lit("a,b,c")).alias("a"), F.elt(F.lit(2), F.lit("p"), F.lit("q")).alias("b"),
                  F.position(F.lit("c"), "w").alias("c"), F.replace("w", F.lit("i"), F.lit("I")).alias("d"),
                  F.regexp_extract_all("w", F.lit("([a-z])"), 1).alias("e"), F.str_to_map(F.lit("a:1,b:2")).alias("f"),
                  F.to_csv(F.struct("w", "x")).alias("g"), F.negate("x").alias("h"),
                  F.call_function("upper", F.col("w")).alias("i")).collect()[0]
    assert (r.a, r.b, r.c, r.d, r.e, r.f, r.g, r.h, r.i) == (2, "q", 2, "Icu", ["i", "c", "u"], {"a": "1", "b": "2"},
                                                              "icu,1", -1, "ICU")
    got = df.select(F.from_csv(F.lit("1,abc"), "a INT, b STRING").alias("c")).collect()[0].c
    assert got == Row(a=1, b="abc")
    h = df.agg(F.histogram_numeric("x", 2).alias("h")).collect()[0].h
    assert [(p.x, p.y) for p in h] == [(1.5, 2.0), (3.5, 2.0)]


def test_partition_transforms(df):
    s = df.sparkSession if hasattr(df, "sparkSession") else None
    t = SparkSession.builder.master("local[1]").getOrCreate().createDataFrame(
        [(dt.datetime(2024, 3, 5, 7, 30),)], "t timestamp")
    r = t.select(F.years("t").alias("y"), F.months("t").alias("m"), F.days("t").alias("d"),
                 F.hours("t").alias("h")).collect()[0]
    assert r.y == 54 and r.m == 54 * 12 + 2 and r.d == dt.date(2024, 3, 5)
    assert r.h == (dt.datetime(2024, 3, 5, 7, 30) - dt.datetime(1970, 1, 1)).days * 24 + 7


def test_nth_value(df):
    w = Window.partitionBy("w").orderBy("x").rowsBetween(Window.unboundedPreceding, Window.unboundedFollowing)
    r = df.select("w", "x", F.nth_value("y", 2).over(w).alias("n2"), F.nth_value("y", 1, True).over(w).alias("n1"))
    got = {(x.w, x.x): (x.n2, x.n1) for x in r.collect()}
    assert got[("icu", 1)] == (4.0, 4.0) and got[("er", 2)] == (None, 3.5)
    wr = Window.partitionBy("w").orderBy("x")  # default frame: unbounded preceding .. current row
    got = {(x.w, x.x): x.n for x in df.select("w", "x", F.nth_value("y", 2).over(wr).alias("n")).collect()}
    assert got[("icu", 1)] is None and got[("icu", 3)] == 4.0
