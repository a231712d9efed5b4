"""pyspark.sql.functions completed in round 2 (sql/functions_extra.py, sql/hashing.py,
sql/datetimefmt.py): values from Spark's own function documentation where it gives them
(hash / xxhash64 / conv / shiftrightunsigned / soundex / format_number / ...), Python references
otherwise. The device hash lanes are checked against the host recipes row by row."""
import datetime as dt
import math

import numpy as np
import pytest

from clustermachinelearningforhospitalnetworks_apache_spark_amd.sql import SparkSession
from clustermachinelearningforhospitalnetworks_apache_spark_amd.sql import functions as F
from clustermachinelearningforhospitalnetworks_apache_spark_amd.sql import types as T
from clustermachinelearningforhospitalnetworks_apache_spark_amd.sql.hashing import hash_value


@pytest.fixture(scope="module")
def spark():
    s = SparkSession.builder.appName("fx").master("local[1]").getOrCreate()
    yield s
    s.stop()


def one(spark, *cols, schema="s string", row=("Spark",)):
    return spark.createDataFrame([row], schema).select(*cols).collect()[0]


def test_hash_doc_values(spark):
    r = one(spark, F.hash("s", F.array(F.lit(123)), F.lit(2)), F.xxhash64("s", F.array(F.lit(123)), F.lit(2)))
    assert r[0] == -1321691492
    assert r[1] == 5602566077635097486


def test_device_hash_lanes_match_host(spark):
    rs = np.random.RandomState(0)
    n = 300
    rows = []
    for i in range(n):
        rows.append((int(rs.randint(-2 ** 31, 2 ** 31)), int(rs.randint(-2 ** 62, 2 ** 62)), float(rs.normal()),
                     bool(rs.rand() > 0.5), dt.date(2020, 1, 1) + dt.timedelta(days=int(rs.randint(0, 900))),
                     dt.datetime(2024, 1, 1) + dt.timedelta(seconds=int(rs.randint(0, 10 ** 7)))))
    rows[3] = (0, 0, -0.0, False, rows[3][4], rows[3][5])
    rows[4] = (None, None, float("nan"), None, None, None)
    schema = "i int, l long, d double, b boolean, dd date, t timestamp"
    df = spark.createDataFrame(rows, schema)
    got = df.select(F.hash("i", "l", "d", "b", "dd", "t"), F.xxhash64("i", "l", "d", "b", "dd", "t")).collect()
    types = [T.IntegerType(), T.LongType(), T.DoubleType(), T.BooleanType(), T.DateType(), T.TimestampType()]
    for r, g in zip(rows, got):
        for algo, val, width in (("murmur3", g[0], 32), ("xx", g[1], 64)):
            h = 42
            for v, t in zip(r, types):
                h = hash_value(v, t, h, algo)
            h = h - (1 << width) if h >= (1 << (width - 1)) else h
            assert val == h, (algo, r)
    # -0.0 and 0.0 hash alike
    z = spark.createDataFrame([(0.0,), (-0.0,)], "d double").select(F.hash("d")).collect()
    assert z[0][0] == z[1][0]


def test_math_and_bits(spark):
    r = one(spark, F.conv(F.lit("100"), 2, 10), F.conv(F.lit("-10"), 16, -10), F.bin(F.lit(12)), F.hex(F.lit(17)),
            F.unhex(F.lit("537061726B2053514C")), F.shiftleft(F.lit(21), 1), F.shiftright(F.lit(42), 1),
            F.shiftrightunsigned(F.lit(-42), 1), F.factorial(F.lit(5)), F.bitwise_not(F.lit(0)),
            F.acosh(F.lit(1.0)), F.hex(F.lit("Spark SQL")))
    assert list(r[:6]) == ["4", "-16", "1100", "11", b"Spark SQL", 42]
    assert r[6] == 21 and r[7] == 2147483627 and r[8] == 120 and r[9] == -1 and r[10] == 0.0
    assert r[11] == "537061726B2053514C"
    vals = spark.range(2000).select(F.randn(7).alias("z")).toPandas()["z"].to_numpy()
    assert abs(vals.mean()) < 0.1 and abs(vals.std() - 1) < 0.1


def test_strings(spark):
    r = one(spark, F.ascii("s"), F.base64("s"), F.levenshtein(F.lit("kitten"), F.lit("sitting")),
            F.soundex(F.lit("Miller")), F.soundex(F.lit("Peters")), F.format_number(F.lit(12332.123456), 4),
            F.format_number(F.lit(5), 4), F.format_string("%d %s", F.lit(5), F.lit("hello")),
            F.substring_index(F.lit("a.b.c.d"), ".", 2), F.substring_index(F.lit("a.b.c.d"), ".", -3),
            F.overlay(F.lit("SPARK_SQL"), F.lit("CORE"), 7), F.overlay(F.lit("SPARK_SQL"), F.lit("ANSI "), 7, 0),
            F.bit_length("s"), F.octet_length("s"), F.char_length("s"), F.unbase64(F.lit("U3BhcmsgU1FM")),
            F.decode(F.encode("s", "utf-8"), "utf-8"), F.typeof("s"))
    assert list(r) == [83, "U3Bhcms=", 3, "M460", "P362", "12,332.1235", "5.0000", "5 hello", "a.b", "b.c.d",
                       "SPARK_CORE", "SPARK_ANSI SQL", 40, 5, 5, b"Spark SQL", "Spark", "string"]


def test_null_helpers(spark):
    df = spark.createDataFrame([(1, None, 4), (2, 3, 0)], "a int, b int, c int")
    rows = df.select(F.nvl("b", "a"), F.nvl2("b", "a", "c"), F.nullif("a", F.lit(2)), F.try_divide("a", "c"),
                     F.try_add("a", "c"), F.ifnull("b", F.lit(-1))).collect()
    assert [tuple(r) for r in rows] == [(1, 4, 1, 0.25, 5, -1), (3, 2, None, None, 2, 3)]
    big = spark.createDataFrame([(2 ** 63 - 1, 1)], "a long, b long").select(F.try_add("a", "b")).collect()
    assert big[0][0] is None


def test_collections(spark):
    df = spark.createDataFrame([([1, 2, 3], [1, 3, 5], [[1, 2], [3]])], "a array<int>, b array<int>, n array<array<int>>")
    r = df.select(F.array_except("a", "b"), F.array_intersect("a", "b"), F.array_union("a", "b"),
                  F.arrays_overlap("a", "b"), F.array_position("a", 3), F.array_remove("b", 3),
                  F.array_repeat(F.lit("ab"), 3), F.flatten("n"), F.sequence(F.lit(1), F.lit(5)),
                  F.sequence(F.lit(5), F.lit(1)), F.slice("a", 2, 2), F.array_append("a", 9),
                  F.array_prepend("a", 0), F.array_size("a"), F.cardinality("b"),
                  F.array_sort(F.array(F.lit(3), F.lit(1), F.lit(2))),
                  F.array_compact(F.array(F.lit(1), F.lit(None), F.lit(2)))).collect()[0]
    assert list(r) == [[2], [1, 3], [1, 2, 3, 5], True, 3, [1, 5], ["ab", "ab", "ab"], [1, 2, 3], [1, 2, 3, 4, 5],
                       [5, 4, 3, 2, 1], [2, 3], [1, 2, 3, 9], [0, 1, 2, 3], 3, 3, [1, 2, 3], [1, 2]]
    z = df.select(F.arrays_zip("a", "b").alias("z")).collect()[0].z
    assert [(e.a, e.b) for e in z] == [(1, 1), (2, 3), (3, 5)]
    srt = df.select(F.array_sort("b", lambda x, y: F.when(x < y, 1).when(x > y, -1).otherwise(0))).collect()[0][0]
    assert srt == [5, 3, 1]
    sh = df.select(F.shuffle("a", seed=3)).collect()[0][0]
    assert sorted(sh) == [1, 2, 3]


def test_higher_order(spark):
    df = spark.createDataFrame([([1, 2, 3, 4], 10), ([], 1), (None, 2)], "a array<int>, k int")
    r = df.select(F.transform("a", lambda x: x + 1), F.transform("a", lambda x, i: x * i),
                  F.transform("a", lambda x: x * F.col("k")), F.filter("a", lambda x: x % 2 == 1),
                  F.exists("a", lambda x: x > 3), F.forall("a", lambda x: x > 0),
                  F.aggregate("a", F.lit(0), lambda acc, x: acc + x),
                  F.aggregate("a", F.lit(0), lambda acc, x: acc + x, lambda acc: acc * 10),
                  F.zip_with("a", "a", lambda x, y: x * y)).collect()
    assert list(r[0]) == [[2, 3, 4, 5], [0, 2, 6, 12], [10, 20, 30, 40], [1, 3], True, True, 10, 100, [1, 4, 9, 16]]
    assert list(r[1]) == [[], [], [], [], False, True, 0, 0, []]
    assert list(r[2]) == [None] * 9


def test_maps(spark):
    df = spark.createDataFrame([("a", 1, "b", 2)], "k1 string, v1 int, k2 string, v2 int")
    m = F.create_map("k1", "v1", "k2", "v2")
    r = df.select(m.alias("m"), F.map_keys(m), F.map_values(m), F.map_from_arrays(F.array("k1", "k2"), F.array("v1", "v2")),
                  F.map_filter(m, lambda k, v: v > 1), F.transform_values(m, lambda k, v: v * 10),
                  F.transform_keys(m, lambda k, v: F.upper(k)), F.map_concat(m, F.create_map(F.lit("c"), F.lit(3))),
                  F.element_at(m, "b")).collect()[0]
    assert r[0] == {"a": 1, "b": 2} and r[1] == ["a", "b"] and r[2] == [1, 2] and r[3] == {"a": 1, "b": 2}
    assert r[4] == {"b": 2} and r[5] == {"a": 10, "b": 20} and r[6] == {"A": 1, "B": 2}
    assert r[7] == {"a": 1, "b": 2, "c": 3} and r[8] == 2
    e = df.select(F.map_entries(m).alias("e")).collect()[0].e
    assert [(x.key, x.value) for x in e] == [("a", 1), ("b", 2)]
    ns = df.select(F.named_struct(F.lit("x"), F.col("v1"), F.lit("y"), F.col("k2")).alias("s")).collect()[0].s
    assert ns.x == 1 and ns.y == "b"


def test_json(spark):
    df = spark.createDataFrame([('{"a": 1, "b": 0.8, "c": {"d": [1, 2]}}',), ("not json",)], "j string")
    r = df.select(F.from_json("j", "a INT, b DOUBLE").alias("s"), F.get_json_object("j", "$.c.d[1]"),
                  F.get_json_object("j", "$.c"), F.json_object_keys("j")).collect()
    assert r[0].s.a == 1 and r[0].s.b == 0.8 and r[0][1] == "2" and r[0][2] == '{"d":[1,2]}'
    assert r[0][3] == ["a", "b", "c"]
    assert r[1].s is None and r[1][1] is None
    t = df.select(F.json_tuple("j", "a", "b", "zz")).collect()
    assert [tuple(x) for x in t] == [("1", "0.8", None), (None, None, None)]
    s = spark.createDataFrame([(1, "x", None)], "a int, b string, c double").select(
        F.to_json(F.struct("a", "b", "c"))).collect()[0][0]
    assert s == '{"a":1,"b":"x"}'
    nested = spark.createDataFrame([('[{"x": 1}, {"x": 2}]',)], "j string").select(
        F.from_json("j", "array<struct<x: int>>").alias("v")).collect()[0].v
    assert [e.x for e in nested] == [1, 2]
    assert spark.range(1).select(F.schema_of_json(F.lit('{"a": 1, "b": [1.5]}'))).collect()[0][0] == \
        "STRUCT<a: BIGINT, b: ARRAY<DOUBLE>>"


def test_dates_and_zones(spark):
    df = spark.createDataFrame([(dt.datetime(1997, 2, 28, 10, 30), dt.date(2015, 7, 27), "08/04/2015 12:12")],
                               "t timestamp, d date, s string")
    r = df.select(F.from_utc_timestamp("t", "Asia/Tokyo"), F.to_utc_timestamp("t", "Asia/Tokyo"),
                  F.next_day("d", "Sun"), F.make_date(F.lit(2020), F.lit(6), F.lit(26)),
                  F.to_timestamp("s", "dd/MM/yyyy HH:mm"), F.to_date("s", "dd/MM/yyyy HH:mm"),
                  F.date_format("t", "yyyy-MM-dd'T'HH:mm:ss EEE MMM a"), F.unix_timestamp(F.lit("2015-04-08 12:12:12"),
                                                                               "yyyy-MM-dd HH:mm:ss"),
                  F.from_unixtime(F.lit(1428495132), "dd.MM.yy HH:mm"), F.date_part(F.lit("YEAR"), "t"),
                  F.extract(F.lit("second"), "t"), F.timestamp_seconds(F.lit(1230219000)), F.unix_seconds("t"),
                  F.unix_date("d"), F.window_time(F.struct(F.col("t").alias("start"), F.col("t").alias("end"))),
                  F.make_timestamp(F.lit(2014), F.lit(12), F.lit(28), F.lit(6), F.lit(30), F.lit(45.887))).collect()[0]
    assert r[0] == dt.datetime(1997, 2, 28, 19, 30) and r[1] == dt.datetime(1997, 2, 28, 1, 30)
    assert r[2] == dt.date(2015, 8, 2) and r[3] == dt.date(2020, 6, 26)
    assert r[4] == dt.datetime(2015, 4, 8, 12, 12) and r[5] == dt.date(2015, 4, 8)
    assert r[6] == "1997-02-28T10:30:00 Fri Feb AM"
    assert r[7] == 1428495132 and r[8] == "08.04.15 12:12" and r[9] == 1997 and r[10] == 0.0
    assert r[11] == dt.datetime(2008, 12, 25, 15, 30) and r[12] == 857125800 and r[13] == 16643
    assert r[14] == dt.datetime(1997, 2, 28, 10, 29, 59, 999999)
    assert r[15] == dt.datetime(2014, 12, 28, 6, 30, 45, 887000)
    bad = spark.createDataFrame([("2015-13-45",)], "s string").select(F.to_date("s", "yyyy-MM-dd")).collect()[0][0]
    assert bad is None


def test_inline_and_misc(spark):
    df = spark.createDataFrame([(1, [(1, "a"), (2, "b")]), (2, [])], "id int, xs array<struct<n: int, s: string>>")
    rows = df.select("id", F.inline("xs")).collect()
    assert [tuple(r) for r in rows] == [(1, 1, "a"), (1, 2, "b")]
    rows = df.select("id", F.inline_outer("xs")).collect()
    assert [tuple(r) for r in rows] == [(1, 1, "a"), (1, 2, "b"), (2, None, None)]
    assert df.select(F.spark_partition_id()).collect()[0][0] == 0
    assert F.broadcast(df) is df
    o = spark.createDataFrame([(None,), (2,), (1,)], "x int").orderBy(F.asc_nulls_last("x")).collect()
    assert [r.x for r in o] == [1, 2, None]
    o = spark.createDataFrame([(None,), (2,), (1,)], "x int").orderBy(F.desc_nulls_last("x")).collect()
    assert [r.x for r in o] == [2, 1, None]
    assert spark.range(1).select(F.input_file_name()).collect()[0][0] == ""


def test_grouping_in_rollup_and_cube(spark):
    df = spark.createDataFrame([("a", "x", 1), ("a", "y", 2), ("b", "x", 3)], "g string, h string, v int")
    rows = df.rollup("g", "h").agg(F.sum("v").alias("s"), F.grouping("g").alias("gg"), F.grouping_id().alias("gid")) \
        .orderBy("gid", "g", "h").collect()
    got = [(r.g, r.h, r.s, r.gg, r.gid) for r in rows]
    assert got == [("a", "x", 1, 0, 0), ("a", "y", 2, 0, 0), ("b", "x", 3, 0, 0),
                   ("a", None, 3, 0, 1), ("b", None, 3, 0, 1), (None, None, 6, 1, 3)]
    cube = df.cube("g", "h").agg(F.grouping_id("g", "h").alias("gid"), F.count("*").alias("n")).collect()
    assert sorted({r.gid for r in cube}) == [0, 1, 2, 3]
    with pytest.raises(ValueError):
        df.select(F.grouping("g")).collect()


def test_session_window(spark):
    t0 = dt.datetime(2024, 1, 1, 10, 0)
    m = lambda k: t0 + dt.timedelta(minutes=k)
    rows = [("h1", m(0)), ("h1", m(3)), ("h1", m(7)), ("h1", m(20)), ("h2", m(1)), ("h2", m(30)), ("h2", None)]
    df = spark.createDataFrame(rows, "h string, t timestamp")
    out = df.groupBy("h", F.session_window("t", "5 minutes")).agg(F.count("*").alias("n")).collect()
    got = sorted((r.h, r.session_window.start if r.session_window else None,
                  r.session_window.end if r.session_window else None, r.n) for r in out if r.session_window)
    assert got == [("h1", m(0), m(12), 3), ("h1", m(20), m(25), 1), ("h2", m(1), m(6), 1), ("h2", m(30), m(35), 1)]
