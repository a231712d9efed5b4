"""SQL front end: joins, set operations, CTEs, IN subqueries, GROUP BY expressions and the DDL/DML
statements, checked against sqlite3 (Python's stdlib) running the same queries on the same rows."""
import sqlite3

import pytest

from helpers import session


@pytest.fixture()
def spark(tmp_path):
    s = session()
    s.conf.set("spark.sql.warehouse.dir", str(tmp_path / "wh"))
    return s


ADM = [(1, "H0", 3.0, 10), (2, "H1", 5.5, 20), (3, "H0", 1.0, 10), (4, "H2", 8.0, 30), (5, "H3", 2.0, None)]
HOS = [("H0", "north", 100), ("H1", "south", 80), ("H2", "north", 50), ("H9", "east", 10)]


@pytest.fixture()
def db(spark):
    spark.createDataFrame(ADM, "id INT, hid STRING, los DOUBLE, ward INT").createOrReplaceTempView("adm")
    spark.createDataFrame(HOS, "hid STRING, region STRING, beds INT").createOrReplaceTempView("hos")
    con = sqlite3.connect(":memory:")
    con.execute("CREATE TABLE adm (id INT, hid TEXT, los REAL, ward INT)")
    con.execute("CREATE TABLE hos (hid TEXT, region TEXT, beds INT)")
    con.executemany("INSERT INTO adm VALUES (?,?,?,?)", ADM)
    con.executemany("INSERT INTO hos VALUES (?,?,?)", HOS)
    return con


def _norm(rows):
    out = [tuple(None if v is None else (round(v, 9) if isinstance(v, float) else v) for v in r) for r in rows]
    return sorted(out, key=lambda t: tuple((v is None, str(type(v)), v if v is not None else 0) for v in t))


def _same(spark, con, q, sq=None):
    got = _norm(tuple(r) for r in spark.sql(q).collect())
    want = _norm(tuple(r) for r in con.execute(sq or q).fetchall())
    assert got == want, q


@pytest.mark.parametrize("q", [
    "SELECT a.id, h.region FROM adm a JOIN hos h ON a.hid = h.hid",
    "SELECT a.id, h.region, h.beds FROM adm a LEFT JOIN hos h ON a.hid = h.hid",
    "SELECT a.id, h.hid FROM adm AS a INNER JOIN hos AS h ON h.hid = a.hid AND h.beds > 60",
    "SELECT a.id, h.region FROM adm a, hos h WHERE a.hid = h.hid AND a.los > 2",
    "SELECT h.region, COUNT(*) AS n, SUM(a.los) AS total FROM adm a JOIN hos h ON a.hid = h.hid GROUP BY h.region",
    "SELECT hid, id FROM adm UNION SELECT hid, beds FROM hos",
    "SELECT hid FROM adm UNION ALL SELECT hid FROM hos",
    "SELECT hid FROM adm INTERSECT SELECT hid FROM hos",
    "SELECT hid FROM hos EXCEPT SELECT hid FROM adm",
    "SELECT id FROM adm WHERE hid IN (SELECT hid FROM hos WHERE region = 'north')",
    "SELECT id FROM adm WHERE hid NOT IN (SELECT hid FROM hos WHERE region = 'north')",
    "SELECT hid, COUNT(*) * 2 AS c2, MAX(los) - MIN(los) AS spread FROM adm GROUP BY hid",
    "SELECT ward * 10 AS w10, COUNT(*) AS n FROM adm GROUP BY ward * 10",
    "SELECT hid, AVG(los) AS m FROM adm GROUP BY hid HAVING COUNT(*) > 1",
    "SELECT UPPER(hid) AS u, SUM(los) AS s FROM adm GROUP BY hid",
])
def test_queries_match_sqlite(spark, db, q):
    _same(spark, db, q)


def test_join_variants(spark, db):
    # FULL / RIGHT joins and USING (sqlite in this image may predate RIGHT/FULL JOIN: checked directly)
    full = _norm((r.id, r.region) for r in spark.sql(
        "SELECT a.id, h.region FROM adm a FULL OUTER JOIN hos h ON a.hid = h.hid").collect())
    assert full == _norm([(1, "north"), (2, "south"), (3, "north"), (4, "north"), (5, None), (None, "east")])
    right = spark.sql("SELECT a.id, h.hid FROM adm a RIGHT JOIN hos h ON a.hid = h.hid").collect()
    assert sorted((r.id is None, r.hid) for r in right) == sorted(
        [(False, "H0"), (False, "H0"), (False, "H1"), (False, "H2"), (True, "H9")])
    using = spark.sql("SELECT * FROM adm JOIN hos USING (hid)")
    assert using.columns == ["id", "hid", "los", "ward", "region", "beds"] and using.count() == 4
    semi = sorted(r.id for r in spark.sql("SELECT id FROM adm a LEFT SEMI JOIN hos h ON a.hid = h.hid").collect())
    anti = sorted(r.id for r in spark.sql("SELECT id FROM adm a LEFT ANTI JOIN hos h ON a.hid = h.hid").collect())
    assert semi == [1, 2, 3, 4] and anti == [5]
    star = spark.sql("SELECT a.*, h.region FROM adm a JOIN hos h ON a.hid = h.hid")
    assert star.columns == ["id", "hid", "los", "ward", "region"]
    both = spark.sql("SELECT a.hid, h.hid FROM adm a JOIN hos h ON a.hid = h.hid").collect()
    assert all(r[0] == r[1] for r in both)


def test_cte_and_statements(spark, db):
    q = ("WITH big AS (SELECT hid FROM hos WHERE beds >= 80), "
         "l AS (SELECT * FROM adm WHERE los > 1.5) SELECT l.id FROM l JOIN big ON l.hid = big.hid")
    assert sorted(r.id for r in spark.sql(q).collect()) == [1, 2]
    assert "big" not in spark.catalog._views  # CTE views are scoped to the statement
    spark.sql("CREATE OR REPLACE TEMP VIEW north AS SELECT * FROM hos WHERE region = 'north'")
    assert spark.table("north").count() == 2
    spark.sql("CREATE TABLE stays AS SELECT id, los FROM adm WHERE los > 2")
    assert spark.table("stays").count() == 3
    spark.sql("INSERT INTO stays SELECT id, los FROM adm WHERE los <= 2")
    assert spark.table("stays").count() == 5
    spark.sql("INSERT OVERWRITE TABLE stays SELECT id, los FROM adm WHERE id = 1")
    assert [tuple(r) for r in spark.table("stays").collect()] == [(1, 3.0)]
    names = {r.tableName for r in spark.sql("SHOW TABLES").collect()}
    assert {"stays", "north", "adm"} <= names
    desc = {r.col_name: r.data_type for r in spark.sql("DESCRIBE adm").collect()}
    assert desc == {"id": "int", "hid": "string", "los": "double", "ward": "int"}
    spark.sql("DROP TABLE IF EXISTS stays")
    spark.sql("DROP VIEW north")
    assert not spark.catalog.tableExists("stays") and not spark.catalog.tableExists("north")


def test_sql_grouping_sets_lambdas_and_access():
    from clustermachinelearningforhospitalnetworks_apache_spark_amd.sql import SparkSession
    spark = SparkSession.builder.appName("sqlx").master("local[1]").getOrCreate()
    df = spark.createDataFrame([("a", "x", 1, [1, 2, 3]), ("a", "y", 2, [4]), ("b", "x", 3, [])],
                               "g string, h string, v int, arr array<int>")
    df.createOrReplaceTempView("gs")
    q = spark.sql("SELECT g, h, SUM(v) AS s, GROUPING_ID() AS gid FROM gs GROUP BY ROLLUP(g, h)")
    got = sorted((r.gid, r.g or "", r.h or "", r.s) for r in q.collect())
    assert got == [(0, "a", "x", 1), (0, "a", "y", 2), (0, "b", "x", 3), (1, "a", "", 3), (1, "b", "", 3),
                   (3, "", "", 6)]
    cube = spark.sql("SELECT g, h, COUNT(*) AS n FROM gs GROUP BY CUBE(g, h)").collect()
    assert len(cube) == 3 + 2 + 2 + 1
    sets = spark.sql("SELECT g, h, SUM(v) AS s, grouping(h) AS gh FROM gs GROUP BY GROUPING SETS ((g), (h), ())")
    assert sorted((r.g or "", r.h or "", r.s, r.gh) for r in sets.collect()) == [
        ("", "", 6, 1), ("", "x", 4, 0), ("", "y", 2, 0), ("a", "", 3, 1), ("b", "", 3, 1)]
    wr = spark.sql("SELECT g, SUM(v) FROM gs GROUP BY g WITH ROLLUP")
    assert wr.columns == ["g", "sum(v)"] and sorted((r[0] or "", r[1]) for r in wr.collect()) == [
        ("", 6), ("a", 3), ("b", 3)]
    lam = spark.sql("SELECT transform(arr, x -> x + v) AS a, filter(arr, (x, i) -> i > 0) AS f, "
                    "aggregate(arr, 0, (acc, x) -> acc + x) AS s, exists(arr, x -> x > 3) AS e, "
                    "arr[0] AS first, named_struct('k', v).k AS k FROM gs").collect()
    assert [tuple(r) for r in lam] == [([2, 3, 4], [2, 3], 6, False, 1, 1), ([6], [], 4, True, 4, 2),
                                       ([], [], 0, False, None, 3)]
    nested = spark.sql("SELECT s.g AS sg, s.v FROM (SELECT struct(g, v) AS s FROM gs)").collect()
    assert [tuple(r) for r in nested] == [("a", 1), ("a", 2), ("b", 3)]
    assert spark.sql("SELECT COUNT(*) AS n FROM gs TABLESAMPLE (2 ROWS)").collect()[0].n == 2
    spark.stop()


def test_catalog_metadata_and_sql_udf(tmp_path):
    from clustermachinelearningforhospitalnetworks_apache_spark_amd.sql import SparkSession
    from clustermachinelearningforhospitalnetworks_apache_spark_amd.sql import types as T
    spark = SparkSession.builder.appName("cat").master("local[1]").config(
        "spark.sql.warehouse.dir", str(tmp_path / "wh")).getOrCreate()
    df = spark.createDataFrame([(1, "a"), (2, "b")], "id int, s string")
    df.createOrReplaceTempView("v")
    cols = spark.catalog.listColumns("v")
    assert [(c.name, c.dataType, c.nullable) for c in cols] == [("id", "int", True), ("s", "string", True)]
    assert spark.catalog.getTable("v").isTemporary and spark.catalog.isCached("v")
    assert spark.catalog.databaseExists("default") and spark.catalog.currentCatalog() == "spark_catalog"
    spark.catalog.createTable("empty_t", schema="x double, y string")
    assert spark.table("empty_t").count() == 0 and spark.table("empty_t").columns == ["x", "y"]
    assert spark.catalog.functionExists("sqrt") and not spark.catalog.functionExists("nope_fn")
    spark.udf.register("plus_one", lambda x: x + 1, T.IntegerType())
    assert spark.catalog.functionExists("plus_one")
    assert [r.p for r in spark.sql("SELECT plus_one(id) AS p FROM v").collect()] == [2, 3]
    assert any(f.name == "plus_one" and f.isTemporary for f in spark.catalog.listFunctions())
    spark.stop()


def test_sql_standard_forms_and_intervals():
    import datetime as dt
    from clustermachinelearningforhospitalnetworks_apache_spark_amd.sql import SparkSession
    spark = SparkSession.builder.appName("sqlf").master("local[1]").getOrCreate()
    spark.createDataFrame([(dt.datetime(2024, 1, 31, 3, 4, 5), "  ab  ", dt.date(2024, 1, 31), None)],
                          "t timestamp, s string, d date, n int").createOrReplaceTempView("sf")
    r = spark.sql("SELECT EXTRACT(YEAR FROM t) AS y, t + INTERVAL 1 DAY 2 HOURS AS t2, t - INTERVAL '2' HOUR AS t3, "
                  "d + INTERVAL 1 MONTH AS d2, d - INTERVAL 3 DAYS AS d3, POSITION('b' IN s) AS p, "
                  "TRIM(BOTH ' ' FROM s) AS z1, TRIM(LEADING FROM s) AS z2, SUBSTRING(s FROM 3 FOR 2) AS z3, "
                  "n <=> NULL AS ns FROM sf").collect()[0]
    assert r.y == 2024 and r.t2 == dt.datetime(2024, 2, 1, 5, 4, 5) and r.t3 == dt.datetime(2024, 1, 31, 1, 4, 5)
    assert r.d2 == dt.date(2024, 2, 29) and r.d3 == dt.date(2024, 1, 28) and r.p == 4
    assert (r.z1, r.z2, r.z3) == ("ab", "ab  ", "ab") and r.ns is True
    assert spark.sql("SELECT regr_count(1.0, 2.0) AS rc FROM sf").collect()[0].rc == 1
    spark.stop()
