"""Hive-style partitioned writes / partition discovery (parquet, csv, orc) and text / orc formats."""
import os

import pytest

from helpers import session


@pytest.fixture()
def spark(tmp_path):
    return session()


ROWS = [("H0", 2024, 1.5, "a"), ("H1", 2024, 2.5, "b"), ("H0", 2025, 3.5, "c"), (None, 2025, 4.5, "d")]


@pytest.mark.parametrize("fmt", ["parquet", "csv", "orc"])
def test_partition_roundtrip(spark, tmp_path, fmt):
    df = spark.createDataFrame(ROWS, "hid STRING, yr INT, los DOUBLE, note STRING")
    out = str(tmp_path / fmt)
    w = df.write.partitionBy("yr", "hid").mode("overwrite")
    if fmt == "csv":
        w = w.option("header", True)
    w.format(fmt).save(out)
    assert sorted(os.listdir(out)) == ["_SUCCESS", "yr=2024", "yr=2025"]
    assert sorted(os.listdir(os.path.join(out, "yr=2025"))) == ["hid=H0", "hid=__HIVE_DEFAULT_PARTITION__"]
    r = spark.read.format(fmt)
    if fmt == "csv":
        r = r.option("header", True).schema("los DOUBLE, note STRING")
    back = r.load(out)
    assert set(back.columns) == {"los", "note", "yr", "hid"}
    assert dict(back.dtypes)["yr"] == "int" and dict(back.dtypes)["hid"] == "string"
    got = sorted((r.hid or "", r.yr, r.los, r.note) for r in back.collect())
    assert got == sorted((h or "", y, l, n) for h, y, l, n in ROWS)
    # partition pruning by filter on the discovered column
    assert back.filter("yr = 2025").count() == 2


def test_text_format(spark, tmp_path):
    df = spark.createDataFrame([("first line",), ("second",)], "value STRING")
    df.write.text(str(tmp_path / "t"))
    back = spark.read.text(str(tmp_path / "t"))
    assert sorted(r.value for r in back.collect()) == ["first line", "second"]
    with pytest.raises(ValueError):
        spark.createDataFrame([(1, 2)], "a INT, b INT").write.text(str(tmp_path / "t2"))


def test_parquet_strings_dictionary_encoded_on_read(tmp_path, monkeypatch):
    from clustermachinelearningforhospitalnetworks_apache_spark_amd.sql import SparkSession, builder
    from clustermachinelearningforhospitalnetworks_apache_spark_amd.sql.column import DictColumnData
    s = SparkSession.builder.master("local[1]").getOrCreate()
    rows = [([None, "H1", "H2", "H3"][i % 4], i) for i in range(400)]
    s.createDataFrame(rows, "h string, i int").write.mode("overwrite").parquet(str(tmp_path / "p"))
    monkeypatch.setattr(builder, "DICT_MIN_ROWS", 16)
    df = s.read.parquet(str(tmp_path / "p"))
    assert isinstance(df._cols["h"], DictColumnData)
    assert sorted((r.h or "", r.i) for r in df.collect()) == sorted((h or "", i) for h, i in rows)
    assert df.na.drop().count() == 300 and df.groupBy("h").count().count() == 4
