"""JSON round trip of non-finite doubles: Spark writes NaN / Infinity / -Infinity as quoted strings and
reads them back (allowNonNumericNumbers); a null stays a missing field."""
import math

import pandas as pd

from clustermachinelearningforhospitalnetworks_apache_spark_amd.sql import SparkSession
from clustermachinelearningforhospitalnetworks_apache_spark_amd.sql import types as T


def test_json_nan_inf_round_trip(tmp_path):
    spark = SparkSession.builder.master("local[1]").getOrCreate()
    schema = T.StructType([T.StructField("id", T.IntegerType()), T.StructField("v", T.DoubleType())])
    rows = [(1, 1.5), (2, float("nan")), (3, float("inf")), (4, float("-inf")), (5, None)]
    df = spark.createDataFrame(rows, schema)
    path = str(tmp_path / "j")
    df.write.mode("overwrite").json(path)
    text = "".join(open(f).read() for f in sorted((tmp_path / "j").glob("*.json")))
    assert '"v":"NaN"' in text and '"v":"Infinity"' in text and '"v":"-Infinity"' in text
    for back in (spark.read.schema(schema).json(path), spark.read.json(path)):
        got = {r["id"]: r["v"] for r in back.collect()}
        assert got[1] == 1.5 and math.isnan(got[2]) and got[3] == math.inf and got[4] == -math.inf
        assert got[5] is None


def test_json_nan_strings_without_numbers_stay_strings(tmp_path):
    """a column whose present values are only such strings (no JSON number at all) is a
    string column, as Spark infers it; a "NaN" inside an ordinary string value changes nothing."""
    p = tmp_path / "s.json"
    p.write_text('{"a":"NaN","b":1.5,"c":"x \\"NaN\\" y"}\n{"a":"Infinity","b":2.0,"c":"z"}\n{"b":3.0,"c":"w"}\n')
    spark = SparkSession.builder.master("local[1]").getOrCreate()
    df = spark.read.json(str(p))
    types = {f.name: f.dataType for f in df.schema.fields}
    assert isinstance(types["a"], T.StringType), types
    assert isinstance(types["b"], T.DoubleType) and isinstance(types["c"], T.StringType)
    rows = sorted(df.collect(), key=lambda r: r["b"])
    assert [r["a"] for r in rows] == ["NaN", "Infinity", None]
    assert rows[0]["c"] == 'x "NaN" y'


def test_json_all_null_rows_round_trip(tmp_path):
    """Rows whose every field is null are written as {} (Spark omits null fields) and read back as rows of
    nulls under the schema — also when EVERY record is {} (no column at all in the files; found by
    tests/test_properties.py)."""
    spark = SparkSession.builder.master("local[1]").getOrCreate()
    schema = T.StructType([T.StructField("h", T.StringType()), T.StructField("a", T.LongType()),
                           T.StructField("x", T.DoubleType())])
    for rows in ([(None, None, None)], [(None, None, None), (None, None, None)], [(None, None, None), ("p", 2, 0.5)]):
        path = str(tmp_path / f"n{len(rows)}{rows[-1][0]}")
        spark.createDataFrame(rows, schema).write.mode("overwrite").json(path)
        back = spark.read.schema(schema).json(path)
        assert [tuple(r) for r in back.collect()] == rows
