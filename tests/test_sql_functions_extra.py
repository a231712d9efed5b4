"""UDFs (row-wise and pandas-vectorised) and the string/date helpers commonly used next to the
reference's `when`/`current_timestamp` (ref.py:28)."""
import datetime as dt

import pandas as pd
import pytest

from helpers import session
from clustermachinelearningforhospitalnetworks_apache_spark_amd.sql import functions as F
from clustermachinelearningforhospitalnetworks_apache_spark_amd.sql import types as T


@pytest.fixture()
def df():
    spark = session()
    pdf = pd.DataFrame({"hospital_id": ["H01", "H02", None, "H10"], "los": [3.5, 6.25, 1.0, None],
                        "ts": pd.to_datetime(["2025-03-31 21:05:00", "2025-03-31 22:30:15", "2025-04-01 00:00:00",
                                              "2025-04-02 12:00:00"])})
    return spark.createDataFrame(pdf)


def test_udf_rowwise_and_decorator(df):
    long_stay = F.udf(lambda x: None if x is None else x > 5.0, T.BooleanType())

    @F.udf(returnType="string")
    def tag(h, los):
        return f"{h}:{los}" if h is not None else "unknown"
    out = df.select(long_stay("los").alias("ls"), tag("hospital_id", "los").alias("t")).collect()
    assert [r.ls for r in out] == [False, True, False, False]  # pandas NaN stays NaN (not null), as in Spark
    assert out[0].t == "H01:3.5" and out[2].t == "unknown"


def test_pandas_udf(df):
    @F.pandas_udf("double")
    def doubled(s):
        return s * 2
    got = [r[0] for r in df.select(doubled("los")).collect()]
    assert got[:3] == [7.0, 12.5, 2.0] and (got[3] is None or got[3] != got[3])


def test_string_functions(df):
    r = df.select(F.substring("hospital_id", 2, 2).alias("num"), F.concat_ws("-", "hospital_id", F.lit("x")).alias("c"),
                  F.regexp_replace("hospital_id", r"H(\d+)", "h$1").alias("r"),
                  F.lpad("hospital_id", 5, "0").alias("p")).collect()
    assert [x.num for x in r] == ["01", "02", None, "10"]
    assert r[0].c == "H01-x" and r[2].c == "x"
    assert r[1].r == "h02" and r[0].p == "00H01"


def test_date_functions(df):
    r = df.select(F.date_format("ts", "yyyy-MM-dd HH:mm").alias("f"), F.to_date("ts").alias("d"),
                  F.datediff(F.to_date("ts"), F.to_date(F.lit("2025-03-31"))).alias("dd"),
                  F.date_add(F.to_date("ts"), 1).alias("next"), F.unix_timestamp("ts").alias("u")).collect()
    assert r[0].f == "2025-03-31 21:05"
    assert r[2].d == dt.date(2025, 4, 1) and [x.dd for x in r] == [0, 0, 1, 2]
    assert r[3].next == dt.date(2025, 4, 3)
    assert r[0].u == int(dt.datetime(2025, 3, 31, 21, 5, tzinfo=dt.timezone.utc).timestamp())
    back = df.select(F.from_unixtime(F.unix_timestamp("ts")).alias("s")).collect()
    assert back[1].s == "2025-03-31 22:30:15"
