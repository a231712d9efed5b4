"""CSV (native parser) / Parquet / JSON / transactional table IO and the streaming engine
(reference ingest path ref.py:75-118) on the local backend."""
import json
import os
import time

import numpy as np
import pandas as pd
import pytest

from helpers import hospital_frame, hospital_schema, session, write_csv_files
from clustermachinelearningforhospitalnetworks_apache_spark_amd.io import table as tbl
from clustermachinelearningforhospitalnetworks_apache_spark_amd.io.csv import parse_csv_bytes
from clustermachinelearningforhospitalnetworks_apache_spark_amd.sql import functions as F
from clustermachinelearningforhospitalnetworks_apache_spark_amd.sql import types as T


@pytest.fixture()
def spark(tmp_path):
    s = session()
    s.conf.set("spark.sql.warehouse.dir", str(tmp_path / "warehouse"))
    return s


def test_native_csv_parser_types_nulls_quotes():
    data = (b'name,t,i,d,b\n'
            b'"Smith, J",2025-03-31 22:00:05,12,1.5,true\n'
            b'"say ""hi""",2025-03-31T23:59:59.250,,nan?,false\n'
            b'\n'
            b'plain,bad-ts,7,-2e3,TRUE\n'
            b'"multi\nline",2025-01-01,3\n')
    st = T.StructType([T.StructField("name", T.StringType()), T.StructField("t", T.TimestampType()),
                       T.StructField("i", T.IntegerType()), T.StructField("d", T.DoubleType()),
                       T.StructField("b", T.BooleanType())])
    out, n = parse_csv_bytes(data, st, header=True)
    assert n == 4
    names, nv = out["name"]
    assert list(names) == ["Smith, J", 'say "hi"', "plain", "multi\nline"]
    t, tv = out["t"]
    assert tv.tolist() == [True, True, False, True]
    assert t[0] == int(pd.Timestamp("2025-03-31 22:00:05").value // 1000)
    assert t[1] == int(pd.Timestamp("2025-03-31 23:59:59.250").value // 1000)
    i, iv = out["i"]
    assert iv.tolist() == [True, False, True, True] and i[0] == 12 and i[2] == 7
    d, dv = out["d"]
    assert dv.tolist() == [True, False, True, False] and d[2] == -2000.0  # short record -> null
    b, bv = out["b"]
    assert b[:3].tolist() == [True, False, True] and bv.tolist() == [True, True, True, False]


def test_read_csv_with_schema_and_infer(spark, tmp_path):
    pdf = hospital_frame(200)
    write_csv_files(pdf, str(tmp_path / "in"), nfiles=3)
    df = spark.read.option("header", True).schema(hospital_schema()).csv(str(tmp_path / "in"))
    assert df.count() == 200
    got = df.toPandas().sort_values(["event_time", "hospital_id", "length_of_stay"]).reset_index(drop=True)
    want = pdf.sort_values(["event_time", "hospital_id", "length_of_stay"]).reset_index(drop=True)
    np.testing.assert_allclose(got.length_of_stay, want.length_of_stay, rtol=1e-12)
    assert (got.admission_count.values == want.admission_count.values).all()
    inf = spark.read.csv(str(tmp_path / "in"), header=True, inferSchema=True)
    assert dict(inf.dtypes)["admission_count"] == "int"
    assert dict(inf.dtypes)["seasonality_index"] == "double"
    assert dict(inf.dtypes)["event_time"] == "timestamp"


def test_parquet_json_roundtrip(spark, tmp_path):
    df = spark.createDataFrame(hospital_frame(50))
    df.write.mode("overwrite").parquet(str(tmp_path / "p"))
    back = spark.read.parquet(str(tmp_path / "p"))
    assert back.count() == 50 and back.columns == df.columns
    df.write.json(str(tmp_path / "j"))
    assert spark.read.json(str(tmp_path / "j")).count() == 50
    with pytest.raises(FileExistsError):
        df.write.parquet(str(tmp_path / "p"))


def test_transactional_table_append_overwrite(spark, tmp_path):
    df = spark.createDataFrame(hospital_frame(30))
    df.write.saveAsTable("t1")
    df.write.mode("append").saveAsTable("t1")
    assert spark.table("t1").count() == 60
    assert spark.sql("select count(*) as n from t1").collect()[0].n == 60
    df.limit(5).write.mode("overwrite").saveAsTable("t1")
    assert spark.table("t1").count() == 5
    hist = spark.catalog.history("t1")
    assert [h["version"] for h in hist] == [0, 1, 2]
    assert spark.catalog.tableExists("t1")


def _start(spark, src, ckpt, table="hospital_unbounded_table", fn=None, trigger="availableNow"):
    sdf = (spark.readStream.option("header", True).schema(hospital_schema()).csv(src)
           .withWatermark("event_time", "10 minutes").withColumn("ingest_time", F.current_timestamp()))
    w = sdf.writeStream
    if fn is not None:
        w = w.foreachBatch(fn)
    w = w.format("delta").outputMode("append").option("checkpointLocation", ckpt)
    if trigger == "availableNow":
        w = w.trigger(availableNow=True)
    return w.table(table)  # the reference's spelling (ref.py:115)


def test_stream_to_unbounded_table_with_foreach_batch(spark, tmp_path):
    src = str(tmp_path / "incoming")
    pdf = hospital_frame(300)
    write_csv_files(pdf.iloc[:150], src, nfiles=2, prefix="a")
    seen = []

    def ml(batch_df, batch_id):  # the intended per-batch hook (ref.py:91-106)
        seen.append((batch_id, batch_df.count(), "ingest_time" in batch_df.columns))

    q = _start(spark, src, str(tmp_path / "ckpt"), fn=ml)
    assert spark.table("hospital_unbounded_table").count() == 150
    assert seen == [(0, 150, True)]
    # new uploads -> next micro-batch
    write_csv_files(pdf.iloc[150:], src, nfiles=1, prefix="b")
    q2 = _start(spark, src, str(tmp_path / "ckpt"), fn=ml)
    assert spark.table("hospital_unbounded_table").count() == 300
    assert seen[-1][0] == 1 and q2.lastProgress["numInputRows"] == 150
    assert q2.lastProgress["eventTime"]["watermark"] > 0
    # training window over the unbounded table (ref.py:123-128)
    w = spark.sql("SELECT * FROM hospital_unbounded_table WHERE event_time BETWEEN "
                  "'2025-03-31 22:00:00' AND '2025-03-31 23:00:00'").na.drop()
    lo, hi = pd.Timestamp("2025-03-31 22:00:00"), pd.Timestamp("2025-03-31 23:00:00")
    assert w.count() == int(((pdf.event_time >= lo) & (pdf.event_time <= hi)).sum())


def test_stream_restart_is_exactly_once(spark, tmp_path):
    """Crash after the offsets entry (and even after the sink commit) but before the
    checkpoint commit: the restarted query re-plans the SAME batch and the table sink
    skips the already-committed (queryId, batchId) transaction."""
    src, ckpt = str(tmp_path / "in"), str(tmp_path / "ck")
    write_csv_files(hospital_frame(100), src, nfiles=2)
    _start(spark, src, ckpt)
    assert spark.table("hospital_unbounded_table").count() == 100
    # simulate a crash of batch 0 after its sink commit: drop the checkpoint commit
    os.remove(os.path.join(ckpt, "commits", "0"))
    q = _start(spark, src, ckpt)
    assert q.lastProgress["replayed"] is True
    assert spark.table("hospital_unbounded_table").count() == 100  # no duplicates
    # and crash BEFORE the sink commit: remove the table's last version and the commit
    root = spark.catalog._table_path("hospital_unbounded_table")
    last = tbl.versions(root)[-1]
    os.remove(os.path.join(root, "_txn_log", f"{last:020d}.json"))
    os.remove(os.path.join(ckpt, "commits", "0"))
    _start(spark, src, ckpt)
    assert spark.table("hospital_unbounded_table").count() == 100


def test_stream_background_thread_process_all_available(spark, tmp_path):
    src = str(tmp_path / "in")
    write_csv_files(hospital_frame(60), src, nfiles=2)
    q = (spark.readStream.option("header", True).schema(hospital_schema()).csv(src)
         .writeStream.format("memory").queryName("mem").option("checkpointLocation", str(tmp_path / "c"))
         .trigger(processingTime="100 milliseconds").start())
    q.processAllAvailable()
    assert spark.table("mem").count() == 60
    write_csv_files(hospital_frame(40, seed=3), src, nfiles=1, prefix="late")
    q.processAllAvailable()
    assert spark.table("mem").count() == 100
    q.stop()
    assert not q.isActive


def test_table_write_in_parallel_parts_keeps_row_order(spark, tmp_path, monkeypatch):
    """A commit of more rows than CML_TABLE_PART_ROWS writes consecutive row slices as separate part
    files (parallel writer threads); the commit lists them in row order, so the table reads back in the
    frame's order, from the synchronous and the streaming (background) writer alike."""
    monkeypatch.setenv("CML_TABLE_PART_ROWS", "7")
    pdf = hospital_frame(40)
    df = spark.createDataFrame(pdf)
    df.write.saveAsTable("tp")
    root = spark.catalog._table_path("tp")
    files, _, commits = tbl.snapshot(root)
    assert len(commits[0]["add"]) == 6 and all(f.endswith(f"-c{i:03d}.parquet") for i, f in enumerate(files))
    back = spark.table("tp").toPandas()
    assert back.length_of_stay.tolist() == pdf.length_of_stay.tolist()
    pend = tbl.write_frame_async(df, root, "append", "STREAMING UPDATE", {"appId": "q", "version": 0})
    assert pend.finish() == 1
    back = spark.table("tp").toPandas()
    assert back.length_of_stay.tolist() == pdf.length_of_stay.tolist() * 2
