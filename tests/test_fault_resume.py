"""Failure handling: injected crashes at the worst moments, then restart.

* KMeans killed mid-fit resumes from its iteration checkpoint and ends bitwise where an
  uninterrupted fit ends.
* A streaming query killed after its sink wrote but before the checkpoint commit replays the
  batch without duplicating rows (table txn dedupe); killed right after planning, it re-runs
  the same files.
* A model save killed after its metadata leaves the previous model loadable and no partial
  directory behind.
Also: tracing ranges and the rank-aware logger.
"""
import logging
import os

import numpy as np
import pytest

from helpers import hospital_frame, hospital_schema, session, write_csv_files
from clustermachinelearningforhospitalnetworks_apache_spark_amd.ml.clustering import KMeans, KMeansModel
from clustermachinelearningforhospitalnetworks_apache_spark_amd.ml.feature import VectorAssembler
from clustermachinelearningforhospitalnetworks_apache_spark_amd.sql import functions as F
from clustermachinelearningforhospitalnetworks_apache_spark_amd.utils.fault import InjectedFault
from clustermachinelearningforhospitalnetworks_apache_spark_amd.utils.trace import TRACER


@pytest.fixture()
def spark(tmp_path):
    s = session()
    s.conf.set("spark.sql.warehouse.dir", str(tmp_path / "warehouse"))
    yield s
    for k in ("cml.ml.checkpointDir", "cml.ml.checkpointInterval"):
        s.conf.unset(k)


def _blobs(spark, n=3000, d=6, k=4, seed=0):
    rs = np.random.RandomState(seed)
    c = rs.randn(k, d) * 6
    x = c[rs.randint(0, k, n)] + rs.randn(n, d)
    import pandas as pd
    df = spark.createDataFrame(pd.DataFrame(x, columns=[f"f{i}" for i in range(d)]))
    return VectorAssembler(inputCols=[f"f{i}" for i in range(d)], outputCol="features").transform(df)


def test_kmeans_resumes_from_checkpoint(spark, tmp_path, monkeypatch):
    df = _blobs(spark)
    km = KMeans(k=4, seed=3, maxIter=12, tol=0.0)
    want = np.stack(km.fit(df).clusterCenters())
    spark.conf.set("cml.ml.checkpointDir", str(tmp_path / "ck"))
    spark.conf.set("cml.ml.checkpointInterval", "2")
    monkeypatch.setenv("CML_FAULT", "kmeans.iteration=7")
    with pytest.raises(InjectedFault):
        km.fit(df)
    saved = os.listdir(tmp_path / "ck")
    assert saved == [f"kmeans-{km.uid}"]
    monkeypatch.delenv("CML_FAULT")
    from clustermachinelearningforhospitalnetworks_apache_spark_amd.models import kmeans as engine_mod
    starts = []
    orig = engine_mod.LloydEngine.fit

    def spy(self, max_iter, tol, start_iter=0, on_iter=None):
        starts.append(start_iter)
        return orig(self, max_iter, tol, start_iter=start_iter, on_iter=on_iter)

    monkeypatch.setattr(engine_mod.LloydEngine, "fit", spy)
    model = km.fit(df)
    assert starts == [6]  # last checkpoint before the crash at iteration 7
    np.testing.assert_array_equal(np.stack(model.clusterCenters()), want)
    assert model.summary.numIter == 12
    assert os.listdir(tmp_path / "ck") == []  # cleared after a completed fit


def _start(spark, src, ckpt):
    sdf = (spark.readStream.option("header", True).schema(hospital_schema()).csv(src)
           .withColumn("ingest_time", F.current_timestamp()))
    return (sdf.writeStream.format("delta").outputMode("append").option("checkpointLocation", ckpt)
            .trigger(availableNow=True).toTable("t_fault"))


def test_stream_crash_before_commit_is_exactly_once(spark, tmp_path, monkeypatch):
    src, ck = str(tmp_path / "in"), str(tmp_path / "ck")
    pdf = hospital_frame(200)
    write_csv_files(pdf.iloc[:120], src, nfiles=2, prefix="a")
    _start(spark, src, ck)
    write_csv_files(pdf.iloc[120:], src, nfiles=1, prefix="b")
    monkeypatch.setenv("CML_FAULT", "stream.before_commit=1")
    with pytest.raises(InjectedFault):
        _start(spark, src, ck)
    assert spark.table("t_fault").count() == 200          # batch 1 reached the sink ...
    assert not os.path.exists(os.path.join(ck, "commits", "1"))  # ... but never committed
    monkeypatch.delenv("CML_FAULT")
    q = _start(spark, src, ck)
    assert q.lastProgress["replayed"] is True and q.lastProgress["batchId"] == 1
    assert spark.table("t_fault").count() == 200          # replay did not duplicate


def test_stream_crash_after_offsets_replays_same_files(spark, tmp_path, monkeypatch):
    src, ck = str(tmp_path / "in"), str(tmp_path / "ck")
    write_csv_files(hospital_frame(90), src, nfiles=3)
    monkeypatch.setenv("CML_FAULT", "stream.after_offsets=0")
    with pytest.raises(InjectedFault):
        _start(spark, src, ck)
    assert os.path.exists(os.path.join(ck, "offsets", "0"))
    monkeypatch.delenv("CML_FAULT")
    # a late upload must NOT join the replayed batch 0: it becomes batch 1
    write_csv_files(hospital_frame(30, seed=5), src, nfiles=1, prefix="late")
    q = _start(spark, src, ck)
    progress = {p["batchId"]: p for p in q.recentProgress}
    assert progress[0]["replayed"] is True and progress[0]["numInputRows"] == 90
    assert progress[1]["numInputRows"] == 30
    assert spark.table("t_fault").count() == 120


def test_model_save_crash_keeps_previous_model(spark, tmp_path, monkeypatch):
    df = _blobs(spark, n=500)
    path = str(tmp_path / "model")
    m1 = KMeans(k=2, seed=1).fit(df)
    m1.write().overwrite().save(path)
    m2 = KMeans(k=3, seed=1).fit(df)
    monkeypatch.setenv("CML_FAULT", "ml.save")
    with pytest.raises(InjectedFault):
        m2.write().overwrite().save(path)
    monkeypatch.delenv("CML_FAULT")
    back = KMeansModel.load(path)
    assert len(back.clusterCenters()) == 2
    assert sorted(os.listdir(tmp_path)) == ["model"]  # no temp/old directories left


def test_trace_ranges_and_rank_logger(spark, capsys):
    TRACER.reset()
    TRACER.enable(sync=False)
    try:
        KMeans(k=2, seed=1, maxIter=3).fit(_blobs(spark, n=400))
    finally:
        TRACER.disable()
    s = TRACER.summary()
    assert s["KMeans.fit"]["count"] == 1 and s["kmeans.step"]["count"] >= 1
    assert "VectorAssembler.transform" in s
    assert "KMeans.fit" in TRACER.report()
    from clustermachinelearningforhospitalnetworks_apache_spark_amd.utils.log import get_logger
    lg = get_logger("test")
    lg.setLevel(logging.INFO)
    lg.info("hello from rank zero")
    assert "[rank 0/1] cml.test INFO: hello from rank zero" in capsys.readouterr().err
