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
    assert len(saved) == 1 and saved[0].startswith("kmeans-")
    assert sorted(os.listdir(tmp_path / "ck" / saved[0])) == ["LATEST", "v-00000004", "v-00000006"]
    monkeypatch.delenv("CML_FAULT")
    # a restarted process builds a NEW estimator (new uid): the key-derived name still finds it
    km = KMeans(k=4, seed=3, maxIter=12, tol=0.0)
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


def test_checkpoint_survives_crash_between_renames(tmp_path):
    """A writer killed at any point of save() leaves a loadable checkpoint (the old
    two-rename scheme left none between its renames)."""
    from clustermachinelearningforhospitalnetworks_apache_spark_amd.utils import checkpoint as ck
    d = str(tmp_path)
    name = ck.name_for("kmeans", "key")
    assert name == ck.name_for("kmeans", "key") and name != ck.name_for("kmeans", "other")
    ck.save(d, name, "key", 4, {"centers": np.ones((2, 3))})
    root = tmp_path / name
    # crash after the new version was renamed into place but before LATEST moved
    os.makedirs(root / "v-00000006.tmp-999")
    (root / "v-00000006.tmp-999" / "centers.npy").write_bytes(b"partial")
    it, arrs = ck.load(d, name, "key")
    assert it == 4 and arrs["centers"].shape == (2, 3)
    ck.save(d, name, "key", 6, {"centers": np.zeros((2, 3))})
    # the new version and the one before it are kept; crashed writers' leftovers are gone
    assert sorted(os.listdir(root)) == ["LATEST", "v-00000004", "v-00000006"]
    # the same iteration saved again (a resumed fit) lands under a fresh name: the old copy is never
    # removed before the new one is complete and LATEST names it
    ck.save(d, name, "key", 6, {"centers": np.full((2, 3), 7.0)})
    assert sorted(os.listdir(root)) == ["LATEST", "v-00000006", "v-00000006-1"]
    assert (root / "LATEST").read_text().strip() == "v-00000006-1"
    assert float(ck.load(d, name, "key")[1]["centers"][0, 0]) == 7.0
    # LATEST lost or torn: the newest complete version is found by scanning
    (root / "LATEST").write_text("v-000")
    assert ck.load(d, name, "key")[0] == 6
    os.remove(root / "LATEST")
    assert ck.load(d, name, "key")[0] == 6
    assert ck.load(d, name, "different-fit") is None


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


def test_model_save_crash_between_renames_recovers(spark, tmp_path):
    """A writer that died after moving the old model aside but before renaming the new one into
    place: load() promotes the complete new model."""
    df = _blobs(spark, n=500)
    path = str(tmp_path / "model")
    KMeans(k=2, seed=1).fit(df).write().overwrite().save(path)
    KMeans(k=3, seed=1).fit(df).write().overwrite().save(str(tmp_path / "new"))
    dead = 2 ** 22 + 12345  # above pid_max on this box: never a live process
    os.replace(path, str(tmp_path / f".model.old-{dead}"))
    os.replace(str(tmp_path / "new"), str(tmp_path / f".model.tmp-{dead}"))
    back = KMeansModel.load(path)
    assert len(back.clusterCenters()) == 3
    assert sorted(os.listdir(tmp_path)) == ["model"]
    # only the old copy survived (the crash hit before the new one was complete): it is restored
    os.replace(path, str(tmp_path / f".model.old-{dead}"))
    assert len(KMeansModel.load(path).clusterCenters()) == 3
    assert sorted(os.listdir(tmp_path)) == ["model"]


def test_stream_crash_between_plan_writes_loses_nothing(spark, tmp_path, monkeypatch):
    """Killed after offsets/<bid> but before sources/0/<bid>: the restart replays
    the batch from its offsets entry; no file is hidden or read twice."""
    src, ck = str(tmp_path / "in"), str(tmp_path / "ck")
    write_csv_files(hospital_frame(90), src, nfiles=3)
    monkeypatch.setenv("CML_FAULT", "stream.between_plan_writes=0")
    with pytest.raises(InjectedFault):
        _start(spark, src, ck)
    assert os.path.exists(os.path.join(ck, "offsets", "0"))
    assert not os.path.exists(os.path.join(ck, "sources", "0", "0"))
    monkeypatch.delenv("CML_FAULT")
    write_csv_files(hospital_frame(30, seed=5), src, nfiles=1, prefix="late")
    q = _start(spark, src, ck)
    progress = {p["batchId"]: p for p in q.recentProgress}
    assert progress[0]["replayed"] is True and progress[0]["numInputRows"] == 90
    assert progress[1]["numInputRows"] == 30
    assert spark.table("t_fault").count() == 120
    assert os.path.exists(os.path.join(ck, "sources", "0", "0"))


def test_stream_restart_restores_watermark(spark, tmp_path):
    src, ck = str(tmp_path / "in"), str(tmp_path / "ck")
    write_csv_files(hospital_frame(60), src, nfiles=1)

    def start():
        sdf = (spark.readStream.option("header", True).schema(hospital_schema()).csv(src)
               .withWatermark("event_time", "10 minutes"))
        return (sdf.writeStream.format("delta").outputMode("append").option("checkpointLocation", ck)
                .trigger(availableNow=True).toTable("t_wm"))

    wm = start().lastProgress["eventTime"]["watermark"]
    assert wm > 0
    q = start()  # nothing new to read: the restarted query still reports the committed watermark
    assert q._watermark_ms == wm


def _labelled(spark, n=2500, d=5, seed=1, classes=2):
    import pandas as pd
    rs = np.random.RandomState(seed)
    X = rs.randn(n, d) * (1 + np.arange(d))
    if classes == 2:
        y = (X @ rs.randn(d) + rs.randn(n) > 0).astype(float)
    else:
        y = np.argmax(X[:, :classes] + rs.randn(n, classes), 1).astype(float)
    pdf = pd.DataFrame(X, columns=[f"f{i}" for i in range(d)])
    pdf["label"] = y
    pdf["y"] = X @ np.arange(1, d + 1) + rs.randn(n)
    df = spark.createDataFrame(pdf)
    return VectorAssembler(inputCols=[f"f{i}" for i in range(d)], outputCol="features").transform(df)


def _kill_and_resume(spark, tmp_path, monkeypatch, make, fault, prefix, read):
    """Fit uninterrupted; fit with checkpoints and a crash at ``fault``; refit (new estimator): equal."""
    df = make[0]
    want = read(make[1]().fit(df))
    spark.conf.set("cml.ml.checkpointDir", str(tmp_path / "ck"))
    spark.conf.set("cml.ml.checkpointInterval", "2")
    monkeypatch.setenv("CML_FAULT", fault)
    with pytest.raises(InjectedFault):
        make[1]().fit(df)
    saved = os.listdir(tmp_path / "ck")
    assert len(saved) == 1 and saved[0].startswith(prefix), saved
    assert any(v.startswith("v-") for v in os.listdir(tmp_path / "ck" / saved[0]))
    monkeypatch.delenv("CML_FAULT")
    got = read(make[1]().fit(df))
    assert os.listdir(tmp_path / "ck") == []
    return want, got


@pytest.mark.parametrize("classes,reg,en", [(2, 0.0, 0.0), (2, 0.05, 0.5), (3, 0.01, 0.0)])
def test_logreg_resumes_from_lbfgs_checkpoint(spark, tmp_path, monkeypatch, classes, reg, en):
    from clustermachinelearningforhospitalnetworks_apache_spark_amd.ml.classification import LogisticRegression
    from clustermachinelearningforhospitalnetworks_apache_spark_amd.models import optim
    df = _labelled(spark, classes=classes)
    starts = []
    orig = optim.lbfgs

    def spy(*a, **kw):
        starts.append(None if kw.get("state") is None else kw["state"]["it"])
        return orig(*a, **kw)

    from clustermachinelearningforhospitalnetworks_apache_spark_amd.ml import classification as C
    monkeypatch.setattr(C, "lbfgs", spy)
    mk = lambda: LogisticRegression(maxIter=40, tol=1e-12, regParam=reg, elasticNetParam=en)  # noqa: E731
    read = lambda m: (m.coefficientMatrix.toArray(), m.interceptVector.toArray(), m.summary.objectiveHistory)  # noqa: E731
    want, got = _kill_and_resume(spark, tmp_path, monkeypatch, (df, mk), "logreg.iteration=7", "logreg-", read)
    assert starts[-1] == 6  # resumed from the checkpoint of iteration 6
    np.testing.assert_array_equal(got[0], want[0])
    np.testing.assert_array_equal(got[1], want[1])
    assert got[2] == want[2]


def test_forest_resumes_from_level_checkpoint(spark, tmp_path, monkeypatch):
    from clustermachinelearningforhospitalnetworks_apache_spark_amd.ml.regression import RandomForestRegressor
    df = _labelled(spark)
    mk = lambda: RandomForestRegressor(labelCol="y", numTrees=6, maxDepth=5, seed=4)  # noqa: E731
    read = lambda m: (m.featureImportances.toArray(), [t.toDebugString.split("\n", 1)[1] for t in m.trees])  # noqa: E731
    want, got = _kill_and_resume(spark, tmp_path, monkeypatch, (df, mk), "forest.level=3", "forest-", read)
    np.testing.assert_array_equal(got[0], want[0])
    assert got[1] == want[1]


def test_gbt_resumes_from_tree_checkpoint(spark, tmp_path, monkeypatch):
    from clustermachinelearningforhospitalnetworks_apache_spark_amd.ml.regression import GBTRegressor
    df = _labelled(spark)
    mk = lambda: GBTRegressor(labelCol="y", maxIter=9, maxDepth=3, seed=2)  # noqa: E731
    read = lambda m: (m.featureImportances.toArray(), [t.toDebugString.split("\n", 1)[1] for t in m.trees], m.treeWeights)  # noqa: E731
    want, got = _kill_and_resume(spark, tmp_path, monkeypatch, (df, mk), "forest.tree=5", "gbt-", read)
    np.testing.assert_array_equal(got[0], want[0])
    assert got[1] == want[1] and list(got[2]) == list(want[2])
