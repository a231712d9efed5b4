"""Estimators vs float64 numpy / sklearn oracles, Spark model format, pipelines (local backend)."""
import json
import os

import numpy as np
import pandas as pd
import pyarrow.parquet as pq
import pytest

from helpers import hospital_frame, session
from clustermachinelearningforhospitalnetworks_apache_spark_amd.ml import Pipeline, PipelineModel
from clustermachinelearningforhospitalnetworks_apache_spark_amd.ml import util as U
from clustermachinelearningforhospitalnetworks_apache_spark_amd.ml.classification import (
    DecisionTreeClassifier, LogisticRegression, LogisticRegressionModel, RandomForestClassificationModel,
    RandomForestClassifier)
from clustermachinelearningforhospitalnetworks_apache_spark_amd.ml.clustering import KMeans, KMeansModel
from clustermachinelearningforhospitalnetworks_apache_spark_amd.ml.evaluation import (
    BinaryClassificationEvaluator, ClusteringEvaluator, MulticlassClassificationEvaluator, RegressionEvaluator)
from clustermachinelearningforhospitalnetworks_apache_spark_amd.ml.feature import (
    Binarizer, MinMaxScaler, StandardScaler, StandardScalerModel, StringIndexer, VectorAssembler)
from clustermachinelearningforhospitalnetworks_apache_spark_amd.ml.regression import (
    DecisionTreeRegressionModel, DecisionTreeRegressor, LinearRegression, LinearRegressionModel,
    RandomForestRegressor)
from clustermachinelearningforhospitalnetworks_apache_spark_amd.sql import functions as F

FEATS = ["admission_count", "current_occupancy", "emergency_visits", "seasonality_index"]


@pytest.fixture(scope="module")
def spark():
    return session()


@pytest.fixture(scope="module")
def hosp(spark):
    pdf = hospital_frame(1500, seed=5)
    df = spark.createDataFrame(pdf)
    fd = VectorAssembler(inputCols=FEATS, outputCol="features").transform(df)
    return pdf, fd


def test_vector_assembler_handle_invalid(spark):
    df = spark.createDataFrame([(1.0, 2.0), (None, 3.0), (float("nan"), 1.0)], "a DOUBLE, b DOUBLE")
    va = VectorAssembler(inputCols=["a", "b"], outputCol="f")
    with pytest.raises(ValueError):
        va.transform(df)
    assert va.setHandleInvalid("skip").transform(df).count() == 1
    kept = VectorAssembler(inputCols=["a", "b"], outputCol="f", handleInvalid="keep").transform(df).collect()
    assert np.isnan(kept[1].f[0]) and kept[0].f.toArray().tolist() == [1.0, 2.0]


def test_linear_regression_matches_lstsq(hosp):
    pdf, fd = hosp
    m = LinearRegression(featuresCol="features", labelCol="length_of_stay").fit(fd)
    A = np.c_[pdf[FEATS].values.astype(float), np.ones(len(pdf))]
    sol = np.linalg.lstsq(A, pdf.length_of_stay.values, rcond=None)[0]
    np.testing.assert_allclose(m.coefficients.toArray(), sol[:4], rtol=1e-8, atol=1e-10)
    assert abs(m.intercept - sol[4]) < 1e-8
    pred = m.transform(fd)
    rmse = RegressionEvaluator(labelCol="length_of_stay", metricName="rmse").evaluate(pred)
    want = np.sqrt(np.mean((A @ sol - pdf.length_of_stay.values) ** 2))
    assert abs(rmse - want) < 1e-9
    s = m.summary
    assert abs(s.r2 - (1 - np.sum((A @ sol - pdf.length_of_stay) ** 2) /
                       np.sum((pdf.length_of_stay - pdf.length_of_stay.mean()) ** 2))) < 1e-9
    assert len(s.pValues) == 5 and all(0 <= p <= 1 for p in s.pValues)


def test_ridge_and_lasso(hosp):
    pdf, fd = hosp
    X = pdf[FEATS].values.astype(float)
    y = pdf.length_of_stay.values
    lam = 0.1
    m = LinearRegression(featuresCol="features", labelCol="length_of_stay", regParam=lam).fit(fd)
    # closed form in the standardized space (features and label scaled by unbiased std)
    mx, my = X.mean(0), y.mean()
    sx, sy = X.std(0, ddof=1), y.std(ddof=1)
    Z = (X - mx) / sx
    t = (y - my) / sy
    n = len(y)
    # Spark's effectiveRegParam = regParam / std(label) in the label-standardized space
    beta = np.linalg.solve(Z.T @ Z / n + lam / sy * np.eye(4), Z.T @ t / n)
    np.testing.assert_allclose(m.coefficients.toArray(), beta * sy / sx, rtol=1e-6)
    l1 = LinearRegression(featuresCol="features", labelCol="length_of_stay", regParam=0.5,
                          elasticNetParam=1.0).fit(fd)
    assert (np.abs(l1.coefficients.toArray()) < np.abs(m.coefficients.toArray()) + 1e-12).all()


def test_standard_scaler_unbiased(hosp):
    pdf, fd = hosp
    m = StandardScaler(inputCol="features", outputCol="s", withMean=True).fit(fd)
    X = pdf[FEATS].values.astype(float)
    np.testing.assert_allclose(m.std.toArray(), X.std(0, ddof=1), rtol=1e-10)
    np.testing.assert_allclose(m.mean.toArray(), X.mean(0), rtol=1e-10)
    z = np.stack([r.s.toArray() for r in m.transform(fd).select("s").collect()])
    np.testing.assert_allclose(z, (X - X.mean(0)) / X.std(0, ddof=1), rtol=1e-9, atol=1e-12)
    # default withMean=False: only scaling
    m2 = StandardScaler(inputCol="features", outputCol="s").fit(fd)
    z2 = np.stack([r.s.toArray() for r in m2.transform(fd).select("s").collect()])
    np.testing.assert_allclose(z2, X / X.std(0, ddof=1), rtol=1e-9)


def test_logistic_regression_matches_sklearn(hosp):
    from sklearn.linear_model import LogisticRegression as SkLR
    pdf, fd = hosp
    d = fd.withColumn("label", F.when(F.col("length_of_stay") > 5.0, 1).otherwise(0))
    m = LogisticRegression(maxIter=200, tol=1e-10).fit(d)
    X = pdf[FEATS].values.astype(float)
    y = (pdf.length_of_stay.values > 5.0).astype(int)
    sk = SkLR(penalty=None, max_iter=5000, tol=1e-12).fit(X, y)
    np.testing.assert_allclose(m.coefficients.toArray(), sk.coef_[0], rtol=2e-3, atol=2e-4)
    assert abs(m.intercept - sk.intercept_[0]) < 5e-3 * max(1, abs(sk.intercept_[0]))
    pred = m.transform(d)
    acc = MulticlassClassificationEvaluator(metricName="accuracy").evaluate(pred)
    assert abs(acc - sk.score(X, y)) < 0.01
    assert m.summary.totalIterations > 0 and m.summary.objectiveHistory[-1] < m.summary.objectiveHistory[0]
    auc = BinaryClassificationEvaluator().evaluate(pred)
    from sklearn.metrics import roc_auc_score
    assert abs(auc - roc_auc_score(y, sk.decision_function(X))) < 1e-3


def test_logistic_sgd_and_multinomial(spark):
    rs = np.random.RandomState(0)
    X = rs.randn(3000, 3)
    w = np.array([1.5, -2.0, 0.5])
    y = (X @ w + 0.3 + rs.randn(3000) * 0.3 > 0).astype(float)
    df = VectorAssembler(inputCols=["a", "b", "c"], outputCol="features").transform(
        spark.createDataFrame(pd.DataFrame({"a": X[:, 0], "b": X[:, 1], "c": X[:, 2], "label": y})))
    sgd = LogisticRegression(solver="sgd", maxIter=30, stepSize=0.5, batchSize=256).fit(df)
    lb = LogisticRegression().fit(df)
    cos = np.dot(sgd.coefficients.toArray(), lb.coefficients.toArray()) / (
        np.linalg.norm(sgd.coefficients.toArray()) * np.linalg.norm(lb.coefficients.toArray()))
    assert cos > 0.99
    y3 = np.digitize(X @ w, [-1.0, 1.0])
    df3 = VectorAssembler(inputCols=["a", "b", "c"], outputCol="features").transform(
        spark.createDataFrame(pd.DataFrame({"a": X[:, 0], "b": X[:, 1], "c": X[:, 2], "label": y3.astype(float)})))
    mm = LogisticRegression(maxIter=200).fit(df3)
    assert mm.numClasses == 3 and mm.coefficientMatrix.toArray().shape == (3, 3)
    acc = MulticlassClassificationEvaluator(metricName="accuracy").evaluate(mm.transform(df3))
    assert acc > 0.9


def test_trees_regression_and_importances(hosp):
    pdf, fd = hosp
    dt = DecisionTreeRegressor(featuresCol="features", labelCol="length_of_stay").fit(fd)
    assert dt.depth <= 5 and dt.numNodes <= 63
    imp = dt.featureImportances.toArray()
    assert abs(imp.sum() - 1.0) < 1e-12 and (imp >= 0).all()
    rmse_dt = RegressionEvaluator(labelCol="length_of_stay").evaluate(dt.transform(fd))
    rf = RandomForestRegressor(featuresCol="features", labelCol="length_of_stay").fit(fd)
    assert len(rf.trees) == 20
    rmse_rf = RegressionEvaluator(labelCol="length_of_stay").evaluate(rf.transform(fd))
    std = pdf.length_of_stay.std()
    assert rmse_dt < std and rmse_rf < std
    # deterministic for a fixed seed
    rf2 = RandomForestRegressor(featuresCol="features", labelCol="length_of_stay").fit(fd)
    np.testing.assert_array_equal(rf.featureImportances.toArray(), rf2.featureImportances.toArray())


def test_tree_perfect_split_and_spark_split_rule(spark):
    # one feature, label = x > 3.5 -> a single split at the midpoint 3.5 (Spark: midpoint of distinct values)
    df = spark.createDataFrame(pd.DataFrame({"x": np.arange(8.0), "label": (np.arange(8) > 3.5).astype(float)}))
    f = VectorAssembler(inputCols=["x"], outputCol="features").transform(df)
    m = DecisionTreeClassifier().fit(f)
    root = m._trees[0]
    assert root.feature == 0 and root.threshold == 3.5 and root.left.is_leaf and root.right.is_leaf
    acc = MulticlassClassificationEvaluator(metricName="accuracy").evaluate(m.transform(f))
    assert acc == 1.0
    from clustermachinelearningforhospitalnetworks_apache_spark_amd.models.trees import continuous_splits
    s = continuous_splits(np.repeat(np.arange(100.0), 3), 31)
    assert len(s) <= 31 and np.all(np.diff(s) > 0)


def test_continuous_splits_match_value_walk():
    """Binary-search split finding == Spark's value-by-value walk (kept as _continuous_splits_loop)."""
    from clustermachinelearningforhospitalnetworks_apache_spark_amd.models.trees import (
        _continuous_splits_loop, continuous_splits)
    rs = np.random.RandomState(7)
    cases = [np.repeat(np.arange(100.0), 3), rs.randn(10000), np.round(rs.exponential(3.0, 20000), 1),
             rs.randint(0, 40, 5000).astype(float), np.concatenate([np.zeros(9000), rs.randn(1000)]),
             rs.zipf(1.5, 8000).astype(float), np.array([1.0]), np.array([2.0, 2.0, 3.0])]
    for v in cases:
        for ns in (1, 3, 7, 31, 63, 127):
            np.testing.assert_array_equal(continuous_splits(v, ns), _continuous_splits_loop(v, ns))


def test_classifiers_on_hospital_binary_label(hosp):
    pdf, fd = hosp
    d = fd.withColumn("LOS_binary", F.when(F.col("length_of_stay") > 5.0, 1).otherwise(0))
    tr, te = d.randomSplit([0.7, 0.3], seed=42)
    ev = MulticlassClassificationEvaluator(labelCol="LOS_binary", predictionCol="prediction", metricName="accuracy")
    for est in (DecisionTreeClassifier(featuresCol="features", labelCol="LOS_binary"),
                RandomForestClassifier(featuresCol="features", labelCol="LOS_binary")):
        m = est.fit(tr)
        out = m.transform(te)
        assert {"rawPrediction", "probability", "prediction"} <= set(out.columns)
        assert ev.evaluate(out) > 0.75


def test_evaluators_match_sklearn(spark):
    from sklearn import metrics as M
    rs = np.random.RandomState(1)
    y = rs.randint(0, 3, 500).astype(float)
    p = np.where(rs.rand(500) < 0.8, y, rs.randint(0, 3, 500)).astype(float)
    df = spark.createDataFrame(pd.DataFrame({"label": y, "prediction": p}))
    ev = MulticlassClassificationEvaluator()
    assert abs(ev.evaluate(df) - M.f1_score(y, p, average="weighted")) < 1e-12
    assert abs(ev.setMetricName("accuracy").evaluate(df) - M.accuracy_score(y, p)) < 1e-12
    assert abs(ev.setMetricName("weightedPrecision").evaluate(df) -
               M.precision_score(y, p, average="weighted")) < 1e-12
    r = RegressionEvaluator(metricName="mae")
    yy = rs.randn(200)
    pp = yy + rs.randn(200) * 0.1
    df2 = spark.createDataFrame(pd.DataFrame({"label": yy, "prediction": pp}))
    assert abs(r.evaluate(df2) - M.mean_absolute_error(yy, pp)) < 1e-12
    assert abs(r.setMetricName("r2").evaluate(df2) - M.r2_score(yy, pp)) < 1e-12


def test_kmeans_estimator_and_silhouette(spark):
    rs = np.random.RandomState(2)
    true = rs.randn(4, 5) * 8
    X = true[rs.randint(0, 4, 2000)] + rs.randn(2000, 5)
    df = VectorAssembler(inputCols=[f"c{i}" for i in range(5)], outputCol="features").transform(
        spark.createDataFrame(pd.DataFrame(X, columns=[f"c{i}" for i in range(5)])))
    m = KMeans(k=4, seed=3).fit(df)
    c = np.stack(m.clusterCenters())
    dmin = np.sqrt(((true[:, None] - c[None]) ** 2).sum(2)).min(1)
    assert dmin.max() < 0.3
    assert sum(m.summary.clusterSizes) == 2000 and m.summary.k == 4
    sil = ClusteringEvaluator().evaluate(m.transform(df))
    from sklearn.metrics import silhouette_score
    lab = np.array([r.prediction for r in m.transform(df).select("prediction").collect()])
    assert abs(sil - silhouette_score(X, lab, metric="sqeuclidean")) < 0.05
    assert abs(m.computeCost(df) - ((X - c[lab]) ** 2).sum()) < 1e-6 * ((X - c[lab]) ** 2).sum()


def test_spark_model_format_layout(hosp, tmp_path):
    pdf, fd = hosp
    lr = LinearRegression(featuresCol="features", labelCol="length_of_stay").fit(fd)
    p = str(tmp_path / "lr")
    lr.write().overwrite().save(p)  # ref.py:241
    md = json.loads(open(os.path.join(p, "metadata", "part-00000")).readline())
    assert md["class"] == "org.apache.spark.ml.regression.LinearRegressionModel"
    assert set(md) >= {"class", "timestamp", "sparkVersion", "uid", "paramMap", "defaultParamMap"}
    assert md["paramMap"]["labelCol"] == "length_of_stay" and md["defaultParamMap"]["maxIter"] == 100
    assert os.path.exists(os.path.join(p, "metadata", "_SUCCESS"))
    data = pq.read_table(os.path.join(p, "data"))
    assert data.schema.names == ["intercept", "coefficients", "scale"]
    assert data.schema.field("coefficients").type.names == ["type", "size", "indices", "values"]
    with pytest.raises(FileExistsError):
        lr.save(p)  # plain save refuses an existing path (ref.py:103 semantics)
    back = LinearRegressionModel.load(p)
    np.testing.assert_array_equal(back.coefficients.toArray(), lr.coefficients.toArray())
    assert U.load(p).intercept == lr.intercept
    rf = RandomForestClassifier(featuresCol="features", labelCol="lab", numTrees=3).fit(
        fd.withColumn("lab", F.when(F.col("length_of_stay") > 5, 1).otherwise(0)))
    q = str(tmp_path / "rf")
    rf.write().overwrite().save(q)
    t = pq.read_table(os.path.join(q, "data"))
    assert t.schema.names == ["treeID", "nodeData"]
    assert [f.name for f in t.schema.field("nodeData").type] == [
        "id", "prediction", "impurity", "impurityStats", "rawCount", "gain", "leftChild", "rightChild", "split"]
    assert pq.read_table(os.path.join(q, "treesMetadata")).schema.names == ["treeID", "metadata", "weights"]
    rf2 = RandomForestClassificationModel.load(q)
    np.testing.assert_array_equal(rf2.featureImportances.toArray(), rf.featureImportances.toArray())


def test_pipeline_fit_save_load(spark, tmp_path):
    rs = np.random.RandomState(4)
    X = rs.randn(800, 3) * [1, 10, 100]
    y = ((X[:, 0] + X[:, 1] / 10) > 0).astype(float)
    df = spark.createDataFrame(pd.DataFrame({"a": X[:, 0], "b": X[:, 1], "c": X[:, 2], "label": y}))
    pipe = Pipeline(stages=[VectorAssembler(inputCols=["a", "b", "c"], outputCol="raw"),
                            StandardScaler(inputCol="raw", outputCol="features", withMean=True),
                            KMeans(k=3, featuresCol="features", predictionCol="cluster", seed=1),
                            LogisticRegression(featuresCol="features", labelCol="label")])
    model = pipe.fit(df)
    out = model.transform(df)
    assert {"raw", "features", "cluster", "prediction", "probability"} <= set(out.columns)
    p = str(tmp_path / "pipe")
    model.write().overwrite().save(p)
    md = json.loads(open(os.path.join(p, "metadata", "part-00000")).readline())
    assert md["class"] == "org.apache.spark.ml.PipelineModel" and len(md["paramMap"]["stageUids"]) == 4
    assert sorted(os.listdir(os.path.join(p, "stages")))[0].startswith("0_")
    back = PipelineModel.load(p)
    a = np.array([r.prediction for r in out.select("prediction").collect()])
    b = np.array([r.prediction for r in back.transform(df).select("prediction").collect()])
    np.testing.assert_array_equal(a, b)
    pipe.write().overwrite().save(str(tmp_path / "pipe_est"))
    assert len(Pipeline.load(str(tmp_path / "pipe_est")).getStages()) == 4


def test_string_indexer_binarizer_minmax(spark, tmp_path):
    df = spark.createDataFrame([("b", 0.2), ("a", 0.9), ("b", 0.6), ("c", 0.1)], ["h", "x"])
    si = StringIndexer(inputCol="h", outputCol="hi").fit(df)
    assert si.labels == ["b", "a", "c"]
    assert [r.hi for r in si.transform(df).collect()] == [0.0, 1.0, 0.0, 2.0]
    si.write().overwrite().save(str(tmp_path / "si"))
    assert U.load(str(tmp_path / "si")).labels == ["b", "a", "c"]
    assert [r.y for r in Binarizer(threshold=0.5, inputCol="x", outputCol="y").transform(df).collect()] == \
        [0.0, 1.0, 1.0, 0.0]
    v = VectorAssembler(inputCols=["x"], outputCol="v").transform(df)
    mm = MinMaxScaler(inputCol="v", outputCol="m").fit(v)
    got = [r.m[0] for r in mm.transform(v).collect()]
    np.testing.assert_allclose(got, [(x - 0.1) / 0.8 for x in [0.2, 0.9, 0.6, 0.1]])


def test_fit_pauses_cyclic_gc_and_restores_it(monkeypatch):
    """Estimator.fit runs with Python's cyclic collector paused (host-latency guard) and restores it."""
    import gc
    from clustermachinelearningforhospitalnetworks_apache_spark_amd.utils.device import gc_paused
    assert gc.isenabled()
    with gc_paused():
        assert not gc.isenabled()
        with gc_paused():  # nested: stays paused, and the inner exit does not re-enable it
            assert not gc.isenabled()
        assert not gc.isenabled()
    assert gc.isenabled()
    monkeypatch.setenv("CML_GC_PAUSE", "0")
    with gc_paused():
        assert gc.isenabled()
