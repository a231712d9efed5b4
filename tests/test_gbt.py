"""GBTRegressor / GBTClassifier: boosting recurrence vs an independent chain of single-tree fits,
Spark loss/probability formulas, validation early stop, Spark ensemble save layout, GPU parity."""
import numpy as np
import pyarrow.parquet as pq
import pytest
import torch

from helpers import hospital_frame, session
from clustermachinelearningforhospitalnetworks_apache_spark_amd.ml import Pipeline, PipelineModel
from clustermachinelearningforhospitalnetworks_apache_spark_amd.ml.classification import (
    GBTClassificationModel, GBTClassifier)
from clustermachinelearningforhospitalnetworks_apache_spark_amd.ml.evaluation import (
    MulticlassClassificationEvaluator, RegressionEvaluator)
from clustermachinelearningforhospitalnetworks_apache_spark_amd.ml.feature import VectorAssembler
from clustermachinelearningforhospitalnetworks_apache_spark_amd.ml.regression import (
    DecisionTreeRegressor, GBTRegressionModel, GBTRegressor)
from clustermachinelearningforhospitalnetworks_apache_spark_amd.models import trees as TR
from clustermachinelearningforhospitalnetworks_apache_spark_amd.sql import functions as F

FEATS = ["admission_count", "current_occupancy", "emergency_visits", "seasonality_index"]


@pytest.fixture(scope="module")
def spark():
    return session()


@pytest.fixture(scope="module")
def hosp(spark):
    pdf = hospital_frame(2000, seed=11)
    df = spark.createDataFrame(pdf)
    fd = VectorAssembler(inputCols=FEATS, outputCol="features").transform(df)
    return pdf, fd


def _col(df, name):
    return np.asarray(df.toPandas()[name].tolist(), dtype=np.float64)


def test_gbt_one_iteration_is_a_decision_tree(hosp):
    _, fd = hosp
    g = GBTRegressor(featuresCol="features", labelCol="length_of_stay", maxIter=1).fit(fd)
    d = DecisionTreeRegressor(featuresCol="features", labelCol="length_of_stay").fit(fd)
    np.testing.assert_allclose(_col(g.transform(fd), "prediction"), _col(d.transform(fd), "prediction"),
                               rtol=1e-12, atol=1e-12)
    assert g.treeWeights == [1.0]


def test_gbt_recurrence_matches_chain_of_tree_fits(hosp, spark):
    """Tree 0 on y (weight 1), tree m on 2(y - F) (weight stepSize): rebuilt with the public
    DecisionTreeRegressor on explicit residual columns (n <= 10000, so candidates use every row)."""
    pdf, fd = hosp
    iters, step = 4, 0.3
    g = GBTRegressor(featuresCol="features", labelCol="length_of_stay", maxIter=iters, stepSize=step).fit(fd)
    assert g.getNumTrees == iters and g.treeWeights == [1.0] + [step] * (iters - 1)
    y = pdf.length_of_stay.values.astype(np.float64)
    f = np.zeros_like(y)
    cur = fd.withColumn("r", F.col("length_of_stay"))
    for m in range(iters):
        t = DecisionTreeRegressor(featuresCol="features", labelCol="r").fit(cur)
        f += (1.0 if m == 0 else step) * _col(t.transform(cur), "prediction")
        pdf2 = pdf.copy()
        pdf2["r"] = 2.0 * (y - f)
        cur = VectorAssembler(inputCols=FEATS, outputCol="features").transform(spark.createDataFrame(pdf2))
    np.testing.assert_allclose(_col(g.transform(fd), "prediction"), f, rtol=1e-10, atol=1e-10)
    errs = g.evaluateEachIteration(fd)
    assert len(errs) == iters and all(b <= a + 1e-12 for a, b in zip(errs, errs[1:]))
    np.testing.assert_allclose(errs[-1], np.mean((y - f) ** 2), rtol=1e-10)
    rmse = RegressionEvaluator(labelCol="length_of_stay").evaluate(g.transform(fd))
    assert rmse < pdf.length_of_stay.std()
    imp = g.featureImportances.toArray()
    assert abs(imp.sum() - 1.0) < 1e-12 and (imp >= 0).all()


def test_gbt_absolute_loss_residuals():
    f = torch.tensor([0.0, 2.0, 1.0], dtype=torch.float64)
    y = torch.tensor([1.0, 1.0, 1.0], dtype=torch.float64)
    assert TR.gbt_residual("absolute", f, y).tolist() == [1.0, -1.0, 0.0]
    ys = torch.tensor([1.0, -1.0], dtype=torch.float64)
    fs = torch.tensor([0.3, 0.3], dtype=torch.float64)
    want = 4 * ys / (1 + torch.exp(2 * ys * fs))
    np.testing.assert_allclose(TR.gbt_residual("logistic", fs, ys).numpy(), want.numpy(), rtol=1e-14)
    np.testing.assert_allclose(TR.gbt_loss("logistic", fs, ys).numpy(),
                               (2 * torch.log1p(torch.exp(-2 * ys * fs))).numpy(), rtol=1e-14)


def test_gbt_classifier_probabilities_and_accuracy(hosp, spark, tmp_path):
    pdf, fd = hosp
    fdb = fd.withColumn("LOS_binary", F.when(F.col("length_of_stay") > 5.0, 1).otherwise(0))
    clf = GBTClassifier(featuresCol="features", labelCol="LOS_binary", maxIter=10)
    m = clf.fit(fdb)
    out = m.transform(fdb).toPandas()
    raw = np.stack(out.rawPrediction.map(lambda v: v.toArray()).values)
    prob = np.stack(out.probability.map(lambda v: v.toArray()).values)
    np.testing.assert_allclose(raw[:, 0], -raw[:, 1])
    np.testing.assert_allclose(prob[:, 1], 1.0 / (1.0 + np.exp(-2.0 * raw[:, 1])), rtol=1e-12)
    np.testing.assert_array_equal(out.prediction.values, (raw[:, 1] > 0).astype(float))
    acc = MulticlassClassificationEvaluator(labelCol="LOS_binary", metricName="accuracy").evaluate(m.transform(fdb))
    base = max(out.LOS_binary.mean(), 1 - out.LOS_binary.mean())
    assert acc > base and acc > 0.85
    # Spark ensemble layout: data/ (treeID, nodeData) + treesMetadata/ weights; load round trip
    p = str(tmp_path / "gbtc")
    m.write().overwrite().save(p)
    tm = pq.read_table(p + "/treesMetadata").to_pandas().sort_values("treeID")
    np.testing.assert_allclose(tm.weights.values, [1.0] + [0.1] * 9)
    m2 = GBTClassificationModel.load(p)
    np.testing.assert_array_equal(_col(m2.transform(fdb), "prediction"), out.prediction.values)
    with pytest.raises(ValueError):
        GBTClassifier(featuresCol="features", labelCol="length_of_stay").fit(fd)


def test_gbt_validation_early_stop_and_pipeline(hosp, tmp_path):
    pdf, fd = hosp
    fv = fd.withColumn("is_val", F.col("seasonality_index") > 0.8)
    m = GBTRegressor(featuresCol="features", labelCol="length_of_stay", maxIter=200, stepSize=0.5,
                     validationIndicatorCol="is_val", validationTol=0.01).fit(fv)
    assert 1 <= m.getNumTrees < 200
    pm = Pipeline(stages=[GBTRegressor(featuresCol="features", labelCol="length_of_stay", maxIter=3)]).fit(fd)
    p = str(tmp_path / "pm")
    pm.write().overwrite().save(p)
    back = PipelineModel.load(p)
    assert isinstance(back.stages[0], GBTRegressionModel)
    np.testing.assert_allclose(_col(back.transform(fd), "prediction"), _col(pm.transform(fd), "prediction"))


@pytest.mark.gpu
def test_gbt_gpu_matches_cpu():
    """GPU histogram (fixed point, K18) + K21 margin updates vs the CPU float64 engine."""
    rs = np.random.RandomState(3)
    n, d = 50000, 6
    x = rs.rand(n, d)
    y = np.sin(6 * x[:, 0]) + x[:, 1] * x[:, 2] + 0.05 * rs.randn(n)
    p = TR.TreeParams(max_depth=4, seed=7)
    tc, wc = TR.fit_gbt(torch.as_tensor(x), torch.as_tensor(y), p, 8, 0.2, "squared")
    dev = torch.device("cuda", 0)
    tg, wg = TR.fit_gbt(torch.as_tensor(x, device=dev), torch.as_tensor(y, device=dev), p, 8, 0.2, "squared")
    assert wc == wg
    xc = torch.as_tensor(x)
    fc = TR.predict_forest(tc, xc, "variance", 1, False, False, wc)[:, 0].numpy()
    fg = TR.predict_forest(tg, xc.to(dev), "variance", 1, False, False, wg)[:, 0].cpu().numpy()
    np.testing.assert_allclose(fg, fc, rtol=1e-6, atol=1e-6)
    assert np.sqrt(np.mean((y - fg) ** 2)) < np.std(y) * 0.5
