"""GPU runs of the round-2 MLlib additions: the K13 hinge / squared loss instantiations vs the
float64 torch reference, and the new estimators / transformers on a device session ("mi355x")
against the same code on the local[1] CPU session."""
import numpy as np
import pandas as pd
import pytest
import torch

from clustermachinelearningforhospitalnetworks_apache_spark_amd.ops import glm_ops

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("dtype", [torch.float64, torch.float32, torch.bfloat16, torch.float8_e4m3fn])
@pytest.mark.parametrize("n,d", [(1000, 4), (4097, 31), (20000, 256), (3000, 513)])
@pytest.mark.parametrize("loss", ["hinge", "squared"])
def test_loss_grad_kernel(dtype, n, d, loss):
    torch.manual_seed(2)
    x = torch.randn(n, d, dtype=torch.float64).to(dtype)
    coef = torch.randn(d + 1, dtype=torch.float64) * 0.1
    y = (torch.rand(n) > 0.5).double()
    if loss == "hinge":
        # keep rows away from the hinge point so f32 and f64 margins take the same branch
        m = x.double() @ coef[:d] + coef[d]
        keep = (1 - (2 * y - 1) * m).abs() > 1e-3
        x, y = x[keep].contiguous(), y[keep].contiguous()
    w = torch.rand(x.shape[0], dtype=torch.float64) + 0.5
    for wt in (None, w):
        oc = glm_ops.loss_grad(x, d, y, coef, wt, loss=loss)
        og = glm_ops.loss_grad(x.cuda(), d, y.cuda(), coef.cuda(), None if wt is None else wt.cuda(), loss=loss)
        tol = 1e-8 if dtype == torch.float64 else 2e-6
        np.testing.assert_allclose(og.cpu().numpy(), oc.numpy(), rtol=tol, atol=tol * n)


def _vec(df, name):
    return np.stack([v.toArray() for v in df.toPandas()[name]])


def test_ml_more_gpu_equals_cpu():
    from clustermachinelearningforhospitalnetworks_apache_spark_amd.ml.classification import (
        LinearSVC, MultilayerPerceptronClassifier, OneVsRest, LogisticRegression)
    from clustermachinelearningforhospitalnetworks_apache_spark_amd.ml.clustering import GaussianMixture
    from clustermachinelearningforhospitalnetworks_apache_spark_amd.ml.feature import (
        MaxAbsScaler, PolynomialExpansion, RFormula, RobustScaler, VectorAssembler, VectorIndexer)
    from clustermachinelearningforhospitalnetworks_apache_spark_amd.ml.regression import (
        AFTSurvivalRegression, IsotonicRegression)
    from clustermachinelearningforhospitalnetworks_apache_spark_amd.ml.stat import Summarizer
    from clustermachinelearningforhospitalnetworks_apache_spark_amd.sql import SparkSession
    from clustermachinelearningforhospitalnetworks_apache_spark_amd.sql import functions as F
    rs = np.random.RandomState(9)
    n = 4000
    X = rs.normal(size=(n, 4))
    pdf = pd.DataFrame(X, columns=list("abcd"))
    pdf["ward"] = np.array(["icu", "er", "gen"])[rs.randint(0, 3, n)]
    pdf["y"] = (X @ [1, -1, 0.5, 0] + 0.3 * rs.normal(size=n) > 0).astype(float)
    pdf["cls"] = rs.randint(0, 3, n).astype(float) + (X[:, 0] > 1)
    pdf["t"] = np.exp(0.3 * X[:, 0] + 0.5 * np.log(rs.exponential(size=n)))
    pdf["cens"] = (rs.rand(n) > 0.2).astype(float)
    pdf["cat"] = rs.randint(0, 3, n).astype(float)
    outs = {}
    for master in ("mi355x", "local[1]"):
        rs2 = np.random.RandomState(11)
        spark = SparkSession.builder.appName("mlmore").master(master).getOrCreate()
        df = VectorAssembler(inputCols=list("abcd"), outputCol="features").transform(spark.createDataFrame(pdf))
        r = {}
        r["maxabs"] = _vec(MaxAbsScaler(inputCol="features", outputCol="o").fit(df).transform(df), "o")
        r["robust"] = _vec(RobustScaler(inputCol="features", outputCol="o").fit(df).transform(df), "o")
        r["poly"] = _vec(PolynomialExpansion(degree=3, inputCol="features", outputCol="o").transform(df), "o")
        dfi = VectorAssembler(inputCols=["cat", "a"], outputCol="ci").transform(df)
        r["vi"] = _vec(VectorIndexer(maxCategories=4, inputCol="ci", outputCol="o").fit(dfi).transform(dfi), "o")
        r["rform"] = _vec(RFormula(formula="y ~ ward + a + b").fit(df).transform(df), "features")
        svc = LinearSVC(labelCol="y", regParam=0.01, maxIter=50).fit(df)
        r["svc"] = np.r_[svc.coefficients.toArray(), svc.intercept]
        ovr = OneVsRest(classifier=LogisticRegression(maxIter=30), labelCol="cls").fit(df)
        r["ovr"] = _vec(ovr.transform(df), "rawPrediction")
        mlp = MultilayerPerceptronClassifier(layers=[4, 6, 2], labelCol="y", seed=1, maxIter=40).fit(df)
        r["mlp"] = mlp.weights.toArray()
        gmm = GaussianMixture(k=3, seed=5, maxIter=20).fit(df)
        r["gmm"] = np.array(gmm.weights)
        aft = AFTSurvivalRegression(labelCol="t", censorCol="cens").fit(df)
        r["aft"] = np.r_[aft.coefficients.toArray(), aft.intercept, aft.scale]
        iso = IsotonicRegression(labelCol="y").fit(df)
        r["iso"] = iso.predictions.toArray()
        from clustermachinelearningforhospitalnetworks_apache_spark_amd.ml.regression import FMRegressor
        from clustermachinelearningforhospitalnetworks_apache_spark_amd.ml.recommendation import ALS
        fm = FMRegressor(labelCol="t", factorSize=3, maxIter=30, stepSize=0.05, seed=2).fit(df)
        r["fm"] = np.r_[fm.intercept, fm.linear.toArray(), fm.factors.toArray().ravel()]
        rt = spark.createDataFrame(pd.DataFrame({"user": rs2.randint(0, 50, 2000), "item": rs2.randint(0, 40, 2000),
                                                 "rating": rs2.rand(2000) * 5}))
        als = ALS(rank=4, maxIter=5, seed=3).fit(rt)
        r["als"] = np.stack([np.array(x.features) for x in sorted(als.userFactors.collect(), key=lambda x: x.id)])
        s = df.select(Summarizer.metrics("mean", "variance", "max").summary(F.col("features"))).collect()[0][0]
        r["summ"] = np.r_[s.mean.toArray(), s.variance.toArray(), s.max.toArray()]
        outs[master] = r
        spark.stop()
    g, c = outs["mi355x"], outs["local[1]"]
    for key in ("maxabs", "robust", "poly", "vi", "rform", "iso"):
        np.testing.assert_allclose(g[key], c[key], rtol=1e-12, atol=1e-12, err_msg=key)
    np.testing.assert_allclose(g["summ"], c["summ"], rtol=1e-10, err_msg="summ")
    for key in ("svc", "aft", "gmm"):
        np.testing.assert_allclose(g[key], c[key], rtol=1e-4, atol=1e-5, err_msg=key)
    np.testing.assert_allclose(g["ovr"], c["ovr"], rtol=1e-5, atol=1e-5, err_msg="ovr")
    np.testing.assert_allclose(g["mlp"], c["mlp"], rtol=1e-4, atol=1e-4, err_msg="mlp")
    np.testing.assert_allclose(g["fm"], c["fm"], rtol=1e-5, atol=1e-7, err_msg="fm")
    np.testing.assert_allclose(g["als"], c["als"], rtol=1e-4, atol=1e-5, err_msg="als")
