"""GeneralizedLinearRegression (IRLS on the K15 Gram kernel) vs numpy / sklearn oracles."""
import numpy as np
import pytest
from sklearn.linear_model import GammaRegressor, LogisticRegression, PoissonRegressor

from helpers import session
from clustermachinelearningforhospitalnetworks_apache_spark_amd.ml.feature import VectorAssembler
from clustermachinelearningforhospitalnetworks_apache_spark_amd.ml.regression import (
    GeneralizedLinearRegression, GeneralizedLinearRegressionModel)


def _frame(X, y):
    spark = session()
    rows = [tuple(map(float, r)) + (float(t),) for r, t in zip(X, y)]
    df = spark.createDataFrame(rows, "a DOUBLE, b DOUBLE, c DOUBLE, label DOUBLE")
    return VectorAssembler(inputCols=list("abc"), outputCol="features").transform(df)


@pytest.fixture(scope="module")
def X():
    rs = np.random.RandomState(0)
    return rs.randn(3000, 3) * [0.5, 0.3, 0.8]


def test_gaussian_identity_is_ols(X):
    rs = np.random.RandomState(1)
    y = X @ [1.0, -2.0, 0.5] + 3 + rs.randn(len(X)) * 0.1
    m = GeneralizedLinearRegression().fit(_frame(X, y))
    sol = np.linalg.lstsq(np.c_[X, np.ones(len(X))], y, rcond=None)[0]
    np.testing.assert_allclose(m.coefficients.toArray(), sol[:3], rtol=1e-9)
    assert abs(m.intercept - sol[3]) < 1e-9


def test_poisson_log_matches_sklearn(X, tmp_path):
    rs = np.random.RandomState(2)
    y = rs.poisson(np.exp(X @ [0.4, -0.3, 0.2] + 1.0))
    f = _frame(X, y)
    m = GeneralizedLinearRegression(family="poisson", tol=1e-10).fit(f)
    sk = PoissonRegressor(alpha=0.0, tol=1e-12, max_iter=10000).fit(X, y)
    np.testing.assert_allclose(m.coefficients.toArray(), sk.coef_, rtol=1e-5, atol=1e-7)
    assert abs(m.intercept - sk.intercept_) < 1e-6
    pred = np.asarray(m.transform(f).toPandas().prediction)
    np.testing.assert_allclose(pred, sk.predict(X), rtol=1e-5)
    s = m.summary
    mu = sk.predict(X)
    dev = 2 * np.sum(np.where(y > 0, y * np.log(np.where(y > 0, y, 1) / mu), 0) - (y - mu))
    np.testing.assert_allclose(s.deviance, dev, rtol=1e-6)
    assert s.deviance < s.nullDeviance and s.dispersion == 1.0 and 2 < s.numIterations <= 25
    p = str(tmp_path / "glr")
    m.write().overwrite().save(p)
    back = GeneralizedLinearRegressionModel.load(p)
    np.testing.assert_allclose(np.asarray(back.transform(f).toPandas().prediction), pred, rtol=1e-12)


def test_gamma_log_and_binomial_logit(X):
    rs = np.random.RandomState(3)
    mu = np.exp(X @ [0.3, 0.1, -0.2] + 1.5)
    y = rs.gamma(2.0, mu / 2.0)
    m = GeneralizedLinearRegression(family="gamma", link="log", tol=1e-10).fit(_frame(X, y))
    sk = GammaRegressor(alpha=0.0, tol=1e-12, max_iter=10000).fit(X, y)
    np.testing.assert_allclose(m.coefficients.toArray(), sk.coef_, rtol=1e-4, atol=1e-6)
    assert abs(m.intercept - sk.intercept_) < 1e-5
    yb = (rs.rand(len(X)) < 1 / (1 + np.exp(-(X @ [1.0, -1.0, 0.5])))).astype(float)
    mb = GeneralizedLinearRegression(family="binomial", tol=1e-10).fit(_frame(X, yb))
    lr = LogisticRegression(penalty=None, tol=1e-12, max_iter=10000).fit(X, yb)
    np.testing.assert_allclose(mb.coefficients.toArray(), lr.coef_[0], rtol=1e-5, atol=1e-6)
    with pytest.raises(ValueError):
        GeneralizedLinearRegression(family="gamma").fit(_frame(X, y - 100))


@pytest.mark.gpu
def test_glr_gpu_equals_cpu(X):
    import pandas as pd
    from clustermachinelearningforhospitalnetworks_apache_spark_amd.sql import SparkSession
    rs = np.random.RandomState(4)
    y = rs.poisson(np.exp(X @ [0.4, -0.3, 0.2] + 1.0)).astype(float)
    pdf = pd.DataFrame(X, columns=list("abc"))
    pdf["label"] = y
    out = {}
    for master in ("mi355x", "local[1]"):
        spark = SparkSession.builder.appName("glr").master(master).getOrCreate()
        f = VectorAssembler(inputCols=list("abc"), outputCol="features").transform(spark.createDataFrame(pdf))
        m = GeneralizedLinearRegression(family="poisson").fit(f)
        out[master] = np.r_[m.coefficients.toArray(), m.intercept, m.summary.deviance]
        spark.stop()
    np.testing.assert_allclose(out["mi355x"], out["local[1]"], rtol=1e-9)
