"""AFTSurvivalRegression (vs a scipy optimum of the same likelihood), IsotonicRegression (vs sklearn),
GaussianMixture (E-step probabilities vs scipy densities; recovers well-separated components); Spark-layout persistence round trips."""
import numpy as np
import pytest

from helpers import session
from clustermachinelearningforhospitalnetworks_apache_spark_amd.ml import util as U
from clustermachinelearningforhospitalnetworks_apache_spark_amd.ml.clustering import GaussianMixture, GaussianMixtureModel
from clustermachinelearningforhospitalnetworks_apache_spark_amd.ml.feature import VectorAssembler
from clustermachinelearningforhospitalnetworks_apache_spark_amd.ml.regression import (
    AFTSurvivalRegression, AFTSurvivalRegressionModel, IsotonicRegression, IsotonicRegressionModel)


@pytest.fixture(scope="module")
def spark():
    return session()


def _frame(spark, X, extra: dict):
    cols = [f"c{j}" for j in range(X.shape[1])]
    names = list(extra)
    rows = [tuple(float(v) for v in r) + tuple(float(extra[k][i]) for k in names) for i, r in enumerate(X)]
    df = spark.createDataFrame(rows, ", ".join(f"{c} DOUBLE" for c in cols + names))
    return VectorAssembler(inputCols=cols, outputCol="features").transform(df)


def _col(df, name):
    v = df.toPandas()[name].tolist()
    return np.stack([a.toArray() for a in v]) if hasattr(v[0], "toArray") else np.asarray(v, dtype=float)


def test_aft_matches_scipy_optimum(spark, tmp_path):
    from scipy.optimize import minimize
    rs = np.random.RandomState(0)
    n = 500
    X = rs.normal(size=(n, 2))
    beta, b, sigma = np.array([0.5, -0.3]), 1.0, 0.7
    eps = np.log(rs.exponential(size=n))  # standard extreme value (min) distribution
    t = np.exp(X @ beta + b + sigma * eps)
    c = (rs.rand(n) > 0.3).astype(float)
    t = np.where(c == 1, t, t * rs.uniform(0.3, 1.0, n))  # censored: observed earlier
    df = _frame(spark, X, {"label": t, "censor": c})
    m = AFTSurvivalRegression(quantileProbabilities=[0.1, 0.5, 0.9], quantilesCol="q").fit(df)

    def nll(p):
        e = (np.log(t) - X @ p[:2] - p[2]) / np.exp(p[3])
        return np.mean(c * p[3] - c * e + np.exp(e))

    ref = minimize(nll, np.zeros(4), method="BFGS", options={"gtol": 1e-10})
    got = np.r_[m.coefficients.toArray(), m.intercept, np.log(m.scale)]
    np.testing.assert_allclose(got, ref.x, atol=2e-4)
    out = m.transform(df)
    lam = np.exp(X @ m.coefficients.toArray() + m.intercept)
    np.testing.assert_allclose(_col(out, "prediction"), lam, rtol=1e-10)
    q = _col(out, "q")
    np.testing.assert_allclose(q[:, 1], lam * (-np.log(0.5)) ** m.scale, rtol=1e-10)
    assert m.predict(X[0]) == pytest.approx(lam[0])
    p = str(tmp_path / "aft")
    m.write().overwrite().save(p)
    back = AFTSurvivalRegressionModel.load(p)
    assert back.scale == pytest.approx(m.scale) and back.getQuantilesCol() == "q"
    with pytest.raises(ValueError):
        AFTSurvivalRegression().fit(_frame(spark, X, {"label": -t, "censor": c}))


def test_isotonic_matches_sklearn(spark, tmp_path):
    from sklearn.isotonic import IsotonicRegression as SkIso
    rs = np.random.RandomState(1)
    n = 200
    x = np.round(rs.uniform(0, 10, n), 1)  # ties in x
    y = np.log1p(x) + rs.normal(scale=0.3, size=n)
    w = rs.uniform(0.5, 2.0, n)
    df = _frame(spark, x[:, None], {"label": y, "w": w})
    m = IsotonicRegression(weightCol="w").fit(df)
    sk = SkIso(out_of_bounds="clip").fit(x, y, sample_weight=w)
    grid = np.linspace(-1, 11, 97)
    ours = np.array([m.predict(v) for v in grid])
    np.testing.assert_allclose(ours, sk.predict(grid), atol=1e-10)
    np.testing.assert_allclose(_col(m.transform(df), "prediction"), sk.predict(x), atol=1e-10)
    assert np.all(np.diff(m.predictions.toArray()) >= -1e-12)
    anti = IsotonicRegression(isotonic=False).fit(_frame(spark, x[:, None], {"label": -y}))
    assert np.all(np.diff(anti.predictions.toArray()) <= 1e-12)
    p = str(tmp_path / "iso")
    m.write().overwrite().save(p)
    back = U.load(p)
    assert isinstance(back, IsotonicRegressionModel)
    np.testing.assert_allclose(back.boundaries.toArray(), m.boundaries.toArray())


def test_gaussian_mixture(spark, tmp_path):
    rs = np.random.RandomState(2)
    A = rs.multivariate_normal([0, 0], [[1, 0.5], [0.5, 1]], 300)
    B = rs.multivariate_normal([6, 5], [[0.5, 0], [0, 2]], 200)
    X = np.vstack([A, B])
    df = _frame(spark, X, {})
    m = GaussianMixture(k=2, seed=3, maxIter=1, tol=0.0).fit(df)
    m50 = GaussianMixture(k=2, seed=3, maxIter=200, tol=1e-8).fit(df)
    order = np.argsort([g[0].toArray()[0] for g in m50.gaussians])
    mus = np.stack([m50.gaussians[i][0].toArray() for i in order])
    np.testing.assert_allclose(mus, [A.mean(0), B.mean(0)], atol=0.05)
    np.testing.assert_allclose(np.array(m50.weights)[order], [0.6, 0.4], atol=0.01)
    # E-step probabilities of a model vs scipy densities
    w0 = np.array(m.weights)
    m2 = GaussianMixtureModel(w0, np.stack([g[0].toArray() for g in m.gaussians]),
                              np.stack([g[1].toArray() for g in m.gaussians]))
    prob = _col(m2.setFeaturesCol("features").transform(df), "probability")
    from scipy.stats import multivariate_normal as mvn
    lp = np.stack([np.log(w0[j]) + mvn(m2._mu[j], m2._cov[j]).logpdf(X) for j in range(2)], 1)
    ref = np.exp(lp - lp.max(1, keepdims=True))
    np.testing.assert_allclose(prob, ref / ref.sum(1, keepdims=True), atol=1e-9)
    s = m50.summary
    assert sum(s.clusterSizes) == 500 and s.numIter >= 2 and np.isfinite(s.logLikelihood)
    pred = _col(m50.transform(df), "prediction")
    assert min((pred[:300] == pred[0]).mean(), (pred[300:] == pred[300]).mean()) > 0.97
    p = str(tmp_path / "gmm")
    m50.write().overwrite().save(p)
    back = U.load(p)
    np.testing.assert_allclose(_col(back.transform(df), "probability"), _col(m50.transform(df), "probability"))


def test_factorization_machines(spark, tmp_path):
    from clustermachinelearningforhospitalnetworks_apache_spark_amd.ml.classification import FMClassifier
    from clustermachinelearningforhospitalnetworks_apache_spark_amd.ml.regression import FMRegressor
    rs = np.random.RandomState(5)
    n, d, f = 600, 4, 2
    X = rs.normal(size=(n, d))
    V = rs.normal(scale=0.7, size=(d, f))
    w = np.array([0.5, -0.3, 0.0, 0.2])
    inter = 0.5 * (((X @ V) ** 2) - (X ** 2) @ (V ** 2)).sum(1)
    y = 1.0 + X @ w + inter + 0.05 * rs.normal(size=n)
    df = _frame(spark, X, {"label": y})
    m = FMRegressor(factorSize=2, stepSize=0.05, maxIter=400, seed=3).fit(df)
    pred = _col(m.transform(df), "prediction")
    assert np.mean((pred - y) ** 2) < 0.1 * np.var(y)
    # prediction formula
    W, Vm = m.linear.toArray(), m.factors.toArray()
    ref = m.intercept + X @ W + 0.5 * (((X @ Vm) ** 2) - (X ** 2) @ (Vm ** 2)).sum(1)
    np.testing.assert_allclose(pred, ref, rtol=1e-10)
    p = str(tmp_path / "fm")
    m.write().overwrite().save(p)
    back = U.load(p)
    np.testing.assert_allclose(_col(back.transform(df), "prediction"), pred)
    yc = (inter > np.median(inter)).astype(float)
    mc = FMClassifier(factorSize=2, stepSize=0.05, maxIter=300, seed=1).fit(_frame(spark, X, {"label": yc}))
    out = mc.transform(_frame(spark, X, {"label": yc}))
    assert (_col(out, "prediction") == yc).mean() > 0.85
    np.testing.assert_allclose(_col(out, "probability").sum(1), 1.0)
    nolin = FMRegressor(factorSize=2, fitLinear=False, fitIntercept=False, maxIter=5, seed=3).fit(df)
    assert np.all(nolin.linear.toArray() == 0) and nolin.intercept == 0.0
