"""LinearSVC, OneVsRest, MultilayerPerceptronClassifier: fits vs sklearn / closed-form oracles,
persistence round trips, and the hinge/squared loss pass (CPU reference of the K13 variants)."""
import numpy as np
import pytest
import torch

from helpers import session
from clustermachinelearningforhospitalnetworks_apache_spark_amd.ml import util as U
from clustermachinelearningforhospitalnetworks_apache_spark_amd.ml.classification import (
    LinearSVC, LinearSVCModel, LogisticRegression, MultilayerPerceptronClassificationModel,
    MultilayerPerceptronClassifier, OneVsRest, OneVsRestModel)
from clustermachinelearningforhospitalnetworks_apache_spark_amd.ml.feature import VectorAssembler
from clustermachinelearningforhospitalnetworks_apache_spark_amd.ops import glm_ops


@pytest.fixture(scope="module")
def spark():
    return session()


def _frame(spark, X, y):
    cols = [f"c{j}" for j in range(X.shape[1])]
    rows = [tuple(float(v) for v in r) + (float(t),) for r, t in zip(X, y)]
    df = spark.createDataFrame(rows, ", ".join(f"{c} DOUBLE" for c in cols) + ", label DOUBLE")
    return VectorAssembler(inputCols=cols, outputCol="features").transform(df)


def _col(df, name):
    v = df.toPandas()[name].tolist()
    return np.stack([a.toArray() for a in v]) if hasattr(v[0], "toArray") else np.asarray(v, dtype=float)


def test_loss_grad_cpu_reference():
    rs = np.random.RandomState(0)
    X = torch.as_tensor(rs.normal(size=(64, 5)))
    y = torch.as_tensor((rs.rand(64) > 0.5).astype(float))
    w = torch.as_tensor(rs.uniform(0.5, 2, 64))
    coef = torch.as_tensor(rs.normal(size=6))
    m = X @ coef[:5] + coef[5]
    ys = 2 * y - 1
    act = (1 - ys * m) > 0
    out = glm_ops.loss_grad(X, 5, y, coef, w, loss="hinge")
    r = torch.where(act, -w * ys, torch.zeros_like(w))
    np.testing.assert_allclose(out[:5].numpy(), (X.T @ r).numpy(), rtol=1e-12)
    assert float(out[6]) == pytest.approx(float((w * (1 - ys * m).clamp(min=0)).sum()))
    sq = glm_ops.loss_grad(X, 5, y, coef, None, loss="squared")
    np.testing.assert_allclose(sq[:5].numpy(), (X.T @ (m - y)).numpy(), rtol=1e-12)
    lg = glm_ops.loss_grad(X, 5, y, coef, w, loss="logistic")
    np.testing.assert_allclose(lg.numpy(), glm_ops.logreg_grad(X, 5, y, coef, w).numpy(), rtol=1e-12)


def test_linear_svc_matches_primal_optimum(spark, tmp_path):
    rs = np.random.RandomState(1)
    n = 400
    X = rs.normal(size=(n, 3)) * [1.0, 3.0, 0.5]
    y = (X @ [1.0, -0.5, 2.0] + 0.3 + 0.4 * rs.normal(size=n) > 0).astype(float)
    df = _frame(spark, X, y)
    lam = 0.01
    m = LinearSVC(regParam=lam, maxIter=200).fit(df)
    # oracle: the same objective (mean hinge + lam/2 |beta_std|^2) minimised by scipy on the host
    from scipy.optimize import minimize
    sd = X.std(0, ddof=1)
    ys = 2 * y - 1

    def obj(p):
        b = p[:3] / sd
        return np.mean(np.maximum(0, 1 - ys * (X @ b + p[3]))) + 0.5 * lam * np.sum(p[:3] ** 2)

    ref = minimize(obj, np.zeros(4), method="Powell", options={"xtol": 1e-10, "ftol": 1e-12, "maxiter": 20000})
    got = np.r_[m.coefficients.toArray() * sd, m.intercept]
    assert obj(got) <= ref.fun + 1e-4
    pred = _col(m.transform(df), "prediction")
    assert (pred == y).mean() > 0.9
    assert m.summary.totalIterations > 0 and len(m.summary.objectiveHistory) > 1
    p = str(tmp_path / "svc")
    m.write().overwrite().save(p)
    back = LinearSVCModel.load(p)
    np.testing.assert_allclose(back.coefficients.toArray(), m.coefficients.toArray())
    np.testing.assert_allclose(_col(back.transform(df), "rawPrediction"), _col(m.transform(df), "rawPrediction"))
    with pytest.raises(ValueError):
        LinearSVC().fit(_frame(spark, X, y * 2))


def test_one_vs_rest(spark, tmp_path):
    rs = np.random.RandomState(2)
    centers = np.array([[0, 0], [4, 0], [0, 4]])
    y = rs.randint(0, 3, 300)
    X = centers[y] + rs.normal(size=(300, 2)) * 0.7
    df = _frame(spark, X, y)
    ovr = OneVsRest(classifier=LogisticRegression(maxIter=50))
    m = ovr.fit(df)
    assert m.numClasses == 3
    pred = _col(m.transform(df), "prediction")
    assert (pred == y).mean() > 0.95
    # the k margins = each binary model's rawPrediction[:, 1]
    raw = _col(m.transform(df), "rawPrediction")
    for c, bm in enumerate(m.models):
        np.testing.assert_allclose(raw[:, c], _col(bm.transform(df), "rawPrediction")[:, 1])
    p = str(tmp_path / "ovr")
    m.write().overwrite().save(p)
    back = U.load(p)
    assert isinstance(back, OneVsRestModel)
    np.testing.assert_array_equal(_col(back.transform(df), "prediction"), pred)
    ovr.write().overwrite().save(str(tmp_path / "ovr_est"))
    est = U.load(str(tmp_path / "ovr_est"))
    assert isinstance(est.getClassifier(), LogisticRegression) and est.getClassifier().getMaxIter() == 50
    svc = OneVsRest(classifier=LinearSVC(maxIter=50)).fit(df)
    assert (_col(svc.transform(df), "prediction") == y).mean() > 0.9


def test_mlp_classifier(spark, tmp_path):
    rs = np.random.RandomState(3)
    n = 300
    X = rs.uniform(-1, 1, size=(n, 2))
    y = ((X[:, 0] * X[:, 1]) > 0).astype(float)  # XOR: not linearly separable
    df = _frame(spark, X, y)
    mlp = MultilayerPerceptronClassifier(layers=[2, 8, 2], seed=7, maxIter=300)
    m = mlp.fit(df)
    out = m.transform(df)
    assert (_col(out, "prediction") == y).mean() > 0.9
    prob = _col(out, "probability")
    np.testing.assert_allclose(prob.sum(1), 1.0)
    assert m.weights.toArray().size == 2 * 8 + 8 + 8 * 2 + 2
    # Spark layout: layer-1 W is 8x2 column-major then b; check the forward pass by hand
    w = m.weights.toArray()
    W1, b1 = w[:16].reshape(2, 8).T, w[16:24]
    W2, b2 = w[24:40].reshape(8, 2).T, w[40:42]
    h = 1 / (1 + np.exp(-(X @ W1.T + b1)))
    np.testing.assert_allclose(_col(out, "rawPrediction"), h @ W2.T + b2, rtol=1e-9)
    p = str(tmp_path / "mlp")
    m.write().overwrite().save(p)
    back = MultilayerPerceptronClassificationModel.load(p)
    np.testing.assert_allclose(_col(back.transform(df), "probability"), prob)
    # same seed -> same model; 'gd' solver runs
    m2 = mlp.fit(df)
    np.testing.assert_allclose(m2.weights.toArray(), w)
    gd = MultilayerPerceptronClassifier(layers=[2, 4, 2], seed=1, maxIter=5, solver="gd", stepSize=0.5).fit(df)
    assert gd.summary.totalIterations >= 1
