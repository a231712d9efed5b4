"""NaiveBayes (multinomial / bernoulli / gaussian) vs sklearn's MultinomialNB / BernoulliNB / GaussianNB."""
import numpy as np
import pytest
from sklearn.naive_bayes import BernoulliNB, GaussianNB, MultinomialNB

from helpers import session
from clustermachinelearningforhospitalnetworks_apache_spark_amd.ml.classification import NaiveBayes, NaiveBayesModel
from clustermachinelearningforhospitalnetworks_apache_spark_amd.ml.feature import VectorAssembler


def _frame(X, y):
    spark = session()
    d = X.shape[1]
    names = [f"x{j}" for j in range(d)]
    rows = [tuple(map(float, r)) + (float(t),) for r, t in zip(X, y)]
    df = spark.createDataFrame(rows, ", ".join(f"{c} DOUBLE" for c in names) + ", label DOUBLE")
    return VectorAssembler(inputCols=names, outputCol="features").transform(df)


def _probs(df):
    return np.stack(df.toPandas().probability.map(lambda v: v.toArray()))


def test_multinomial_matches_sklearn(tmp_path):
    rs = np.random.RandomState(0)
    y = rs.randint(0, 3, 1500)
    X = rs.poisson(1.0 + 2.0 * np.eye(3)[y] @ rs.rand(3, 5))
    f = _frame(X, y)
    m = NaiveBayes(smoothing=1.0).fit(f)
    sk = MultinomialNB(alpha=1.0).fit(X, y)
    np.testing.assert_allclose(m.theta.toArray(), sk.feature_log_prob_, rtol=1e-10)
    # Spark smooths the priors too: log((n_c + 1) / (N + C))
    np.testing.assert_allclose(m.pi.toArray(), np.log((np.bincount(y) + 1.0) / (len(y) + 3.0)), rtol=1e-12)
    out = m.transform(f)
    sk2 = MultinomialNB(alpha=1.0, class_prior=np.exp(m.pi.toArray())).fit(X, y)
    np.testing.assert_allclose(_probs(out), sk2.predict_proba(X), rtol=1e-9)
    np.testing.assert_array_equal(np.asarray(out.toPandas().prediction), sk2.predict(X))
    p = str(tmp_path / "nb")
    m.write().overwrite().save(p)
    np.testing.assert_allclose(_probs(NaiveBayesModel.load(p).transform(f)), _probs(out), rtol=1e-12)


def test_bernoulli_and_gaussian_match_sklearn():
    rs = np.random.RandomState(1)
    y = rs.randint(0, 2, 2000)
    Xb = (rs.rand(2000, 4) < 0.3 + 0.4 * y[:, None] * [1, 0, 1, 0]).astype(float)
    mb = NaiveBayes(modelType="bernoulli").fit(_frame(Xb, y))
    skb = BernoulliNB(alpha=1.0).fit(Xb, y)
    np.testing.assert_allclose(mb.theta.toArray(), skb.feature_log_prob_, rtol=1e-10)
    pb = _probs(mb.transform(_frame(Xb, y)))
    # sklearn's class prior is unsmoothed; compare up to that prior by fitting with Spark's
    skb2 = BernoulliNB(alpha=1.0, class_prior=np.exp(mb.pi.toArray())).fit(Xb, y)
    np.testing.assert_allclose(pb, skb2.predict_proba(Xb), rtol=1e-9)
    Xg = rs.randn(2000, 3) + y[:, None] * [1.0, -0.5, 0.0]
    mg = NaiveBayes(modelType="gaussian").fit(_frame(Xg, y))
    skg = GaussianNB().fit(Xg, y)
    np.testing.assert_allclose(mg.theta.toArray(), skg.theta_, rtol=1e-10)
    np.testing.assert_allclose(mg.sigma.toArray(), skg.var_, rtol=1e-8)
    np.testing.assert_allclose(_probs(mg.transform(_frame(Xg, y))), skg.predict_proba(Xg), rtol=1e-7, atol=1e-12)
    with pytest.raises(ValueError):
        NaiveBayes().fit(_frame(Xg, y))  # negative features for multinomial


@pytest.mark.gpu
def test_naive_bayes_gpu_equals_cpu():
    import pandas as pd
    from clustermachinelearningforhospitalnetworks_apache_spark_amd.sql import SparkSession
    rs = np.random.RandomState(2)
    y = rs.randint(0, 3, 20000)
    X = rs.randn(20000, 4) + y[:, None] * 0.7
    pdf = pd.DataFrame(X, columns=list("abcd"))
    pdf["label"] = y.astype(float)
    out = {}
    for master in ("mi355x", "local[1]"):
        spark = SparkSession.builder.appName("nb").master(master).getOrCreate()
        f = VectorAssembler(inputCols=list("abcd"), outputCol="features").transform(spark.createDataFrame(pdf))
        m = NaiveBayes(modelType="gaussian").fit(f)
        out[master] = (m.theta.toArray(), m.sigma.toArray(), _probs(m.transform(f)))
        spark.stop()
    for g, c in zip(out["mi355x"], out["local[1]"]):
        np.testing.assert_allclose(g, c, rtol=1e-9, atol=1e-14)
