"""ml.stat Correlation (pearson/spearman) and ChiSquareTest vs numpy/scipy oracles."""
import numpy as np
import pytest
from scipy import stats

from helpers import session
from clustermachinelearningforhospitalnetworks_apache_spark_amd.ml.feature import VectorAssembler
from clustermachinelearningforhospitalnetworks_apache_spark_amd.ml.stat import ChiSquareTest, Correlation


@pytest.fixture(scope="module")
def frame():
    spark = session()
    rs = np.random.RandomState(2)
    n = 2500
    a = rs.randn(n)
    b = 0.6 * a + 0.8 * rs.randn(n)
    c = np.round(rs.rand(n) * 4)          # ties for spearman
    e = np.full(n, 3.0)                    # zero variance -> NaN row/col
    X = np.c_[a, b, c, e]
    df = spark.createDataFrame([tuple(map(float, r)) for r in X], "a DOUBLE, b DOUBLE, c DOUBLE, e DOUBLE")
    return X, VectorAssembler(inputCols=list("abce"), outputCol="f").transform(df)


def test_pearson(frame):
    X, f = frame
    row = Correlation.corr(f, "f").head()
    m = row[0].toArray()
    assert f"{Correlation.corr(f, 'f').columns[0]}" == "pearson(f)"
    want = np.corrcoef(X[:, :3], rowvar=False)
    np.testing.assert_allclose(m[:3, :3], want, rtol=1e-10, atol=1e-12)
    assert m[3, 3] == 1.0 and np.isnan(m[3, 0]) and np.isnan(m[0, 3])


def test_spearman(frame):
    X, f = frame
    m = Correlation.corr(f, "f", "spearman").head()[0].toArray()
    want = stats.spearmanr(X[:, :3]).correlation
    np.testing.assert_allclose(m[:3, :3], want, rtol=1e-10, atol=1e-12)


def test_chisquare_matches_scipy():
    spark = session()
    rs = np.random.RandomState(5)
    n = 3000
    lab = rs.randint(0, 2, n).astype(float)
    f0 = np.where(rs.rand(n) < 0.7, lab, rs.randint(0, 2, n))      # dependent
    f1 = rs.randint(0, 3, n).astype(float)                          # independent
    df = spark.createDataFrame([(float(a), float(b), float(c)) for a, b, c in zip(f0, f1, lab)],
                               "f0 DOUBLE, f1 DOUBLE, label DOUBLE")
    v = VectorAssembler(inputCols=["f0", "f1"], outputCol="features").transform(df)
    r = ChiSquareTest.test(v, "features", "label").head()
    for j, col in enumerate((f0, f1)):
        tab = np.array([[np.sum((col == a) & (lab == b)) for b in (0, 1)] for a in np.unique(col)])
        s, p, dof, _ = stats.chi2_contingency(tab, correction=False)
        np.testing.assert_allclose(r.statistics[j], s, rtol=1e-10)
        np.testing.assert_allclose(r.pValues[j], p, rtol=1e-8, atol=1e-300)
        assert r.degreesOfFreedom[j] == dof
    assert r.pValues[0] < 1e-10 and r.pValues[1] > 1e-3


@pytest.mark.gpu
def test_correlation_gpu_equals_cpu():
    import pandas as pd
    from clustermachinelearningforhospitalnetworks_apache_spark_amd.sql import SparkSession
    rs = np.random.RandomState(6)
    pdf = pd.DataFrame(rs.randn(30000, 5) @ rs.randn(5, 5), columns=list("abcde"))
    out = {}
    for master in ("mi355x", "local[1]"):
        spark = SparkSession.builder.appName("corr").master(master).getOrCreate()
        f = VectorAssembler(inputCols=list("abcde"), outputCol="f").transform(spark.createDataFrame(pdf))
        out[master] = [Correlation.corr(f, "f", m).head()[0].toArray() for m in ("pearson", "spearman")]
        spark.stop()
    for g, c in zip(out["mi355x"], out["local[1]"]):
        np.testing.assert_allclose(g, c, rtol=1e-9, atol=1e-12)
    np.testing.assert_allclose(out["mi355x"][0], np.corrcoef(pdf.values, rowvar=False), rtol=1e-9, atol=1e-12)
