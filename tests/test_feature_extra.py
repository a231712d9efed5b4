"""Bucketizer, QuantileDiscretizer, Normalizer, PCA vs numpy oracles; Spark persistence round trip."""
import numpy as np
import pytest

from helpers import session
from clustermachinelearningforhospitalnetworks_apache_spark_amd.ml import Pipeline, PipelineModel
from clustermachinelearningforhospitalnetworks_apache_spark_amd.ml.feature import (
    Bucketizer, Normalizer, PCA, PCAModel, QuantileDiscretizer, VectorAssembler)


@pytest.fixture(scope="module")
def spark():
    return session()


def _col(df, name):
    return np.asarray(df.toPandas()[name].tolist(), dtype=np.float64)


def test_bucketizer_edges_and_invalid(spark):
    df = spark.createDataFrame([(-0.5,), (0.0,), (0.3,), (1.0,), (2.0,), (float("nan"),)], "x DOUBLE")
    b = Bucketizer(splits=[-1.0, 0.0, 1.0, 2.0], inputCol="x", outputCol="b")
    with pytest.raises(ValueError):
        b.transform(df)
    got = _col(b.setHandleInvalid("keep").transform(df), "b")
    np.testing.assert_array_equal(got, [0, 1, 1, 2, 2, 3])
    assert b.setHandleInvalid("skip").transform(df).count() == 5
    with pytest.raises(ValueError):
        Bucketizer(splits=[0.0, 1.0, 2.0], inputCol="x", outputCol="b", handleInvalid="keep").transform(df)


def test_quantile_discretizer_matches_numpy(spark, tmp_path):
    rs = np.random.RandomState(1)
    x = np.round(rs.exponential(3.0, 4001), 2)
    df = spark.createDataFrame([(float(v),) for v in x], "occ DOUBLE")
    bz = QuantileDiscretizer(numBuckets=5, inputCol="occ", outputCol="q").fit(df)
    srt = np.sort(x)
    qs = srt[np.clip(np.ceil(np.arange(6) / 5 * x.size).astype(int) - 1, 0, x.size - 1)]
    np.testing.assert_allclose(bz.getSplits()[1:-1], qs[1:-1])
    assert bz.getSplits()[0] == -np.inf and bz.getSplits()[-1] == np.inf
    q = _col(bz.transform(df), "q")
    counts = np.bincount(q.astype(int), minlength=5)
    assert counts.min() > 0.15 * x.size and counts.max() < 0.25 * x.size
    p = str(tmp_path / "bz")
    bz.write().overwrite().save(p)
    back = Bucketizer.load(p)
    np.testing.assert_array_equal(_col(back.transform(df), "q"), q)


def test_normalizer(spark):
    df = spark.createDataFrame([(3.0, 4.0), (0.0, 0.0), (-1.0, 1.0)], "a DOUBLE, b DOUBLE")
    f = VectorAssembler(inputCols=["a", "b"], outputCol="f").transform(df)
    out = np.stack(Normalizer(inputCol="f", outputCol="n").transform(f).toPandas().n.map(lambda v: v.toArray()))
    np.testing.assert_allclose(out, [[0.6, 0.8], [0, 0], [-2 ** -0.5, 2 ** -0.5]])
    out1 = np.stack(Normalizer(p=1.0, inputCol="f", outputCol="n").transform(f).toPandas().n.map(
        lambda v: v.toArray()))
    np.testing.assert_allclose(out1[0], [3 / 7, 4 / 7])


def test_pca_matches_numpy_eigh(spark, tmp_path):
    rs = np.random.RandomState(4)
    X = rs.randn(3000, 5) @ rs.randn(5, 5) + [1, 2, 3, 4, 50]
    df = spark.createDataFrame([tuple(map(float, r)) for r in X], "a DOUBLE, b DOUBLE, c DOUBLE, d DOUBLE, e DOUBLE")
    f = VectorAssembler(inputCols=list("abcde"), outputCol="f").transform(df)
    m = PCA(k=3, inputCol="f", outputCol="p").fit(f)
    w, v = np.linalg.eigh(np.cov(X, rowvar=False))
    w, v = w[::-1], v[:, ::-1]
    np.testing.assert_allclose(m.explainedVariance.toArray(), w[:3] / w.sum(), rtol=1e-8)
    pc = m.pc.toArray()
    for j in range(3):
        np.testing.assert_allclose(np.abs(pc[:, j] @ v[:, j]), 1.0, rtol=1e-8)
    proj = np.stack(m.transform(f).toPandas().p.map(lambda v: v.toArray()))
    np.testing.assert_allclose(proj, X @ pc, rtol=1e-9, atol=1e-9)
    p = str(tmp_path / "pca")
    Pipeline(stages=[PCA(k=2, inputCol="f", outputCol="p")]).fit(f).write().overwrite().save(p)
    back = PipelineModel.load(p)
    assert isinstance(back.stages[0], PCAModel) and back.stages[0].pc.toArray().shape == (5, 2)


@pytest.mark.gpu
def test_feature_extra_gpu_equals_cpu():
    """PCA through the K15 Gram kernel on the device, Bucketizer/QuantileDiscretizer/Normalizer on
    device tensors, against the local[1] CPU session."""
    import pandas as pd
    from clustermachinelearningforhospitalnetworks_apache_spark_amd.sql import SparkSession
    rs = np.random.RandomState(8)
    pdf = pd.DataFrame(rs.randn(20000, 6) @ rs.randn(6, 6), columns=list("abcdef"))
    outs = {}
    for master in ("mi355x", "local[1]"):
        spark = SparkSession.builder.appName("fx").master(master).getOrCreate()
        f = VectorAssembler(inputCols=list("abcdef"), outputCol="f").transform(spark.createDataFrame(pdf))
        m = PCA(k=3, inputCol="f", outputCol="p").fit(f)
        bz = QuantileDiscretizer(numBuckets=7, inputCol="a", outputCol="q").fit(f)
        nf = Normalizer(inputCol="f", outputCol="n").transform(f)
        outs[master] = (m.explainedVariance.toArray(), np.abs(m.pc.toArray()), bz.getSplits(),
                        _col(bz.transform(f), "q"), np.stack(nf.toPandas().n.map(lambda v: v.toArray())))
        spark.stop()
    g, c = outs["mi355x"], outs["local[1]"]
    np.testing.assert_allclose(g[0], c[0], rtol=1e-9)
    np.testing.assert_allclose(g[1], c[1], rtol=1e-7, atol=1e-9)
    assert g[2] == c[2]
    np.testing.assert_array_equal(g[3], c[3])
    np.testing.assert_allclose(g[4], c[4], rtol=1e-12)
