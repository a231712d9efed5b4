"""BisectingKMeans: recovers well-separated blobs, leaf costs add up, tree-walk prediction, save/load."""
import numpy as np
import pytest

from helpers import session
from clustermachinelearningforhospitalnetworks_apache_spark_amd.ml.clustering import (BisectingKMeans,
                                                                                      BisectingKMeansModel)
from clustermachinelearningforhospitalnetworks_apache_spark_amd.ml.feature import VectorAssembler

# level-wise splitting (Spark): root -> two pairs -> four blobs
CENTERS = np.array([[0.0, 0.0], [4.0, 0.0], [0.0, 30.0], [4.0, 30.0]])


def _frame(master="local[2]"):
    from clustermachinelearningforhospitalnetworks_apache_spark_amd.sql import SparkSession
    rs = np.random.RandomState(0)
    lab = rs.randint(0, 4, 2500)
    X = CENTERS[lab] + rs.randn(2500, 2) * 0.5
    spark = session() if master == "local[2]" else SparkSession.builder.master(master).getOrCreate()
    df = spark.createDataFrame([tuple(map(float, r)) for r in X], "a DOUBLE, b DOUBLE")
    return X, lab, VectorAssembler(inputCols=["a", "b"], outputCol="features").transform(df)


def _check(X, lab, f, tmp_path=None):
    m = BisectingKMeans(k=4, seed=3).fit(f)
    cs = np.stack(m.clusterCenters())
    assert cs.shape == (4, 2)
    # every true centre has a learned centre within 0.2
    d = np.linalg.norm(cs[:, None, :] - CENTERS[None], axis=2)
    assert d.min(0).max() < 0.2
    pred = np.asarray(m.transform(f).toPandas().prediction)
    # clusters are pure: one learned label per true blob
    for c in range(4):
        assert len(np.unique(pred[lab == c])) == 1
    want = sum(((X[pred == j] - X[pred == j].mean(0)) ** 2).sum() for j in range(4))
    np.testing.assert_allclose(m.trainingCost, want, rtol=1e-9)
    np.testing.assert_allclose(m.computeCost(f), want, rtol=1e-6)
    assert BisectingKMeans(k=2, seed=3).fit(f).trainingCost > m.trainingCost
    if tmp_path is not None:
        p = str(tmp_path / "bkm")
        m.write().overwrite().save(p)
        back = BisectingKMeansModel.load(p)
        np.testing.assert_array_equal(np.asarray(back.transform(f).toPandas().prediction), pred)
        np.testing.assert_allclose(np.stack(back.clusterCenters()), cs)
    return cs


def test_bisecting_kmeans_blobs(tmp_path):
    X, lab, f = _frame()
    _check(X, lab, f, tmp_path)


@pytest.mark.gpu
def test_bisecting_kmeans_gpu():
    X, lab, f = _frame("mi355x")
    _check(X, lab, f)
