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


def test_java_random_matches_java_util_random():
    from clustermachinelearningforhospitalnetworks_apache_spark_amd.ml.bisecting import JavaRandom
    r = JavaRandom(42)  # new java.util.Random(42).nextDouble() x 2
    assert r.next_double() == 0.7275636800328681
    assert r.next_double() == 0.6832234717598454


def _pq_frame(n_p=1000, n_q=200):
    """P: one tight uniform blob of n_p rows; Q: two blobs of n_q rows each, far from P."""
    rs = np.random.RandomState(1)
    p = np.c_[rs.uniform(-101, -99, n_p), rs.uniform(-1, 1, n_p)]
    q = np.r_[np.c_[rs.randn(n_q) * 0.1 + 95, rs.randn(n_q) * 0.1], np.c_[rs.randn(n_q) * 0.1 + 105, rs.randn(n_q) * 0.1]]
    X = np.r_[p, q]
    spark = session()
    df = spark.createDataFrame([tuple(map(float, r)) for r in X], "a DOUBLE, b DOUBLE")
    return X, VectorAssembler(inputCols=["a", "b"], outputCol="features").transform(df)


def test_level_takes_largest_divisible_clusters():
    """Spark divides the LARGEST divisible clusters when fewer are needed (not the costliest):
    k = 3 splits the 1000-row blob P, although Q (two blobs, 400 rows) has far more cost."""
    X, f = _pq_frame()
    m = BisectingKMeans(k=3, seed=7).fit(f)
    pred = np.asarray(m.transform(f).toPandas().prediction)
    assert len(m.clusterCenters()) == 3
    assert len(np.unique(pred[:1000])) == 2 and len(np.unique(pred[1000:])) == 1
    # clusters below minDivisibleClusterSize stay whole even if k is not reached: P (1000) and Q (400)
    m3 = BisectingKMeans(k=3, seed=7, minDivisibleClusterSize=1000.5).fit(f)
    assert len(m3.clusterCenters()) == 2
    # a fraction below 1.0 is of the total count: 0.5 * 1400 = 700 -> only P divisible
    m4 = BisectingKMeans(k=4, seed=7, minDivisibleClusterSize=0.5).fit(f)
    p4 = np.asarray(m4.transform(f).toPandas().prediction)
    assert len(m4.clusterCenters()) == 3 and len(np.unique(p4[1000:])) == 1


def test_undivided_active_cluster_is_a_permanent_leaf():
    """Level 2 needs one split (k = 3) and divides P; Q leaves the active set for good, so k = 4
    continues from P's children only (level 3), never returning to Q."""
    X, f = _pq_frame()
    m = BisectingKMeans(k=4, seed=7).fit(f)
    pred = np.asarray(m.transform(f).toPandas().prediction)
    assert len(m.clusterCenters()) == 4
    assert len(np.unique(pred[1000:])) == 2          # Q was divided on level 2 (needed = 2 there)
    m3 = BisectingKMeans(k=3, seed=7).fit(f)
    # tree shapes: internal nodes carry negative indices, leaves 0..k-1 in left-first order
    idx = sorted(nd.index for nd in m3._nodes())
    assert idx == [-2, -1, 0, 1, 2]


def test_save_layout_is_spark_ml_plus_mllib(tmp_path):
    import json
    import os
    import pyarrow.parquet as pq
    X, f = _pq_frame(300, 60)
    m = BisectingKMeans(k=3, seed=7).fit(f)
    p = str(tmp_path / "bkm")
    m.write().overwrite().save(p)
    with open(os.path.join(p, "metadata", "part-00000")) as fh:
        assert json.loads(fh.readline())["class"] == "org.apache.spark.ml.clustering.BisectingKMeansModel"
    with open(os.path.join(p, "data", "metadata", "part-00000")) as fh:
        md = json.loads(fh.readline())
    assert md["class"] == "org.apache.spark.mllib.clustering.BisectingKMeansModel" and md["version"] == "3.0"
    assert md["rootId"] == -1 and md["k"] == 3
    np.testing.assert_allclose(md["trainingCost"], m.trainingCost)
    files = [x for x in os.listdir(os.path.join(p, "data", "data")) if x.endswith(".parquet")]
    t = pq.read_table(os.path.join(p, "data", "data", files[0]))
    assert t.column_names == ["index", "size", "center", "norm", "cost", "height", "children"]
    rows = {r["index"]: r for r in t.to_pylist()}
    assert rows[-1]["size"] == 420 and len(rows[-1]["children"]) == 2 and rows[-1]["height"] > 0
    back = BisectingKMeansModel.load(p)
    np.testing.assert_array_equal(np.asarray(back.transform(f).toPandas().prediction),
                                  np.asarray(m.transform(f).toPandas().prediction))
    assert m.summary.k == 3 and sum(m.summary.clusterSizes) == 420
