"""BucketedRandomProjectionLSH / MinHashLSH: hash definitions, nearest neighbours and similarity
joins vs brute force, java.util.Random coefficient draws, persistence."""
import numpy as np
import pytest

from helpers import session
from clustermachinelearningforhospitalnetworks_apache_spark_amd.ml import util as U
from clustermachinelearningforhospitalnetworks_apache_spark_amd.ml.bisecting import JavaRandom
from clustermachinelearningforhospitalnetworks_apache_spark_amd.ml.feature import (
    BucketedRandomProjectionLSH, MinHashLSH, MinHashLSHModel, VectorAssembler)


@pytest.fixture(scope="module")
def spark():
    return session()


def _frame(spark, X):
    cols = [f"c{j}" for j in range(X.shape[1])]
    df = spark.createDataFrame([(i,) + tuple(float(v) for v in r) for i, r in enumerate(X)],
                               "id INT, " + ", ".join(f"{c} DOUBLE" for c in cols))
    return VectorAssembler(inputCols=cols, outputCol="f").transform(df)


def test_java_random_known_values():
    # java.util.Random(42): nextInt(10) x 5 and the first nextGaussian
    r = JavaRandom(42)
    assert [r.next_int(10) for _ in range(5)] == [0, 3, 8, 4, 0]
    assert JavaRandom(42).next_gaussian() == pytest.approx(1.1419053154730547, rel=1e-15)


def test_brp_lsh(spark, tmp_path):
    rs = np.random.RandomState(0)
    X = rs.normal(size=(80, 3))
    df = _frame(spark, X)
    m = BucketedRandomProjectionLSH(inputCol="f", outputCol="h", bucketLength=2.0, numHashTables=3, seed=7).fit(df)
    h = m.transform(df).toPandas()["h"]
    R = m._R
    np.testing.assert_allclose(np.linalg.norm(R, axis=1), 1.0)
    np.testing.assert_array_equal(np.array([[v[0] for v in row] for row in h]), np.floor(X @ R.T / 2.0))
    key = X[5] + 0.01
    nn = m.approxNearestNeighbors(df, key, 4).toPandas()
    d = np.linalg.norm(X - key, axis=1)
    hk = np.floor(key @ R.T / 2.0)
    cand = (np.floor(X @ R.T / 2.0) == hk).any(1)
    want = np.argsort(np.where(cand, d, np.inf))[:min(4, cand.sum())]
    assert list(nn["id"]) == list(want)
    np.testing.assert_allclose(nn["distCol"], d[want])
    wide = BucketedRandomProjectionLSH(inputCol="f", outputCol="h", bucketLength=1e6, seed=1).fit(df)
    j = wide.approxSimilarityJoin(df, df, 0.5).collect()
    hw = np.floor(X @ wide._R.T / 1e6)
    brute = {(a, b) for a in range(80) for b in range(80)
             if np.linalg.norm(X[a] - X[b]) < 0.5 and (hw[a] == hw[b]).any()}
    assert len(brute) > 80
    assert {(r.datasetA.id, r.datasetB.id) for r in j} == brute
    p = str(tmp_path / "brp")
    m.write().overwrite().save(p)
    np.testing.assert_allclose(U.load(p)._R, R)


def test_minhash_lsh(spark, tmp_path):
    rs = np.random.RandomState(1)
    X = (rs.rand(40, 12) < 0.3).astype(float)
    X[:, 0] = 1.0  # at least one non-zero per row
    df = _frame(spark, X)
    m = MinHashLSH(inputCol="f", outputCol="h", numHashTables=4, seed=11).fit(df)
    r = JavaRandom(11)
    want = []
    for _ in range(4):
        a = 1 + r.next_int(2038074743 - 1)
        b = r.next_int(2038074743 - 1)
        want.append((a, b))
    assert m._coefs == want
    h = np.array([[v[0] for v in row] for row in m.transform(df).toPandas()["h"]])
    for i in range(5):
        nz = np.nonzero(X[i])[0]
        for t, (a, b) in enumerate(want):
            assert h[i, t] == min(((1 + j) * a + b) % 2038074743 for j in nz)
    key = X[3]
    nn = m.approxNearestNeighbors(df, key, 3).toPandas()
    assert nn["id"].iloc[0] == 3 and nn["distCol"].iloc[0] == 0.0
    sets = [set(np.nonzero(x)[0]) for x in X]
    jac = lambda a, b: 1 - len(a & b) / len(a | b)  # noqa: E731
    for _, row in nn.iterrows():
        assert row["distCol"] == pytest.approx(jac(sets[row["id"]], sets[3]))
    p = str(tmp_path / "mh")
    m.write().overwrite().save(p)
    assert MinHashLSHModel.load(p)._coefs == want
