"""ALS: recovers a low-rank rating matrix (explicit), implicit preferences rank observed items first,
cold-start strategies, top-N recommendations vs the factor products, Spark-layout persistence."""
import numpy as np
import pytest

from helpers import session
from clustermachinelearningforhospitalnetworks_apache_spark_amd.ml import util as U
from clustermachinelearningforhospitalnetworks_apache_spark_amd.ml.recommendation import ALS, ALSModel


@pytest.fixture(scope="module")
def spark():
    return session()


def _ratings(seed=0, nu=40, ni=30, k=2, frac=0.5):
    rs = np.random.RandomState(seed)
    Ut, Vt = rs.normal(size=(nu, k)), rs.normal(size=(ni, k))
    R = Ut @ Vt.T
    mask = rs.rand(nu, ni) < frac
    rows = [(int(u), int(i), float(R[u, i])) for u in range(nu) for i in range(ni) if mask[u, i]]
    return R, mask, rows


def test_als_explicit_recovers_low_rank(spark, tmp_path):
    R, mask, rows = _ratings()
    df = spark.createDataFrame(rows, "user INT, item INT, rating DOUBLE")
    m = ALS(rank=2, maxIter=15, regParam=1e-4, seed=1).fit(df)
    pred = m.transform(df).toPandas()
    rmse = np.sqrt(np.mean((pred["prediction"].astype(float) - pred["rating"]) ** 2))
    assert rmse < 0.05
    # held-out cells are predicted too (the matrix is rank 2)
    test = [(u, i, float(R[u, i])) for u in range(40) for i in range(30) if not mask[u, i]][:200]
    tp = m.transform(spark.createDataFrame(test, "user INT, item INT, rating DOUBLE")).toPandas()
    assert np.sqrt(np.mean((tp["prediction"].astype(float) - tp["rating"]) ** 2)) < 0.2
    # cold start
    cold = spark.createDataFrame([(999, 0, 1.0), (0, 0, 1.0)], "user INT, item INT, rating DOUBLE")
    cp = m.transform(cold).toPandas()["prediction"].tolist()
    assert np.isnan(cp[0]) and not np.isnan(cp[1])
    assert m.setColdStartStrategy("drop").transform(cold).count() == 1
    # recommendations = top-N of the factor products
    uf = {r.id: np.array(r.features) for r in m.userFactors.collect()}
    itf = {r.id: np.array(r.features) for r in m.itemFactors.collect()}
    recs = {r.user: r.recommendations for r in m.recommendForAllUsers(3).collect()}
    scores = {i: float(uf[5] @ itf[i]) for i in itf}
    best = sorted(scores, key=lambda i: -scores[i])[:3]
    assert [x.item for x in recs[5]] == best
    assert len(m.recommendForAllItems(2).collect()) == 30
    sub = m.recommendForUserSubset(spark.createDataFrame([(5,), (7,)], "user INT"), 2).collect()
    assert sorted(r.user for r in sub) == [5, 7]
    p = str(tmp_path / "als")
    m.write().overwrite().save(p)
    back = U.load(p)
    assert isinstance(back, ALSModel) and back.rank == 2
    np.testing.assert_allclose(back.transform(df).toPandas()["prediction"], pred["prediction"], rtol=1e-5, atol=1e-5)


def test_als_implicit_and_nonnegative(spark):
    rs = np.random.RandomState(3)
    rows = []
    for u in range(30):
        liked = rs.choice(20, 6, replace=False) if u < 15 else rs.choice(np.arange(10, 30), 6, replace=False)
        rows += [(u, int(i), float(rs.randint(1, 5))) for i in liked]
    df = spark.createDataFrame(rows, "user INT, item INT, rating DOUBLE")
    m = ALS(rank=4, maxIter=10, implicitPrefs=True, alpha=5.0, regParam=0.05, seed=2).fit(df)
    pred = m.transform(df).toPandas()["prediction"].astype(float)
    assert pred.mean() > 0.5  # observed (preferred) items score high
    nn = ALS(rank=3, maxIter=5, nonnegative=True, seed=2).fit(df)
    assert min(min(r.features) for r in nn.userFactors.collect()) >= 0.0
