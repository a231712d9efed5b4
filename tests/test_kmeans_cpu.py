"""CPU (local-mode) Lloyd engine vs a plain numpy Lloyd from the same init."""
import numpy as np
import torch

from clustermachinelearningforhospitalnetworks_apache_spark_amd.models.kmeans import LloydEngine, local_kmeans_pp
from clustermachinelearningforhospitalnetworks_apache_spark_amd.utils import rng


def numpy_lloyd(x, c, iters):
    for _ in range(iters):
        d = ((x[:, None, :] - c[None]) ** 2).sum(2)
        lab = d.argmin(1)
        new = c.copy()
        for j in range(c.shape[0]):
            m = lab == j
            if m.any():
                new[j] = x[m].mean(0)
        c = new
    return c


def test_engine_matches_numpy():
    rs = np.random.RandomState(0)
    x = rs.randn(2000, 5) * 2
    init = x[:7].copy()
    eng = LloydEngine(torch.as_tensor(x), 5, 7)
    eng.set_centers(init)
    for _ in range(5):
        eng.step()
    np.testing.assert_allclose(eng.centers.numpy(), numpy_lloyd(x, init, 5), rtol=1e-10, atol=1e-10)


def test_kmeans_parallel_init_finds_blobs():
    rs = np.random.RandomState(1)
    true = rs.randn(4, 3) * 20
    x = true[rs.randint(0, 4, 4000)] + rs.randn(4000, 3)
    eng = LloydEngine(torch.as_tensor(x), 3, 4)
    init = eng.init_kmeans_parallel(seed=3)
    eng.set_centers(init)
    eng.fit(20, 1e-4)
    got = eng.centers.numpy()
    dmin = np.sqrt(((true[:, None] - got[None]) ** 2).sum(2)).min(1)
    assert dmin.max() < 0.5


def test_local_kmeans_pp_weighted():
    pts = np.array([[0.0, 0], [0.1, 0], [10, 10], [10.1, 10]])
    c = local_kmeans_pp(pts, np.array([1.0, 1, 1, 1]), 2, seed=0)
    assert sorted(np.round(c[:, 0]).tolist()) == [0.0, 10.0]


def test_rng_is_deterministic_and_uniform():
    ids = torch.arange(200000)
    u1 = rng.uniform(ids, 42)
    u2 = rng.uniform(ids, 42)
    assert torch.equal(u1, u2)
    assert 0.49 < u1.mean().item() < 0.51
    assert u1.min() >= 0 and u1.max() < 1
    p = rng.poisson1(ids, 7).double()
    assert abs(p.mean().item() - 1.0) < 0.01 and abs(p.var().item() - 1.0) < 0.02


def test_local_kmeans_pp_device_variant_matches_host():
    import torch
    from clustermachinelearningforhospitalnetworks_apache_spark_amd.models.kmeans import local_kmeans_pp_device
    rs = np.random.RandomState(4)
    pts = rs.randn(400, 6) + rs.randint(0, 6, (400, 1)) * 4.0
    w = rs.rand(400) * 5
    a = local_kmeans_pp(pts, w, 9, seed=11)
    b = local_kmeans_pp_device(torch.as_tensor(pts), torch.as_tensor(w), 9, seed=11)
    np.testing.assert_allclose(a, b, rtol=1e-12, atol=1e-12)


def numpy_spherical_lloyd(x, c, iters):
    """Spark CosineDistanceMeasure Lloyd: argmax cos, centre = normalised mean of the unit rows."""
    u = x / np.linalg.norm(x, axis=1, keepdims=True)
    for _ in range(iters):
        lab = (u @ c.T).argmax(1)
        new = c.copy()
        for j in range(c.shape[0]):
            m = lab == j
            if m.any():
                s = u[m].sum(0)
                new[j] = s / np.linalg.norm(s)
        c = new
    return c, (1.0 - (u * c[lab]).sum(1)).sum()


def _directions(n, d, k, seed):
    rs = np.random.RandomState(seed)
    dirs = rs.randn(k, d)
    dirs /= np.linalg.norm(dirs, axis=1, keepdims=True)
    x = dirs[rs.randint(0, k, n)] + 0.15 * rs.randn(n, d)
    return x * rs.uniform(0.1, 50.0, (n, 1))  # magnitudes must not matter under the cosine measure


def test_spherical_engine_matches_numpy():
    x = _directions(3000, 6, 5, seed=4)
    u = x / np.linalg.norm(x, axis=1, keepdims=True)
    init = u[:5].copy()
    eng = LloydEngine(torch.as_tensor(x), 6, 5, spherical=True)
    eng.set_centers(init)
    for _ in range(6):
        eng.step()
    ref_c, _ = numpy_spherical_lloyd(x, init, 6)
    np.testing.assert_allclose(eng.centers.numpy(), ref_c, rtol=1e-10, atol=1e-10)
    np.testing.assert_allclose(np.linalg.norm(eng.centers.numpy(), axis=1), 1.0, rtol=1e-12)
    # the reported cost is the cost of the assignment made in the last step (against the step's input centres)
    prev_c, _ = numpy_spherical_lloyd(x, init, 5)
    lab = (u @ prev_c.T).argmax(1)
    np.testing.assert_allclose(eng.training_cost(), (1.0 - (u * prev_c[lab]).sum(1)).sum(), rtol=1e-9)


def test_cosine_kmeans_estimator_scale_invariant():
    import pandas as pd
    from helpers import session
    spark = session()
    from clustermachinelearningforhospitalnetworks_apache_spark_amd.ml.clustering import KMeans, KMeansModel
    from clustermachinelearningforhospitalnetworks_apache_spark_amd.ml.feature import VectorAssembler
    x = _directions(2000, 4, 3, seed=5)
    cols = [f"f{i}" for i in range(4)]
    rs = np.random.RandomState(9)
    scaled = x * rs.uniform(0.5, 4.0, (x.shape[0], 1))
    models = []
    for data in (x, scaled):
        df = VectorAssembler(inputCols=cols, outputCol="features").transform(
            spark.createDataFrame(pd.DataFrame(data, columns=cols)))
        m = KMeans(k=3, seed=1, distanceMeasure="cosine", maxIter=30).fit(df)
        pred = np.asarray(m.transform(df).select("prediction").toPandas()["prediction"])
        models.append((m, pred, df))
    (m0, p0, df0), (m1, p1, _) = models
    np.testing.assert_array_equal(p0, p1)
    np.testing.assert_allclose(np.stack(m0.clusterCenters()), np.stack(m1.clusterCenters()), atol=1e-9)
    c = np.stack(m0.clusterCenters())
    np.testing.assert_allclose(np.linalg.norm(c, axis=1), 1.0, rtol=1e-9)
    u = x / np.linalg.norm(x, axis=1, keepdims=True)
    np.testing.assert_array_equal(p0, (u @ c.T).argmax(1))
    cost = (1.0 - (u * c[p0]).sum(1)).sum()
    np.testing.assert_allclose(m0.computeCost(df0), cost, rtol=1e-9)
    assert m0.predict(x[0] * 7.0) == p0[0]
    assert m0.summary.trainingCost >= 0
    # the measure travels with the saved model
    import tempfile
    with tempfile.TemporaryDirectory() as d:
        m0.write().overwrite().save(d + "/m")
        m2 = KMeansModel.load(d + "/m")
        assert m2.getOrDefault("distanceMeasure") == "cosine"
        np.testing.assert_array_equal(np.asarray(m2.transform(df0).select("prediction").toPandas()["prediction"]), p0)


def test_cosine_rejects_zero_rows():
    import pytest
    x = np.ones((10, 3))
    x[4] = 0.0
    with pytest.raises(ValueError, match="zero-length"):
        LloydEngine(torch.as_tensor(x), 3, 2, spherical=True)


def test_precision_modes_cpu():
    import pytest
    x = torch.as_tensor(np.random.RandomState(0).randn(100, 3))
    assert LloydEngine(x, 3, 2).precision == "exact"
    with pytest.raises(ValueError):
        LloydEngine(x, 3, 2, precision="fp16")


def test_candidate_chunks_cover_and_respect_limits():
    e = LloydEngine(torch.zeros(10, 4, dtype=torch.float64), 4, 2)
    e.dp = 256
    e.x = torch.zeros(1, 256, dtype=torch.bfloat16)
    for m in (1, 63, 64, 255, 256, 300, 511, 512, 520, 641, 1025, 3000):
        ch = LloydEngine._candidate_chunks(e, m)
        assert sum(ch) == m and all(0 < c <= 320 for c in ch)
        assert all(c % 64 == 0 for c in ch[:-1])
