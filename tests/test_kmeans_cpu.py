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
