"""The public KMeans fit on the device path (round 4): a tol > 0 fit decides convergence on the device and
reads the flag lagged (frozen steps after convergence are exact no-ops), so it equals the synchronous
loop bit for bit — iteration count, centres, labels, trainingCost; summary.clusterSizes is lazy and
comes from one pruned assign against the final centres, equal to counting a full assign's labels."""
import numpy as np
import pytest
import torch

from clustermachinelearningforhospitalnetworks_apache_spark_amd.models.kmeans import LloydEngine

pytestmark = pytest.mark.gpu


def _blobs(n, d, k, seed, scale=3.0, offset=0.0):
    g = torch.Generator(device="cuda").manual_seed(seed)
    cen = torch.randn(k, d, generator=g, device="cuda") * scale
    lab = torch.randint(0, k, (n,), generator=g, device="cuda")
    return (cen[lab] + torch.randn(n, d, generator=g, device="cuda") + offset).to(torch.bfloat16)


@pytest.mark.parametrize("n,d,k,tol,scale,must", [(200_003, 256, 64, 1e3, 3.0, True),  # converged at step 1
                                                  (90_000, 512, 100, 0.5, 2.0, True),
                                                  (150_000, 128, 32, 0.05, 0.7, False),
                                                  (120_000, 256, 16, 1e-4, 1.0, False)])
def test_lagged_tol_fit_equals_synchronous(monkeypatch, n, d, k, tol, scale, must):
    x = _blobs(n, d, k, seed=n, scale=scale)
    res = {}
    for lagged in ("0", "1"):
        monkeypatch.setenv("CML_KMEANS_LAGGED_TOL", lagged)
        eng = LloydEngine(x, d, k)
        assert eng._pdev
        eng.set_centers(eng.init_kmeans_parallel(seed=5))
        iters = eng.fit(40, tol)
        res[lagged] = (iters, eng.centers.cpu().numpy(), eng.labels[:n].clone(), eng.training_cost(),
                       eng.cluster_sizes())
        # the engine is live again after a lagged fit: one more step moves on from the same state
        assert int(eng._pst.done.item()) == 0
    (i0, c0, l0, t0, s0), (i1, c1, l1, t1, s1) = res["0"], res["1"]
    assert i0 == i1 and (i0 < 40 or not must), (i0, i1)
    if tol >= 1e3:
        assert i0 == 1
    assert np.array_equal(c0, c1)
    assert torch.equal(l0, l1)
    assert t0 == t1
    assert s0 == s1


@pytest.mark.parametrize("n,d,k", [(300_001, 256, 128), (80_000, 128, 40)])
def test_cluster_sizes_from_pruned_final_assign(n, d, k):
    x = _blobs(n, d, k, seed=7, scale=1.5)
    eng = LloydEngine(x, d, k)
    eng.set_centers(eng.init_kmeans_parallel(seed=3))
    eng.fit(6, 0.0)
    lab_state = eng.labels[:n].clone()
    ub_state = eng._pst.ub.clone()
    fast = eng.final_labels()
    full, _ = eng.assign()  # a full K9 pass against the final centres
    assert torch.equal(fast.long(), full.long())
    assert torch.equal(eng.labels[:n], lab_state) and torch.equal(eng._pst.ub, ub_state)  # state untouched
    want = torch.bincount(full.long(), minlength=k).tolist()
    assert eng.cluster_sizes() == want
    eng.step()  # the engine steps on normally after the read
    # the fit's own last use consumes the step state in place: same sizes, and the engine refuses to step on
    cost_before = eng.last_cost
    want2 = torch.bincount(eng.assign()[0].long(), minlength=k).tolist()
    assert eng.cluster_sizes_async(consume=True)() == want2
    assert torch.equal(eng.last_cost, cost_before)
    with pytest.raises(RuntimeError, match="consumed"):
        eng.step()


def test_estimator_fit_lazy_sizes_and_offset_cost():
    """KMeans.fit through a session frame: trainingCost on data offset by +300 equals the f64 oracle of
    the last iteration's assignment; clusterSizes (lazy) equals the counts of transform's predictions."""
    from clustermachinelearningforhospitalnetworks_apache_spark_amd.ml.clustering import KMeans
    from clustermachinelearningforhospitalnetworks_apache_spark_amd.sql import SparkSession
    spark = SparkSession.builder.master("mi355x").getOrCreate()
    n, d, k = 250_000, 256, 32
    x = _blobs(n, d, k, seed=21, scale=2.0, offset=300.0)
    df = spark.createDataFrameFromTensors({"features": x})
    m = KMeans(k=k, seed=9, maxIter=8, tol=0.0).fit(df)
    assert callable(m.summary._sizes)  # not counted during fit
    pred = m.transform(df)._numeric("prediction").long()
    assert m.summary.clusterSizes == torch.bincount(pred, minlength=k).tolist()
    # oracle: refit the same way on an engine and evaluate its last assignment in f64
    eng = LloydEngine(x, d, k)
    eng.set_centers(eng.init_kmeans_parallel(seed=9))
    eng.fit(8, 0.0)
    cb = eng._pst.cb_cost[:k, :d].double()
    ref = float(((x[:, :d].double() - cb[eng.labels[:n].long()]) ** 2).sum())
    assert abs(m.summary.trainingCost - ref) <= 1e-9 * ref
