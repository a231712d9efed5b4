"""GPU numerics of the GLM (K7/K8/K13/K15/K24) and tree (K17/K18/K20/K21) kernels vs the
float64 torch references of the same ops (the CPU code paths)."""
import numpy as np
import pytest
import torch

from clustermachinelearningforhospitalnetworks_apache_spark_amd.models import trees as TR
from clustermachinelearningforhospitalnetworks_apache_spark_amd.ops import glm_ops

pytestmark = pytest.mark.gpu
DT = [torch.float64, torch.float32, torch.bfloat16]
DT_IN = DT + [torch.float8_e4m3fn]  # fp8 storage (SURVEY config 5) is an input dtype only


@pytest.mark.parametrize("dtype", DT_IN)
@pytest.mark.parametrize("n,d", [(1000, 4), (5000, 37), (20000, 256), (3000, 600), (7, 1)])
def test_moments_and_scale(dtype, n, d):
    torch.manual_seed(0)
    x = (torch.randn(n, d, dtype=torch.float64) * 3 + 5).to(dtype)
    xc, xg = x, x.cuda()
    nc, s1c, s2c, shc = glm_ops.moments(xc, d)
    ng, s1g, s2g, shg = glm_ops.moments(xg, d)
    assert nc == ng
    tol = 1e-9 if dtype == torch.float64 else 1e-6
    np.testing.assert_allclose(s1g.cpu().numpy(), s1c.numpy(), rtol=tol, atol=tol * n * 10)
    np.testing.assert_allclose(s2g.cpu().numpy(), s2c.numpy(), rtol=tol, atol=tol * n * 10)
    mean = torch.randn(d, dtype=torch.float64)
    inv = torch.rand(d, dtype=torch.float64) + 0.5
    for od in DT:
        yc = glm_ops.scale_apply(xc, d, mean, inv, True, od)
        yg = glm_ops.scale_apply(xg, d, mean.cuda(), inv.cuda(), True, od)
        np.testing.assert_allclose(yg.cpu().double().numpy(), yc.double().numpy(),
                                   rtol=1e-2 if od == torch.bfloat16 else 1e-6, atol=1e-2)


@pytest.mark.parametrize("dtype", DT_IN)
@pytest.mark.parametrize("n,d", [(1000, 4), (4097, 31), (20000, 256), (3000, 513)])
def test_logreg_grad_and_predict(dtype, n, d):
    torch.manual_seed(1)
    x = torch.randn(n, d, dtype=torch.float64).to(dtype)
    y = (torch.rand(n) > 0.5).double()
    w = torch.rand(n, dtype=torch.float64) + 0.5
    coef = torch.randn(d + 1, dtype=torch.float64) * 0.1
    for wt in (None, w):
        oc = glm_ops.logreg_grad(x, d, y, coef, wt)
        og = glm_ops.logreg_grad(x.cuda(), d, y.cuda(), coef.cuda(), None if wt is None else wt.cuda())
        np.testing.assert_allclose(og.cpu().numpy(), oc.numpy(), rtol=1e-8 if dtype == torch.float64 else 2e-6, atol=(1e-8 if dtype == torch.float64 else 2e-6) * n)
    for link in ("identity", "logistic"):
        pc = glm_ops.linear_predict(x, d, coef, link)
        pg = glm_ops.linear_predict(x.cuda(), d, coef.cuda(), link)
        np.testing.assert_allclose(pg.cpu().numpy(), pc.numpy(), rtol=1e-9 if dtype == torch.float64 else 1e-6, atol=1e-9 if dtype == torch.float64 else 1e-5)


@pytest.mark.parametrize("dtype", DT_IN)
@pytest.mark.parametrize("n,d", [(1000, 4), (50000, 12), (3000, 30)])
def test_gram(dtype, n, d):
    torch.manual_seed(2)
    x = torch.randn(n, d, dtype=torch.float64).to(dtype)
    y = torch.randn(n, dtype=torch.float64)
    w = torch.rand(n, dtype=torch.float64)
    for wt in (None, w):
        gc = glm_ops.gram(x, d, y, wt)
        gg = glm_ops.gram(x.cuda(), d, y.cuda(), None if wt is None else wt.cuda())
        np.testing.assert_allclose(gg.cpu().numpy(), gc.numpy(), rtol=1e-10, atol=1e-8)


@pytest.mark.parametrize("task", ["regression", "classification"])
@pytest.mark.parametrize("trees", [1, 7])
def test_forest_gpu_matches_cpu(task, trees):
    torch.manual_seed(3)
    n, d = 6000, 6
    x = torch.randn(n, d, dtype=torch.float64)
    if task == "regression":
        y = x[:, 0] * 2 + (x[:, 1] > 0).double() + torch.randn(n, dtype=torch.float64) * 0.1
        imp = "variance"
    else:
        y = ((x[:, 0] + x[:, 2] * 0.5) > 0).double() + (x[:, 3] > 1).double()
        imp = "gini"
    p = TR.TreeParams(task=task, num_classes=3, impurity=imp, num_trees=trees, seed=11,
                      feature_subset="auto")
    cpu = TR.ForestEngine(x, y, p).fit()
    gpu = TR.ForestEngine(x.cuda(), y.cuda(), p).fit()
    for a, b in zip(cpu, gpu):
        na, nb = TR.preorder(a), TR.preorder(b)
        assert len(na) == len(nb)
        for u, v in zip(na, nb):
            assert u.feature == v.feature and u.split_bin == v.split_bin
            # same int64 fixed-point histograms on both paths (models/trees.py histogram): exact stats
            assert np.array_equal(u.stats, v.stats)
    kind = imp
    pc = TR.predict_forest(cpu, x, kind, 3, average=True, normalize_leaves=trees > 1)
    pg = TR.predict_forest(gpu, x.cuda(), kind, 3, average=True, normalize_leaves=trees > 1)
    assert torch.equal(pg.cpu(), pc)  # same leaves summed in the same tree order


@pytest.mark.parametrize("imp", ["variance", "entropy", "gini"])
def test_forest_gpu_matches_cpu_wide(imp):
    """40 features, 12 trees with per-node feature subsets: the GPU K19 best-split kernel (fixed-point
    histogram) and the vectorised CPU rule grow the same forests."""
    torch.manual_seed(9)
    n, d = 20000, 40
    x = torch.randn(n, d, dtype=torch.float64)
    task = "regression" if imp == "variance" else "classification"
    if task == "regression":
        y = x[:, 3] * 2 + (x[:, 17] > 0).double() - x[:, 29] + torch.randn(n, dtype=torch.float64) * 0.1
    else:
        y = ((x[:, 5] + x[:, 11] * 0.5) > 0).double() + (x[:, 30] > 0.5).double()
    p = TR.TreeParams(task=task, num_classes=3, impurity=imp, num_trees=12, seed=5, feature_subset="onethird")
    cpu = TR.ForestEngine(x, y, p).fit()
    gpu = TR.ForestEngine(x.cuda(), y.cuda(), p).fit()
    for a, b in zip(cpu, gpu):
        na, nb = TR.preorder(a), TR.preorder(b)
        assert len(na) == len(nb)
        for u, v in zip(na, nb):
            assert u.feature == v.feature and u.split_bin == v.split_bin
            assert np.array_equal(u.stats, v.stats)
            if u.feature >= 0:
                np.testing.assert_allclose(u.gain, v.gain, rtol=1e-9, atol=1e-12)


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float64])
def test_sgd_graph_replay_matches_eager(dtype):
    """The captured SGD step (device-side batch offset, K13 + update in one HIP graph) equals the
    eager step bit for bit, and both match a CPU float64 run to within the kernel's precision."""
    from clustermachinelearningforhospitalnetworks_apache_spark_amd.models.sgd import LogisticSGD
    from clustermachinelearningforhospitalnetworks_apache_spark_amd.parallel.comm import local_comm
    torch.manual_seed(8)
    n, d = 40_000, 24
    x = torch.randn(n, d, dtype=torch.float64)
    y = ((x[:, 0] + 0.5 * x[:, 1]) > 0).double()
    runs = {}
    for dev, g in (("cuda", False), ("cuda", True), ("cpu", False)):
        xx = x.to(dtype) if dev == "cuda" else x.to(dtype).double()
        opt = LogisticSGD(xx.to(dev), d, y.to(dev), None, local_comm(), 4096, 0.5, 0.9, use_graph=g)
        for _ in range(35):  # > one pass: the device batch offset wraps around
            opt.step()
        runs[(dev, g)] = opt.coef.cpu()
    assert torch.equal(runs[("cuda", False)], runs[("cuda", True)])
    tol = 1e-9 if dtype == torch.float64 else 1e-3
    np.testing.assert_allclose(runs[("cuda", True)].numpy(), runs[("cpu", False)].numpy(), rtol=tol, atol=tol)


@pytest.mark.parametrize("nb,m", [(1, 3), (17, 259), (512, 259), (1024, 1030)])
def test_partial_colsum_matches_torch(nb, m):
    part = torch.randn(nb, m, dtype=torch.float64, device="cuda")
    got = glm_ops.partial_colsum(part)
    torch.testing.assert_close(got.cpu(), part.cpu().sum(0), rtol=1e-12, atol=1e-12)
    assert torch.equal(got, glm_ops.partial_colsum(part))  # fixed order: bitwise repeatable


@pytest.mark.parametrize("S", [2, 3, 7])
@pytest.mark.parametrize("thr", [None, "set"])
def test_forest_vote_kernel_matches_torch(S, thr):
    """K21b (class distribution + thresholded first argmax) against the host rule it replaces, including
    rows whose leaf counts sum to zero (uniform distribution) and exact ties (first maximum)."""
    g = torch.Generator().manual_seed(S)
    n = 5000
    raw = torch.randint(0, 4, (n, S), generator=g).to(torch.float64)
    raw[::97] = 0.0
    t = list(np.linspace(0.3, 0.9, S)) if thr else None
    pc, yc = TR.forest_vote(raw, t)
    pg, yg = TR.forest_vote(raw.cuda(), t)
    assert torch.equal(pg.cpu(), pc)
    assert torch.equal(yg.cpu(), yc)
