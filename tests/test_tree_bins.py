"""Bin codes above 256 bins: maxBins > 256 must not wrap the uint8 codes.

A single step at x > 0.9 is recovered exactly whatever maxBins is (Spark accepts any maxBins >= 2);
the GPU variants check the 16-bit codes, the node-chunked LDS histograms and the direct
global-histogram path against the float64 CPU engine."""
import numpy as np
import pytest
import torch

from clustermachinelearningforhospitalnetworks_apache_spark_amd.models import trees as TR


def _step_data(n=5000, seed=0):
    rs = np.random.RandomState(seed)
    x = torch.as_tensor(rs.rand(n, 1))
    y = (x[:, 0] > 0.9).double() * 10.0
    return x, y


@pytest.mark.parametrize("max_bins", [32, 255, 256, 257, 300, 600, 4000])
def test_step_split_any_maxbins(max_bins):
    x, y = _step_data()
    p = TR.TreeParams(max_depth=1, max_bins=max_bins)
    eng = TR.ForestEngine(x, y, p)
    root = eng.fit()[0]
    assert root.feature == 0
    assert abs(root.threshold - 0.9) < 0.01, root.threshold
    assert eng.bins.dtype == (torch.uint8 if eng.nbins <= 256 else torch.int16)
    assert 0 <= int(eng.bins.long().min()) and int(eng.bins.long().max()) < eng.nbins
    left, right = root.left.count, root.right.count
    assert left + right == 5000 and right == int((x[:, 0] > root.threshold).sum())


def test_maxbins_out_of_range():
    x, y = _step_data(100)
    with pytest.raises(ValueError):
        TR.ForestEngine(x, y, TR.TreeParams(max_bins=TR.MAX_BINS + 1))
    with pytest.raises(ValueError):
        TR.ForestEngine(x, y, TR.TreeParams(max_bins=1))


def _compare(cpu, gpu):
    for a, b in zip(cpu, gpu):
        na, nb = TR.preorder(a), TR.preorder(b)
        assert len(na) == len(nb)
        for u, v in zip(na, nb):
            assert u.feature == v.feature and u.split_bin == v.split_bin
            np.testing.assert_allclose(u.stats, v.stats, rtol=1e-9, atol=1e-9)


@pytest.mark.gpu
@pytest.mark.parametrize("max_bins,depth,task", [(600, 5, "regression"), (300, 5, "classification"),
                                                 (6000, 2, "regression")])
def test_gpu_large_maxbins_matches_cpu(max_bins, depth, task):
    """600 bins x 32 nodes x 3 stats exceeds the LDS budget per feature (node-chunked histograms);
    6000 bins x 3 stats exceeds it per (node, feature) (direct global integer adds)."""
    torch.manual_seed(4)
    n, d = 30000, 5
    x = torch.randn(n, d, dtype=torch.float64)
    if task == "regression":
        y = x[:, 0] * 2 + (x[:, 1] > 0.3).double() + torch.randn(n, dtype=torch.float64) * 0.1
        imp = "variance"
    else:
        y = ((x[:, 0] + x[:, 2] * 0.5) > 0).double()
        imp = "gini"
    p = TR.TreeParams(task=task, num_classes=2, impurity=imp, max_depth=depth, max_bins=max_bins, seed=3)
    ce, ge = TR.ForestEngine(x, y, p), TR.ForestEngine(x.cuda(), y.cuda(), p)
    cpu, gpu = ce.fit(), ge.fit()
    assert ge.bins.dtype == torch.int16
    assert torch.equal(ge.bins.cpu(), ce.bins)
    _compare(cpu, gpu)


@pytest.mark.gpu
def test_gpu_binize_wide_table():
    """d * max_splits doubles beyond 64 KiB: thresholds are read from global memory."""
    torch.manual_seed(5)
    n, d = 4000, 300
    x = torch.randn(n, d, dtype=torch.float64)
    y = x[:, 7] + torch.randn(n, dtype=torch.float64) * 0.1
    p = TR.TreeParams(max_depth=2, max_bins=64)
    ce, ge = TR.ForestEngine(x, y, p), TR.ForestEngine(x.cuda(), y.cuda(), p)
    sp = ce.find_splits()
    assert torch.equal(ge.binize(sp).cpu(), ce.binize(sp))
