"""Exact sums are correctly rounded (round 4): double-double accumulation makes the per-cluster sums the
rounded exact sums, independent of the order of the additions — so the host twin, the device kernel, the
certified step's incremental deltas and any partitioning over ranks give the same bits."""
import math

import numpy as np
import pytest
import torch

from clustermachinelearningforhospitalnetworks_apache_spark_amd.ops import kmeans_ops as K


@pytest.mark.parametrize("n,d,k,dt", [(20_000, 5, 7, torch.float64), (9_001, 3, 4, torch.float32)])
def test_host_sums_are_correctly_rounded(n, d, k, dt):
    g = torch.Generator().manual_seed(n)
    # wide dynamic range and cancellation: a naive f64 sum loses bits here
    x = (torch.randn(n, d, generator=g, dtype=torch.float64) * torch.logspace(-6, 9, n, dtype=torch.float64)[:, None])
    x = x.to(dt)
    lab = torch.randint(0, k, (n,), generator=g)
    S, cnt, S_lo = K.sums_reference(x, lab, k, with_lo=True)
    xs = x.to(torch.float64).numpy()
    ln = lab.numpy()
    for c in range(k):
        rows = xs[ln == c]
        for t in range(d):
            assert S[c, t].item() == math.fsum(rows[:, t].tolist())
        assert cnt[c].item() == float((ln == c).sum())
    # any order: a permutation of the rows gives the same bits
    p = torch.randperm(n, generator=g)
    S2, _ = K.sums_reference(x[p], lab[p], k)
    assert torch.equal(S, S2)
    # the rank fold of two halves' double-double sums gives the one-rank bits
    h = n // 3
    a, _, al = K.sums_reference(x[:h], lab[:h], k, with_lo=True)
    b, _, bl = K.sums_reference(x[h:], lab[h:], k, with_lo=True)
    f = K.dd_fold(torch.stack([a, b]), torch.stack([al, bl]))
    assert torch.equal(f, S)


def test_dd_sums_exact_span_guard():
    """The f64 exponent-span guard of the auto screen: ordinary data passes, 1e-9 beside 1e9
    (span ~60 binades) does not; all-zero rows pass; the result is cached on the tensor."""
    import torch
    from clustermachinelearningforhospitalnetworks_apache_spark_amd.models.kmeans import dd_sums_exact
    from clustermachinelearningforhospitalnetworks_apache_spark_amd.parallel.comm import local_comm
    x = torch.randn(5000, 6, dtype=torch.float64)
    assert dd_sums_exact(x, 6, local_comm())
    x[1, 1], x[2, 2] = 1e-9, 1e9
    assert not dd_sums_exact(x, 6, local_comm())
    assert x._cml_f64span[1] == 6
    assert dd_sums_exact(torch.zeros(10, 3, dtype=torch.float64), 3, local_comm())
