"""precision "screen" (round 4, VERDICT r3 missing 1): f32/f64 feature rows fitted with the exact f64
algorithm's results — the same k-means|| init, labels, centres and trainingCost bit for bit as precision
"exact" (kmeans_exact.hip) and as the CPU f64 fit — with the assignments screened on MFMA: a bf16 K9r pass
with top-2 bounds, a certificate covering the bf16 rounding of rows and centres, f64 re-assignment of the
uncertified rows only."""
import numpy as np
import pytest
import torch

from clustermachinelearningforhospitalnetworks_apache_spark_amd.models.kmeans import LloydEngine
from clustermachinelearningforhospitalnetworks_apache_spark_amd.ops import kmeans_ops as K

pytestmark = pytest.mark.gpu


def _blobs(n, d, k, seed, scale, dtype, offset=0.0):
    g = torch.Generator().manual_seed(seed)
    cen = torch.randn(k, d, generator=g, dtype=torch.float64) * scale
    x = cen[torch.randint(0, k, (n,), generator=g)] + torch.randn(n, d, generator=g, dtype=torch.float64) + offset
    return x.to(dtype)


@pytest.mark.parametrize("n,d,k,scale,dt", [(120_000, 128, 64, 3.0, torch.float32),
                                            (60_003, 200, 40, 0.4, torch.float64),
                                            (40_000, 256, 100, 1.0, torch.float32)])
def test_screen_fit_equals_exact_fit(monkeypatch, n, d, k, scale, dt):
    monkeypatch.setenv("CML_KMEANS_INIT_PRUNE", "1")
    x = _blobs(n, d, k, seed=n, scale=scale, dtype=dt, offset=50.0).cuda()
    res = {}
    for prec in ("exact", "screen"):
        eng = LloydEngine(x, d, k, precision=prec)
        assert eng.precision == prec
        eng.track_prune = True
        init = eng.init_kmeans_parallel(seed=3)
        eng.set_centers(init)
        it = eng.fit(8, 0.0)
        res[prec] = (init, it, eng.centers.cpu().numpy(), eng.labels[:n].long().cpu(), eng.training_cost())
        if prec == "screen":
            rech = eng._scr.rechecked
            assert rech and max(rech) < n  # the screen certified rows
    (i0, t0, c0, l0, f0), (i1, t1, c1, l1, f1) = res["exact"], res["screen"]
    assert np.array_equal(i0, i1)
    assert t0 == t1 and np.array_equal(c0, c1) and torch.equal(l0, l1)
    assert f0 == f1


def test_screen_auto_matches_cpu_f64_fit():
    n, d, k = 30_000, 130, 12
    x = _blobs(n, d, k, seed=5, scale=2.0, dtype=torch.float64)
    cpu = LloydEngine(x, d, k)
    gpu = LloydEngine(x.cuda(), d, k)
    assert gpu.precision == "screen" and cpu.precision == "exact"
    for e in (cpu, gpu):
        e.set_centers(e.init_kmeans_parallel(seed=9))
        e.fit(10, 1e-6)
    assert np.array_equal(cpu.centers.numpy(), gpu.centers.cpu().numpy())
    assert abs(cpu.training_cost() - gpu.training_cost()) <= 1e-12 * cpu.training_cost()


def test_screen_kernels():
    n, d = 50_001, 130
    x = _blobs(n, d, 8, seed=1, scale=3.0, dtype=torch.float32).cuda()
    xb, ex = K.to_bf16_err(x, d, 256)
    assert xb.shape == (n, 256) and bool((xb[:, d:] == 0).all())
    assert torch.equal(xb[:, :d], x.to(torch.bfloat16))
    ref = (x.double() - xb[:, :d].double()).norm(dim=1)
    assert bool((ex.double() >= ref).all()) and bool((ex.double() <= ref * (1 + 1e-5) + 1e-20).all())
    C = torch.randn(9, d, dtype=torch.float64, device="cuda") * 3
    lab, best = K.exact_assign(x, C)
    b2 = torch.empty(n, dtype=torch.float64, device="cuda")
    K.exact_dist(x, C, lab, b2)
    assert torch.equal(best, b2[:n])
    # list-restricted assignment touches only the listed rows
    idx = torch.tensor([3, 77, n - 1], dtype=torch.int32, device="cuda")
    cnt = torch.tensor([3], dtype=torch.int32, device="cuda")
    l2 = torch.full((n,), -1, dtype=torch.int32, device="cuda")
    b3 = torch.full((n,), -1.0, dtype=torch.float64, device="cuda")
    K.exact_assign(x, C, labels=l2, idx=idx, n_dev=cnt, best=b3)
    sel = idx.long()
    assert torch.equal(l2[sel], lab[sel]) and torch.equal(b3[sel], best[sel])
    assert int((l2 >= 0).sum()) == 3
