"""Device k-means|| initialisation (``kmeans_init.hip``) against torch / host references: the fused
row pass (norms vs f64, bitwise equal between the fused and the norms-only launch; first costs,
max norm, exponent range), the
sampling and merge kernels, the local k-means kernels against their host twin (bit for bit), and a
whole init on exactly-representable data equal to the CPU session's."""
import numpy as np
import pytest
import torch

from clustermachinelearningforhospitalnetworks_apache_spark_amd.models.kmeans import LloydEngine, to_device_matrix
from clustermachinelearningforhospitalnetworks_apache_spark_amd.ops import kmeans_ops as K
from clustermachinelearningforhospitalnetworks_apache_spark_amd.utils import rng

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("n,d,fp8", [(100_003, 256, False), (7, 16, False), (65_537, 128, False),
                                     (30_001, 512, False), (50_000, 256, True), (9_999, 512, True)])
def test_row_pass_matches_norm_kernel(n, d, fp8):
    g = torch.Generator(device="cuda").manual_seed(n)
    xf = torch.randn(n, d, device="cuda", generator=g) * 3
    xf[::7, 3] = 0.0
    xf[5, 1] = 1e-30  # a tiny exponent
    x = to_device_matrix(xf.to(torch.float8_e4m3fn) if fp8 else xf, d)
    dp = x.shape[1]
    ref = K.row_sqnorm(x, n, dp)  # norms-only launch of the same kernel
    xd0 = (x.view(torch.uint8)[:, :d].view(torch.float8_e4m3fn) if fp8 else x[:, :d]).double()
    torch.testing.assert_close(ref.double(), (xd0 * xd0).sum(1), rtol=2e-6, atol=1e-30)
    xn = torch.empty(n, device="cuda")
    c0 = torch.zeros(dp, device="cuda")
    c0[:d] = xf[1].to(torch.bfloat16).float()
    c0n = float((c0.double() ** 2).sum())
    cost = torch.empty(n, device="cuda")
    near = torch.full((n,), 5, dtype=torch.int32, device="cuda")
    mx = torch.zeros(1, device="cuda")
    er = torch.tensor([2 ** 31 - 1, -1], dtype=torch.int32, device="cuda")
    K.row_pass(x, n, dp, xn, c0, c0n, cost, near, xn_max=mx, erange=er)
    torch.cuda.synchronize()
    assert torch.equal(xn, ref)
    assert float(mx) == float(ref.max())
    assert bool((near == 0).all())
    xd = (x.view(torch.uint8)[:, :d].view(torch.float8_e4m3fn) if fp8 else x[:, :d]).double()
    want = ((xd - c0[:d].double()) ** 2).sum(1)
    torch.testing.assert_close(cost.double(), want, rtol=1e-5, atol=1e-5 * float(ref.max()))
    if not fp8:
        bits = x[:, :d].contiguous().view(torch.int16).to(torch.int32) & 0x7FFF
        nz = bits[bits != 0]
        e = (nz >> 7) & 0xFF
        assert er.tolist() == [int(e.min()), int(e.max())]


def test_init_sample_and_merge_match_torch():
    n = 1_000_003
    g = torch.Generator(device="cuda").manual_seed(3)
    cost = torch.rand(n, device="cuda", generator=g) * 10
    ids = torch.arange(17, 17 + n, device="cuda", dtype=torch.int64)
    key = rng.key(42, 100)
    scale = 2 * 256 / float(cost.double().sum())
    out = torch.empty(n, dtype=torch.int32, device="cuda")
    cnt = torch.zeros(1, dtype=torch.int32, device="cuda")
    K.init_sample(cost, ids, n, key, scale, out, cnt)
    m = int(cnt.item())
    got = torch.sort(out[:m]).values.long().cpu()
    u = rng.uniform(ids.cpu(), 42, 100)
    want = torch.nonzero(u < scale * cost.cpu().double()).flatten()
    assert torch.equal(got, want)
    # capacity: the count is the total, only cap rows are written
    small = torch.full((5,), -7, dtype=torch.int32, device="cuda")
    cnt.zero_()
    K.init_sample(cost, ids, n, key, scale, small, cnt)
    assert int(cnt.item()) == m and bool((small >= 0).all())
    near = torch.zeros(n, dtype=torch.int32, device="cuda")
    best = torch.rand(n, device="cuda", generator=g) * 10
    lab = torch.randint(0, 100, (n,), device="cuda", generator=g, dtype=torch.int32)
    c2, n2 = cost.clone(), near.clone()
    K.init_merge(c2, n2, best, lab, 1000, n)
    better = best < cost
    assert torch.equal(c2, torch.where(better, best, cost))
    assert torch.equal(n2, torch.where(better, lab + 1000, near))


@pytest.mark.parametrize("m,d,k,spherical", [(1025, 256, 256, False), (300, 7, 20, False), (50, 3, 49, False),
                                             (2000, 64, 5, False), (600, 32, 40, True), (12, 5, 12, False),
                                             (1500, 48, 300, False), (2048, 16, 512, False), (200, 4, 30, False)])
def test_local_kmeans_device_equals_host_bitwise(m, d, k, spherical):
    rs = np.random.RandomState(m + k)
    pts = rs.randn(m, d) * 3 + rs.randint(0, 8, (m, 1))
    pts[1] = pts[0]  # duplicate candidate
    if m == 200:  # five distinct points: the weights of every later pick are all zero (the uniform pick)
        pts = np.tile(pts[:5], (40, 1))
    w = rs.randint(0, 50, m).astype(np.float64)
    w[:3] = 0.0
    if spherical:
        pts /= np.linalg.norm(pts, axis=1, keepdims=True)
    host = K.local_kmeans(torch.as_tensor(pts), torch.as_tensor(w), k, seed=9, spherical=spherical)
    dev = K.local_kmeans(torch.as_tensor(pts, device="cuda"), torch.as_tensor(w, device="cuda"), k, seed=9,
                         spherical=spherical)
    assert np.array_equal(host.numpy(), dev.cpu().numpy())
    assert np.isfinite(host.numpy()).all()


def _integer_blobs(n, d, k, seed):
    rs = np.random.RandomState(seed)
    cen = rs.randint(0, 12, (k, d))
    x = np.clip(cen[rs.randint(0, k, n)] + rs.randint(-1, 2, (n, d)), 0, 15)
    return x.astype(np.float64)  # small integers: exact in bf16, every squared distance exact in f32


@pytest.mark.parametrize("n,d,k", [(40_000, 16, 24), (20_011, 128, 64), (8_000, 256, 200)])
def test_init_device_equals_cpu_on_exact_data(n, d, k):
    """With exactly representable data every cost, sampling decision, candidate and weight is the same
    on both sessions, and the local k-means is the same arithmetic: the init centres are bitwise equal."""
    x = _integer_blobs(n, d, k, seed=d)
    cpu = LloydEngine(torch.as_tensor(x), d, k).init_kmeans_parallel(seed=5)
    gpu = LloydEngine(torch.as_tensor(x, device="cuda"), d, k).init_kmeans_parallel(seed=5)
    assert np.array_equal(cpu, gpu)


def test_init_then_fit_on_blobs_gpu():
    """Engine path end to end: the fused first pass fills the norms; the fit recovers the blobs."""
    n, d, k = 200_000, 256, 32
    g = torch.Generator(device="cuda").manual_seed(1)
    cen = torch.randn(k, d, device="cuda", generator=g) * 6
    x = (cen[torch.randint(0, k, (n,), device="cuda", generator=g)] + torch.randn(n, d, device="cuda", generator=g))
    eng = LloydEngine(x.to(torch.bfloat16), d, k)
    assert not eng._norms_ready
    init = eng.init_kmeans_parallel(seed=3)
    assert eng._norms_ready
    torch.testing.assert_close(eng.xnorm[:n], K.row_sqnorm(eng.x, n, eng.dp)[:n], rtol=0, atol=0)
    eng.set_centers(init)
    eng.fit(20, 0.0)
    got = eng.centers
    dmin = torch.cdist(cen.double(), got).min(1).values
    assert float(dmin.max()) < 0.5


@pytest.mark.parametrize("n,d,k,scale", [(300_001, 256, 64, 4.0), (120_013, 128, 100, 3.0), (50_000, 256, 256, 0.3)])
def test_seeded_first_step_equals_full_step(monkeypatch, n, d, k, scale):
    """The first Lloyd step after the device k-means|| init starts from the bounds the init implies
    (kmeans_seed_bounds + candidate pass + full accumulate) instead of a full assign pass: labels after
    step 1, the centres over a whole fit and the costs are bitwise those of the full first step; on
    separated blobs most rows are proven by the seeded bounds. (scale 0.3: overlapping blobs, few rows
    proven.)"""
    monkeypatch.setenv("CML_KMEANS_PRUNE", "1")
    monkeypatch.setenv("CML_KMEANS_PRECISION", "bf16")
    g = torch.Generator(device="cuda").manual_seed(n)
    cen = torch.randn(k, d, device="cuda", generator=g) * scale
    x = (cen[torch.randint(0, k, (n,), device="cuda", generator=g)] +
         torch.randn(n, d, device="cuda", generator=g)).to(torch.bfloat16)
    res = []
    for seeded in ("1", "0"):
        monkeypatch.setenv("CML_KMEANS_SEED_BOUNDS", seeded)
        eng = LloydEngine(x, d, k)
        eng.track_prune = True
        init = eng.init_kmeans_parallel(seed=11)
        eng.set_centers(init)
        assert eng._seeded == (seeded == "1")
        eng.step()
        lab1 = eng.labels[:n].clone()
        st = eng._pst
        idx = torch.arange(0, n, 7, device="cuda")
        xs = eng.x[idx, :d].double()
        own = ((xs - st.cb_old[lab1[idx].long(), :d].double()) ** 2).sum(1).sqrt()
        assert bool((st.ub[idx].double() >= own * (1 - 1e-12)).all())  # valid upper bounds after step 1
        c1 = eng.training_cost()
        eng.fit(12, 0.0, start_iter=1)
        res.append((init, lab1, c1, eng.centers.cpu().numpy(), eng.training_cost(), eng.prune_history()))
    (i_s, l_s, c_s, C_s, f_s, h_s), (i_f, l_f, c_f, C_f, f_f, h_f) = res
    assert np.array_equal(i_s, i_f)
    assert torch.equal(l_s, l_f)
    assert c_s == c_f and f_s == f_f
    assert np.array_equal(C_s, C_f)
    assert h_f[0] == (True, n)  # the unseeded engine ran a full first pass
    full, m = h_s[0]
    assert 0 <= m <= n and (not full or m == n)  # more than _PRUNE_CAP candidates: the full pass instead
    if scale >= 4.0:
        assert not full and m < 0.5 * n, m


@pytest.mark.parametrize("n,d,k", [(120_000, 128, 64), (60_013, 256, 100), (40_000, 512, 64)])
def test_pruned_candidate_pass_equals_full_on_exact_data(monkeypatch, n, d, k):
    """The second k-means|| round skips the (row, candidate) pairs the triangle inequality rules out
    (init_classify / init_near_list / K9r candidate pass on the remaining rows). On exactly representable
    data every distance is exact, so the init centres equal those of the full candidate passes, and the
    pruned pass really skipped rows."""
    monkeypatch.setenv("CML_KMEANS_PRUNE", "1")
    monkeypatch.setenv("CML_KMEANS_PRECISION", "bf16")
    x = torch.as_tensor(_integer_blobs(n, d, k, seed=n), device="cuda")
    res = []
    for pruned in ("1", "0"):
        monkeypatch.setenv("CML_KMEANS_INIT_PRUNE", pruned)
        eng = LloydEngine(x, d, k)
        eng.track_prune = True
        res.append((eng.init_kmeans_parallel(seed=21), getattr(eng, "_init_prune_history", [])))
    assert np.array_equal(res[0][0], res[1][0])
    # one pruned pass per round after the first chunk (Dp = 512: K9r takes 128 centres per launch, so a
    # first round with more candidates prunes its rest too)
    assert res[1][1] == [] and len(res[0][1]) >= 1
    rows, ca, cb = res[0][1][-1]
    assert rows == n and ca + cb < n


@pytest.mark.parametrize("n", [1, 5, 4096, 1_000_003])
def test_sum_f64_matches_torch(n):
    """Σ of f32 values in f64 (the k-means|| cost total) against torch's f64 sum of the same values."""
    g = torch.Generator(device="cuda").manual_seed(n)
    x = torch.rand(n + 3, device="cuda", generator=g) * 1000
    got = float(K.sum_f64(x, n))
    want = float(x[:n].double().sum())
    assert got == pytest.approx(want, rel=1e-12, abs=1e-12)
    assert float(K.sum_f64(x, n)) == got  # deterministic


@pytest.mark.parametrize("mp,m,d", [(1, 1, 3), (257, 513, 256), (640, 1024, 128), (5, 37, 512)])
def test_init_table_kernel(mp, m, d):
    """The pruned pass's table in one launch: each row sorted ascending, each entry a lower bound of the
    real distance within 2e-6 of it, the indices a permutation, the norms rounded up."""
    from clustermachinelearningforhospitalnetworks_apache_spark_amd.ops import kmeans_ops as K
    g = torch.Generator(device="cuda").manual_seed(mp + m)
    P = torch.randn(mp, d, generator=g, device="cuda", dtype=torch.float64) * 5
    Y = torch.randn(m, d, generator=g, device="cuda", dtype=torch.float64) * 5
    tab_v, tab_j, pn32 = K.init_table(P, Y)
    D = torch.cdist(P, Y)
    assert bool((tab_v[:, 1:] >= tab_v[:, :-1]).all())
    assert torch.equal(tab_j.sort(dim=1).values, torch.arange(m, device="cuda", dtype=torch.int32).expand(mp, m))
    dj = D.gather(1, tab_j.long())
    assert bool((tab_v.double() <= dj).all()) and bool((tab_v.double() >= dj * (1 - 2e-6) - 1e-30).all())
    assert bool((pn32.double() >= (P * P).sum(1)).all())


@pytest.mark.parametrize("m,d", [(1, 3), (37, 1), (600, 256), (2049, 40)])
def test_unique_rows_kernel_matches_torch_unique(m, d):
    """The distinct-candidate kernels against torch.unique(dim=0, return_inverse=True) on the host: the same
    lexicographically sorted distinct rows and the same inverse, with exact duplicates, rows equal in their
    first columns only, and integer-valued ties."""
    g = torch.Generator().manual_seed(m + d)
    P = torch.randint(-3, 4, (m, d), generator=g).to(torch.float64)
    if m > 10:
        P[1::7] = P[0]                     # exact duplicates of one row
        P[2::5, : d // 2] = P[3, : d // 2]  # shared prefixes
        P[m // 2:] += torch.rand(m - m // 2, d, generator=g, dtype=torch.float64)
    want_u, want_i = torch.unique(P, dim=0, return_inverse=True)
    got_u, got_i = K.unique_rows(P.cuda())
    assert torch.equal(got_u.cpu(), want_u)
    assert torch.equal(got_i.cpu(), want_i)


@pytest.mark.parametrize("n,d,m,fp8", [(10_000, 256, 513, False), (5_000, 100, 1, False), (3_000, 512, 700, True),
                                       (2_000, 64, 0, False)])
def test_gather_rank_rows_kernel(n, d, m, fp8):
    """A round's sampled rows in row order, widened to f64 from the device count (no sort, no host read),
    equal to sort + gather; rows past the count are zeroed up to pad_rows."""
    from clustermachinelearningforhospitalnetworks_apache_spark_amd.models.kmeans import padded_dim_fp8
    g = torch.Generator(device="cuda").manual_seed(n + m)
    xs = torch.randn(n, d, generator=g, device="cuda") * 3
    if fp8:
        x = torch.zeros((n, padded_dim_fp8(d)), dtype=torch.uint8, device="cuda")
        x[:, :d] = xs.to(torch.float8_e4m3fn).view(torch.uint8)
        x = x.view(torch.float8_e4m3fn)
        ref = x[:, :d].float().double()
    else:
        x = torch.zeros((n, d + 8), dtype=torch.bfloat16, device="cuda")
        x[:, :d] = xs.to(torch.bfloat16)
        ref = x[:, :d].double()
    cap = 1024
    ids = torch.randperm(n, generator=g, device="cuda")[:cap].to(torch.int32)
    cnt = torch.tensor([m], dtype=torch.int32, device="cuda")
    pad = m + 5
    dest = torch.full((max(cap, pad), d), 7.0, dtype=torch.float64, device="cuda")
    assert K.gather_rank_rows(x, ids, cnt, cap, d, dest, pad_rows=pad)
    want = ref[torch.sort(ids[:m]).values.long()]
    assert torch.equal(dest[:m], want)
    assert bool((dest[m:pad] == 0).all())


@pytest.mark.parametrize("m,d,k", [(600, 256, 256), (7, 33, 1), (1000, 128, 64)])
def test_seed_table_kernel(m, d, k):
    """Per distinct candidate: the nearest bf16 centre and outward-rounded distances to it and to the
    second nearest (valid bounds of the f64 distances), the norm rounded up."""
    g = torch.Generator(device="cuda").manual_seed(m * k)
    C = (torch.randn(k, d, generator=g, device="cuda", dtype=torch.float64) * 4)
    cb = torch.zeros((round(k / 32 + 0.5) * 32 + 32, d + 16), dtype=torch.bfloat16, device="cuda")
    cb[:k, :d] = C.to(torch.bfloat16)
    U = C[torch.randint(0, k, (m,), generator=g, device="cuda")].to(torch.bfloat16).double() + \
        torch.randn(m, d, generator=g, device="cuda", dtype=torch.float64) * 0.5
    a, d1, d2, pn = K.seed_table(U, cb, k)
    D = torch.cdist(U, cb[:k, :d].double())
    top = torch.sort(D, dim=1).values
    assert bool((D.gather(1, a[:m].long()[:, None])[:, 0] == top[:, 0]).all())
    assert bool((d1[:m].double() >= top[:, 0]).all()) and bool((d1[:m].double() <= top[:, 0] * (1 + 1e-5) + 1e-30).all())
    if k > 1:
        assert bool((d2[:m].double() <= top[:, 1]).all()) and bool((d2[:m].double() >= top[:, 1] * (1 - 1e-5)).all())
    else:
        assert bool(torch.isinf(d2[:m]).all())
    assert bool((pn[:m].double() >= (U * U).sum(1)).all())

