"""Numerics of the KMeans HIP kernels (K9/K10/K11) against float64 torch references."""
import numpy as np
import pytest
import torch

from clustermachinelearningforhospitalnetworks_apache_spark_amd.models.kmeans import (LloydEngine, assign_gpu,
                                                                                       to_device_matrix)
from clustermachinelearningforhospitalnetworks_apache_spark_amd.ops import kmeans_ops as K

pytestmark = pytest.mark.gpu


@pytest.fixture(autouse=True)
def _full_steps_only(monkeypatch):
    """These tests target the full / incremental MFMA step machinery: pruned steps off by default, and
    f32/f64 rows take the bf16 path (not the source-precision one, tests/test_kmeans_exact_gpu.py)."""
    monkeypatch.setenv("CML_KMEANS_PRUNE", "0")
    monkeypatch.setenv("CML_KMEANS_PRECISION", "bf16")


def _ref_assign(xb, cb):
    """Exact (f64, on the rows' device) argmin over the bf16/fp8 operands: label, distance, top-2 gap."""
    x = xb.double()
    c = cb.double().to(x.device)
    sc = (c * c).sum(1)[None, :] - 2 * x @ c.T
    top = torch.topk(sc, min(2, c.shape[0]), dim=1, largest=False)
    d = (x * x).sum(1) + top.values[:, 0]
    gap = top.values[:, 1] - top.values[:, 0] if c.shape[0] > 1 else torch.full_like(d, 1e9)
    return top.indices[:, 0].cpu(), d.clamp(min=0).cpu(), gap.cpu()


def _band(xb, cb, dp):
    """The assign's own error bound on a squared distance, tau·(|x|² + max|c|²) per row (tau =
    LloydEngine.prune_tau: f32 accumulation of dp bf16 products plus the argmin key truncation). Two
    labels may differ only where the exact top-2 gap is within 2·band."""
    tau = LloydEngine.prune_tau(dp)
    x = xb.double()
    c = cb.double().to(x.device)
    return (tau * ((x * x).sum(1) + float((c * c).sum(1).max()))).cpu()


def _check_labels(lab, ref_lab, gap, band):
    bad = (lab != ref_lab) & (gap > 2 * band)
    assert not bool(bad.any()), f"{int(bad.sum())} label mismatches outside the 2·tau band"


def _check_dist(best, ref_d, band):
    err = (best.double().cpu() - ref_d).abs()
    assert bool((err <= band).all()), f"max distance error {float((err / band).max()):.3g} x the tau band"


@pytest.mark.parametrize("n,d,k", [(1000, 4, 5), (4097, 100, 70), (20000, 256, 256), (3000, 512, 200),
                                   (777, 16, 33), (5000, 128, 64)])
@pytest.mark.parametrize("cached_norm", [False, True])
def test_assign_matches_reference(n, d, k, cached_norm):
    """Every row's label is the bf16-exact argmin up to near-ties; rows equal to a centre keep
    distance ~0 (the rounding-negative case of the packed-key minimum)."""
    torch.manual_seed(0)
    dev = torch.device("cuda")
    x = torch.randn(n, d, device=dev) * 2
    c = torch.randn(k, d, device=dev) * 2
    xm = to_device_matrix(x, d)
    xn = K.row_sqnorm(xm, n, xm.shape[1]) if cached_norm else None
    if xn is not None:
        np.testing.assert_allclose(xn.cpu().double().numpy(), (xm.double() ** 2).sum(1).cpu().numpy(), rtol=1e-5)
    lab, best = assign_gpu(xm, xm.shape[1], d, c.double(), xnorm=xn)
    torch.cuda.synchronize()
    cb = c.to(torch.bfloat16)
    ref_lab, ref_d, gap = _ref_assign(x.to(torch.bfloat16), cb)
    band = _band(x.to(torch.bfloat16), cb, xm.shape[1])
    _check_labels(lab.cpu().long(), ref_lab, gap, band)
    _check_dist(best, ref_d, band)


@pytest.fixture
def assign_variant(request):
    """Variant 0 here is the default dispatch (K9r where it applies, else K9); 9 = K9 forced (variant 0
    with the K9r default switched off)."""
    v = request.param
    K.set_assign_variant(0 if v == 9 else v)
    if v == 9:
        K.set_rr_default(False)
    yield v
    K.set_assign_variant(0)
    K.set_rr_default(True)


@pytest.mark.parametrize("assign_variant", [0, 1, 2, 3, 8, 9], indirect=True)
@pytest.mark.parametrize("mode", [None, "sort"])
@pytest.mark.parametrize("n,d,k", [(1000, 4, 5), (50000, 256, 256), (9999, 100, 70), (2000, 16, 3),
                                   (3000, 512, 40), (40000, 128, 64)])
def test_lloyd_step_matches_reference(n, d, k, mode, assign_variant):
    torch.manual_seed(1)
    dev = torch.device("cuda")
    x = (torch.randn(n, d, device=dev) * 3).to(torch.bfloat16)
    init = x[:k].double().cpu().numpy()
    eng = LloydEngine(x, d, k, accum_mode=mode)
    eng.set_centers(init)
    eng.step()
    torch.cuda.synchronize()
    lab = eng.labels[:n].cpu().long()
    # reference sums with the GPU's labels (tests K10/K11 independently of near-tie flips)
    xs = x.double().cpu()
    sums, counts = K.sums_reference(xs, lab, k)
    old = torch.as_tensor(init)
    want = torch.where(counts[:, None] > 0, sums / counts.clamp(min=1)[:, None], old)
    np.testing.assert_allclose(eng.centers.cpu().numpy(), want.numpy(), rtol=1e-4, atol=1e-4)
    msg = eng.msgs[0].cpu()
    np.testing.assert_array_equal(msg[k * d:k * d + k].numpy(), counts.numpy())
    # label agreement with the exact argmin outside the kernels' own rounding band
    cb0 = torch.as_tensor(init).to(torch.bfloat16)
    ref_lab, ref_d, gap = _ref_assign(x, cb0)
    _check_labels(lab, ref_lab, gap, _band(x, cb0, eng.dp))
    assert abs(eng.training_cost() - ref_d.sum().item()) <= 1e-3 * ref_d.sum().item() + 1e-3


def test_fit_converges_on_blobs():
    torch.manual_seed(2)
    dev = torch.device("cuda")
    k, d, n = 8, 32, 100000
    centers = torch.randn(k, d, device=dev) * 10
    lab = torch.randint(0, k, (n,), device=dev)
    x = (centers[lab] + torch.randn(n, d, device=dev)).to(torch.bfloat16)
    eng = LloydEngine(x, d, k)
    eng.set_centers(eng.init_kmeans_parallel(seed=7))
    it = eng.fit(max_iter=20, tol=1e-4)
    assert it <= 20
    got = torch.as_tensor(eng.centers.cpu())
    # every true centre is matched by a fitted centre
    dist = torch.cdist(centers.double().cpu(), got)
    assert dist.min(1).values.max().item() < 0.5


def test_sort_regime_handles_skew():
    """All rows in one cluster: the segmented sum must still be exact (and not serialise)."""
    dev = torch.device("cuda")
    n, d, k = 30000, 256, 256
    x = (torch.randn(n, d, device=dev) * 0.01).to(torch.bfloat16)
    init = np.zeros((k, d))
    init[1:] = 100.0 + np.arange(1, k)[:, None]  # every row is closest to centre 0
    eng = LloydEngine(x, d, k, accum_mode="sort")
    eng.set_centers(init)
    eng.step()
    torch.cuda.synchronize()
    assert (eng.labels[:n] == 0).all()
    want = x.double().mean(0).cpu().numpy()
    np.testing.assert_allclose(eng.centers[0].cpu().numpy(), want, rtol=1e-6, atol=1e-9)
    np.testing.assert_allclose(eng.centers[1:].cpu().numpy(), init[1:])


@pytest.mark.parametrize("n,d,k", [(200_000, 64, 7), (123_457, 256, 256), (50_000, 16, 1)])
def test_sort_regime_bitwise_deterministic(n, d, k):
    """Atomic-free segmented sums: two identical steps give bitwise-identical messages, and the
    sums match the float64 reference (clusters spanning many slices exercise the fixup)."""
    torch.manual_seed(4)
    x = (torch.randn(n, d, device="cuda") * 2).to(torch.bfloat16)
    init = x[:k].double().cpu().numpy()
    msgs = []
    for _ in range(2):
        eng = LloydEngine(x, d, k, accum_mode="sort")
        eng.set_centers(init)
        eng.step()
        torch.cuda.synchronize()
        msgs.append(eng.msgs[0].clone())
    assert torch.equal(msgs[0], msgs[1])
    lab = eng.labels[:n].cpu().long()
    # the sums are exact: plain f64 sums, or (wide exponent span: models/kmeans.py _sum_grid) integer
    # sums of the rows rounded to the grid, scaled back by the grid step
    unit = eng.sum_grid or 1.0
    xq = x.double().cpu() if eng.sum_grid is None else torch.round(x.double().cpu() / unit) * unit
    sums, counts = K.sums_reference(xq, lab, k)
    assert torch.equal(msgs[0][:k * d].cpu() * unit, sums.reshape(-1))


@pytest.mark.parametrize("n,d,k", [(30_000, 37, 5), (50_000, 256, 256), (20_000, 512, 64), (9_999, 200, 33)])
@pytest.mark.parametrize("mode", [None, "sort"])
def test_fp8_features_lloyd_step(n, d, k, mode):
    """OCP e4m3fn feature storage (SURVEY config 5): the kernels dequantise exactly to bf16, so the
    step must equal the bf16 computation on the dequantised values."""
    torch.manual_seed(5)
    xf = torch.randn(n, d, device="cuda") * 1.5
    x8 = xf.to(torch.float8_e4m3fn)
    xd = x8.to(torch.float32)  # exact dequantisation
    init = xd[:k].double().cpu().numpy()
    eng = LloydEngine(x8, d, k, accum_mode=mode)
    assert eng.x.dtype == torch.float8_e4m3fn and eng.x.shape[1] >= 256
    np.testing.assert_allclose(eng.xnorm[:n].cpu().numpy(), (xd.double() ** 2).sum(1).cpu().numpy(), rtol=1e-5)
    eng.set_centers(init)
    eng.step()
    torch.cuda.synchronize()
    lab = eng.labels[:n].cpu().long()
    sums, counts = K.sums_reference(xd.double().cpu(), lab, k)
    msg = eng.msgs[0].cpu()
    np.testing.assert_array_equal(msg[k * d:k * d + k].numpy(), counts.numpy())
    np.testing.assert_allclose(msg[:k * d].numpy(), sums.reshape(-1).numpy(), rtol=1e-9, atol=1e-6)
    cb0 = torch.as_tensor(init).to(torch.bfloat16)
    ref_lab, ref_d, gap = _ref_assign(xd.to(torch.bfloat16), cb0)
    _check_labels(lab, ref_lab, gap, _band(xd.to(torch.bfloat16), cb0, eng.dp))


@pytest.mark.parametrize("n,d,k,mode", [(200_000, 64, 16, None), (100_000, 256, 256, "sort"), (50_000, 16, 5, None)])
def test_graph_replay_matches_eager(n, d, k, mode):
    """The captured (hipGraph) Lloyd step reproduces eager steps bit for bit, including after
    set_centers() between fits."""
    torch.manual_seed(6)
    x = (torch.randn(n, d, device="cuda") * 2).to(torch.bfloat16)
    init = x[:k].double().cpu().numpy()
    out = {}
    for use_graph in (False, True):
        eng = LloydEngine(x, d, k, accum_mode=mode, use_graph=use_graph)
        eng.set_centers(init)
        for _ in range(4):
            eng.step()
        c1 = eng.centers.clone()
        eng.set_centers(init)
        for _ in range(2):
            eng.step()
        torch.cuda.synchronize()
        out[use_graph] = (c1, eng.centers.clone(), eng.training_cost())
        assert (eng._graph is not None) == use_graph
    assert torch.equal(out[False][0], out[True][0]) and torch.equal(out[False][1], out[True][1])
    assert out[False][2] == out[True][2]


# partial last 64-row tiles and partial last workgroup rounds (round = grid x 64 rows): n = 1, 63, 65 mod
# 64 and mod the round, k not a multiple of the 32-centre tile
@pytest.mark.parametrize("n,d,k", [(20000, 256, 256), (50_001, 128, 64), (3001, 512, 40), (777, 200, 33),
                                   (100_000, 256, 250), (65, 128, 64), (130_000, 100, 100), (63, 256, 40),
                                   (16_385, 256, 256), (16_447, 256, 129), (16_449, 128, 64), (32_831, 256, 200),
                                   (49_153, 512, 97), (1_048_641, 256, 256)])
def test_rr_assign_matches_k9(n, d, k):
    """K9r (register-resident centres, LDS-DMA X ring; variant 8) against K9 and the f64 reference:
    same labels up to near ties, same distances, cost and counting-sort histogram/ranks."""
    torch.manual_seed(11)
    dev = torch.device("cuda")
    x = torch.randn(n, d, device=dev) * 2
    c = x[torch.randperm(n, device=dev)[:k]] + 0.1 * torch.randn(k, d, device=dev)
    xm = to_device_matrix(x, d)
    dp = xm.shape[1]
    xn = K.row_sqnorm(xm, n, dp)
    out = {}
    for v in (0, 8):
        K.set_assign_variant(v)
        K.set_rr_default(False)  # variant 0 = K9 here
        try:
            plan = K.plan_assign(n, dp, k)
            assert (plan.rr_ct > 0) == (v == 8)
            cb = torch.zeros((plan.kp, dp), dtype=torch.bfloat16, device=dev)
            cn = torch.zeros(plan.kp, dtype=torch.float32, device=dev)
            cent = c.double().contiguous().clone()
            K.update_centers(None, k, d, cent, cb, dp, plan.kp, cn, None)
            labels = torch.full((n,), -1, dtype=torch.int32, device=dev)
            best = torch.zeros(n, dtype=torch.float32, device=dev)
            cost = torch.zeros(plan.grid, dtype=torch.float64, device=dev)
            hist = torch.zeros(plan.grid * plan.kp, dtype=torch.int32, device=dev)
            rank = torch.zeros(n, dtype=torch.int32, device=dev)
            K.assign_bf16(xm, n, dp, cb, cn, plan, labels, best, cost, hist, rank, xnorm=xn)
            torch.cuda.synchronize()
            out[v] = (labels.cpu().long(), best.cpu().double(), float(cost.sum()), hist.view(plan.grid, plan.kp).cpu(),
                      rank.cpu(), plan)
        finally:
            K.set_assign_variant(0)
            K.set_rr_default(True)
    lab, best, cost, hist, rank, plan = out[8]
    ref_lab, ref_d, gap = _ref_assign(x.to(torch.bfloat16), c.to(torch.bfloat16))
    band = _band(x.to(torch.bfloat16), c.to(torch.bfloat16), dp)
    _check_labels(lab, ref_lab, gap, band)
    _check_labels(out[0][0], ref_lab, gap, band)
    clear = gap > 2 * band  # K9r == K9 on every row whose label the rounding cannot decide
    assert torch.equal(lab[clear], out[0][0][clear])
    assert lab.min() >= 0 and lab.max() < k  # every row (tail tile / last workgroup included) written
    _check_dist(best, ref_d, band)
    _check_dist(out[0][1], ref_d, band)
    assert abs(cost - best.sum().item()) <= 1e-6 * abs(cost) + 1e-6
    # counting-sort first pass: per-workgroup histograms sum to the label counts, ranks are a
    # permutation of 0..count-1 inside every (workgroup, label) run of the rows that workgroup owns
    np.testing.assert_array_equal(hist.sum(0)[:k].numpy(), torch.bincount(lab, minlength=k).numpy())
    rows = torch.arange(n)
    blk = (rows // plan.round_rows) % plan.grid
    key = blk * plan.kp + lab
    order = torch.argsort(key * n + rank.long())
    ks, rs = key[order], rank.long()[order]
    first = torch.ones(n, dtype=torch.bool)
    first[1:] = ks[1:] != ks[:-1]
    start = torch.cummax(torch.where(first, torch.arange(n), torch.zeros(n, dtype=torch.long)), 0).values
    assert torch.equal(rs, torch.arange(n) - start)


@pytest.mark.parametrize("n,d,k", [(300_000, 256, 256), (200_000, 128, 64)])
def test_rr_lloyd_fit_matches_k9(n, d, k):
    """Whole fits with K9r (incremental sums, graph replay): after every step the centres are exactly
    the means of the rows under the engine's own labels (the incremental sums stay exact), and the fit
    tracks the K9 fit (near-tie label flips make the two trajectories drift apart slightly)."""
    torch.manual_seed(12)
    cen = torch.randn(k, d, device="cuda") * 4
    x = (cen[torch.randint(0, k, (n,), device="cuda")] + torch.randn(n, d, device="cuda")).to(torch.bfloat16)
    init = x[:k].double().cpu().numpy()
    xs = x.double().cpu()
    res = {}
    for v in (0, 8):
        K.set_assign_variant(v)
        K.set_rr_default(False)  # variant 0 = K9 here
        try:
            eng = LloydEngine(x, d, k)
            assert (eng.aplan.rr_ct > 0) == (v == 8)
            eng.set_centers(init)
            for _ in range(6):
                prev = eng.centers.cpu().clone()
                cb0 = eng.cb[:k, :d].clone()
                eng.step()
                torch.cuda.synchronize()
                lab = eng.labels[:n].cpu().long()
                # every step's labels: the exact argmin for the step's bf16 centres outside the band
                ref_lab, _, gap = _ref_assign(x, cb0)
                _check_labels(lab, ref_lab, gap, _band(x, cb0, eng.dp))
                sums, counts = K.sums_reference(xs, lab, k)
                want = torch.where(counts[:, None] > 0, sums / counts.clamp(min=1)[:, None], prev)
                np.testing.assert_allclose(eng.centers.cpu().numpy(), want.numpy(), rtol=1e-9, atol=1e-9)
            res[v] = (eng.centers.cpu(), eng.training_cost(), eng.labels[:n].cpu())
        finally:
            K.set_assign_variant(0)
            K.set_rr_default(True)
    agree = (res[0][2] == res[8][2]).float().mean().item()
    assert agree > 0.99, agree  # trajectories: a near-tie flip in one step moves later centres slightly
    assert abs(res[8][1] - res[0][1]) <= 1e-3 * abs(res[0][1])


@pytest.mark.parametrize("n,d,k", [(40_000, 512, 128), (30_001, 256, 256), (5_000, 300, 40)])
def test_rr_fp8_assign_matches_k9(n, d, k):
    """K9r on OCP e4m3fn rows (SURVEY config 5): fragments widened in registers by
    v_cvt_scalef32_pk_bf16_fp8 give the labels/distances of K9's fp8 path and of the bf16 reference
    on the dequantised values."""
    torch.manual_seed(13)
    dev = torch.device("cuda")
    x8 = (torch.randn(n, d, device=dev) * 1.5).to(torch.float8_e4m3fn)
    xd = x8.to(torch.float32)
    c = xd[torch.randperm(n, device=dev)[:k]] + 0.05 * torch.randn(k, d, device=dev)
    xm = to_device_matrix(x8, d)
    dp = xm.shape[1]
    xn = K.row_sqnorm(xm, n, dp)
    out = {}
    for v in (0, 8):
        K.set_assign_variant(v)
        K.set_rr_default(False)
        try:
            plan = K.plan_assign(n, dp, k, fp8=True)
            assert (plan.rr_ct > 0) == (v == 8)
            cb = torch.zeros((plan.kp, dp), dtype=torch.bfloat16, device=dev)
            cn = torch.zeros(plan.kp, dtype=torch.float32, device=dev)
            K.update_centers(None, k, d, c.double().contiguous().clone(), cb, dp, plan.kp, cn, None)
            labels = torch.full((n,), -1, dtype=torch.int32, device=dev)
            best = torch.zeros(n, dtype=torch.float32, device=dev)
            cost = torch.zeros(plan.grid, dtype=torch.float64, device=dev)
            K.assign_bf16(xm, n, dp, cb, cn, plan, labels, best, cost, xnorm=xn)
            torch.cuda.synchronize()
            out[v] = (labels.cpu().long(), best.cpu().double())
        finally:
            K.set_assign_variant(0)
            K.set_rr_default(True)
    ref_lab, ref_d, gap = _ref_assign(xd.to(torch.bfloat16), c.to(torch.bfloat16))
    band = _band(xd.to(torch.bfloat16), c.to(torch.bfloat16), dp)
    lab, best = out[8]
    _check_labels(lab, ref_lab, gap, band)
    _check_labels(out[0][0], ref_lab, gap, band)
    clear = gap > 2 * band
    assert torch.equal(lab[clear], out[0][0][clear])
    _check_dist(best, ref_d, band)
    _check_dist(out[0][1], ref_d, band)


@pytest.mark.parametrize("n,d,k", [(250_003, 256, 200), (120_000, 128, 64), (70_001, 512, 96)])
def test_rr_and_k9_trajectories_bitwise_on_separated_exact_data(n, d, k):
    """No near-ties anywhere: small-integer rows (exact in bf16) in blobs 40 units apart, so every row's
    nearest centre wins by a margin far above any f32 rounding. The K9r fit (incremental sums) and the K9
    fit then give the same labels after every step and bit-identical centres — a tile-edge or tail bug in
    either kernel at any step fails this exactly, not within a label-agreement tolerance."""
    rs = np.random.RandomState(n)
    cen = rs.randint(0, 3, (k, d)) * 40 + rs.randint(0, 4, (k, d))
    x = torch.as_tensor(cen[rs.randint(0, k, n)] + rs.randint(-2, 3, (n, d)), dtype=torch.float32,
                        device="cuda").to(torch.bfloat16)
    init = cen.astype(np.float64)  # one centre per blob: no centre splits a blob, so no row is near a tie
    traj = {}
    for v in (0, 8):
        K.set_assign_variant(v)
        K.set_rr_default(False)
        try:
            eng = LloydEngine(x, d, k)
            assert (eng.aplan.rr_ct > 0) == (v == 8)
            eng.set_centers(init)
            steps = []
            for _ in range(8):
                eng.step()
                steps.append((eng.labels[:n].clone(), eng.centers.cpu().clone()))
            traj[v] = steps
        finally:
            K.set_assign_variant(0)
            K.set_rr_default(True)
    for (l0, c0), (l8, c8) in zip(traj[0], traj[8]):
        assert torch.equal(l0.long(), l8.long())
        assert torch.equal(c0, c8)


@pytest.mark.parametrize("rows,k,d,pad", [(1, 256, 256, 0), (3, 17, 40, 24), (2, 1, 8, 0)])
def test_cost_combine_kernel_matches_f64_formula(rows, k, d, pad):
    """kmeans_cost_combine (the training cost from the step's sums) against the same formula in f64 torch."""
    g = torch.Generator(device="cpu").manual_seed(k * 7 + d)
    kd = k * d
    msgs = torch.randn(rows, kd + k + 1, generator=g, dtype=torch.float64) * 50
    msgs[:, kd:kd + k] = torch.randint(0, 1000, (rows, k), generator=g).double()
    cb = (torch.randn(k + 5, d + pad, generator=g) * 3).to(torch.bfloat16)
    q = torch.rand(k, generator=g, dtype=torch.float64) * 1e6 + 1e5
    unit = 0.25
    ref = K.cost_combine(q, msgs, k, d, unit, cb)  # host form
    got = K.cost_combine(q.cuda(), msgs.cuda(), k, d, unit, cb.cuda())
    assert got.is_cuda
    torch.testing.assert_close(got.cpu(), ref, rtol=1e-12, atol=1e-6)
    again = K.cost_combine(q.cuda(), msgs.cuda(), k, d, unit, cb.cuda())
    assert float(again) == float(got)  # fixed reduction order
