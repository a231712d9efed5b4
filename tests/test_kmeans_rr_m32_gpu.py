"""K9r compute waves on 32x32x16 MFMA tiles (kmeans_rr.h compute_m32) against the 16x16x32 form and
an f64 reference over the same bf16 / fp8 operands: labels agree outside the rounding band
2·tau·(|x|² + max|c|²) of the exact top-2 gap, distances agree within tau·(|x|² + max|c|²), the
top-2 bounds of mode 1 hold exactly, counting-sort ranks form a permutation of every (workgroup,
label) bucket, and partial last tiles / workgroups (n not a multiple of the 64-row tile) are covered."""
import pytest
import torch

from clustermachinelearningforhospitalnetworks_apache_spark_amd.ops import kmeans_ops as K

pytestmark = pytest.mark.gpu


def _setup(n, d, k, seed, fp8=False):
    from clustermachinelearningforhospitalnetworks_apache_spark_amd.models.kmeans import to_device_matrix
    from clustermachinelearningforhospitalnetworks_apache_spark_amd.utils.device import round_up
    g = torch.Generator(device="cuda").manual_seed(seed)
    cen = torch.randn(max(k, 1), d, device="cuda", generator=g) * 3
    x = cen[torch.randint(0, max(k, 1), (n,), device="cuda", generator=g)] + torch.randn(n, d, device="cuda",
                                                                                          generator=g)
    x = x.to(torch.float8_e4m3fn) if fp8 else x.to(torch.bfloat16)
    x = to_device_matrix(x, d)
    dp = x.shape[1]
    kp = round_up(k, 32)
    pick = torch.randint(0, n, (k,), device="cuda", generator=g)
    xs = x.view(torch.uint8)[pick].view(x.dtype) if fp8 else x[pick]
    cent = xs[:, :d].to(torch.float64).contiguous()
    cb = torch.zeros((kp, dp), dtype=torch.bfloat16, device="cuda")
    cn = torch.zeros(kp, dtype=torch.float32, device="cuda")
    K.update_centers(None, k, d, cent.clone(), cb, dp, kp, cn, None)
    xn = K.row_sqnorm(x, n, dp)
    return x, dp, kp, cb, cn, xn


def _exact(x, d, cb, k, fp8):
    xf = (x.view(torch.float8_e4m3fn) if fp8 else x)[:, :d].to(torch.float64)
    c = cb[:k, :d].double()
    dist = (xf * xf).sum(1, keepdim=True) - 2 * xf @ c.T + (c * c).sum(1)[None]
    top = torch.topk(dist, min(2, k), dim=1, largest=False)
    return dist, top.values


def _run(x, n, dp, cb, cn, xn, k, m32):
    K.set_rr_m32(m32)
    try:
        plan = K.plan_assign(n, dp, k, fp8=K.is_fp8(x))
        assert plan.rr_ct > 0
        lab = torch.full((n,), -1, dtype=torch.int32, device="cuda")
        best = torch.zeros(n, device="cuda")
        cp = torch.zeros(plan.grid, dtype=torch.float64, device="cuda")
        hist = torch.zeros(plan.grid * plan.kp, dtype=torch.int32, device="cuda")
        rank = torch.zeros(n, dtype=torch.int32, device="cuda")
        K.assign_bf16(x, n, dp, cb, cn, plan, lab, best, cp, hist, rank, xnorm=xn)
        torch.cuda.synchronize()
        return plan, lab, best, cp, hist, rank
    finally:
        K.set_rr_m32(False)  # the default form


_SHAPES = [(70_001, 256, 256, False), (33_333, 128, 128, False), (20_011, 256, 100, False), (65, 256, 250, False),
           (40_003, 256, 200, True), (9_001, 512, 128, True)]


@pytest.mark.parametrize("n,d,k,fp8", _SHAPES)
def test_m32_matches_m16_and_exact(n, d, k, fp8):
    x, dp, kp, cb, cn, xn = _setup(n, d, k, seed=n + k, fp8=fp8)
    from clustermachinelearningforhospitalnetworks_apache_spark_amd.models.kmeans import LloydEngine
    tau = LloydEngine.prune_tau(dp)
    _, lab32, best32, cp32, hist32, rank32 = _run(x, n, dp, cb, cn, xn, k, True)
    _, lab16, best16, cp16, _, _ = _run(x, n, dp, cb, cn, xn, k, False)
    dist, top = _exact(x, d, cb, k, fp8)
    mc = float(cn[:k].max())
    band = tau * (xn.double() + mc)
    # distances: both forms within the error allowance of the exact f64 distance of their label
    own32 = dist.gather(1, lab32.long()[:, None]).squeeze(1)
    assert bool(((best32.double() - own32).abs() <= band).all())
    assert bool(((own32 - top[:, 0]) <= 2 * band).all())  # the label is a true minimiser within the band
    # labels: identical wherever the exact top-2 gap exceeds the rounding band
    if k > 1:
        clear = (top[:, 1] - top[:, 0]) > 2 * band
        assert bool(torch.equal(lab32[clear], lab16[clear]))
        if n >= 100 * k:  # (duplicate centres when k approaches n: zero gaps)
            assert float(clear.double().mean()) > 0.95
    # cost partials: the same f64 sum of the per-row f32 distances
    assert abs(float(cp32.sum()) - float(best32.double().sum())) <= 1e-6 * max(1.0, float(best32.double().sum()))
    # counting-sort ranks: per (workgroup, label) a permutation of 0 .. count-1
    plan = K.plan_assign(n, dp, k, fp8=fp8)
    tr = plan.round_rows
    wg = (torch.arange(n, device="cuda") // tr) % plan.grid
    key = wg * plan.kp + lab32.long()
    counts = torch.bincount(key, minlength=plan.grid * plan.kp)
    assert torch.equal(counts.to(torch.int32), hist32)
    order = torch.argsort(key * n + rank32.long())
    ks, rs = key[order], rank32.long()[order]
    start = torch.cumsum(counts, 0) - counts
    assert torch.equal(rs, torch.arange(n, device="cuda") - start[ks])


@pytest.mark.parametrize("n,d,k", [(50_001, 256, 256), (12_345, 128, 64 + 64)])
def test_m32_top2_bounds_hold(n, d, k):
    """Mode 1 on the 32x32 form: ub >= exact own distance, lb <= exact distance to every other centre."""
    x, dp, kp, cb, cn, xn = _setup(n, d, k, seed=7 * n)
    from clustermachinelearningforhospitalnetworks_apache_spark_amd.models.kmeans import LloydEngine
    tau = LloydEngine.prune_tau(dp)
    mc = torch.tensor([float(cn[:k].max())], device="cuda")
    plan = K.plan_assign(n, dp, k)
    lab = torch.zeros(n, dtype=torch.int32, device="cuda")
    ub, lb = torch.zeros(n, device="cuda"), torch.zeros(n, device="cuda")
    K.assign_rr_ext(1, x, n, dp, cb, cn, plan, xn, lab, None, ub, lb, mc, tau)
    torch.cuda.synchronize()
    dist, _ = _exact(x, d, cb, k, False)
    own = dist.gather(1, lab.long()[:, None]).squeeze(1).clamp(min=0).sqrt()
    other = dist.scatter(1, lab.long()[:, None], float("inf")).min(1).values.clamp(min=0).sqrt()
    assert bool((ub.double() >= own * (1 - 1e-12)).all())
    assert bool((lb.double() <= other * (1 + 1e-12)).all())
