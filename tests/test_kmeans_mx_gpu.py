"""MX-scaled fp8 MFMA operands of the K9r screen pass (kmeans_mx.hip): the 16x16x128 lane layout and scale
semantics of v_mfma_scale_f32_16x16x128_f8f6f4 against an f64 reference, and the hi/lo centre split."""
import pytest
import torch

from clustermachinelearningforhospitalnetworks_apache_spark_amd.ops import kmeans_ops as K

pytestmark = pytest.mark.gpu


def _e4m3_bytes(v: torch.Tensor) -> torch.Tensor:
    return v.to(torch.float8_e4m3fn).view(torch.uint8)


def _dec(b: torch.Tensor) -> torch.Tensor:
    return b.view(torch.float8_e4m3fn).to(torch.float64)


def test_mx_probe_layout_and_scales():
    dev = torch.device("cuda", 0)
    g = torch.Generator(device="cpu").manual_seed(3)
    a = _e4m3_bytes(torch.randn(16, 128, generator=g) * 8)
    b = _e4m3_bytes(torch.randn(16, 128, generator=g) * 8)
    sa = torch.randint(118, 136, (64,), generator=g, dtype=torch.int32)
    sb = torch.randint(118, 136, (64,), generator=g, dtype=torch.int32)
    out = K.mx_probe(a.to(dev), b.to(dev), sa.to(dev), sb.to(dev)).cpu().double()
    # byte j of lane group g is k = 16g + j (j < 16) or 64 + 16g + (j - 16): scale block (k // 32) comes
    # from lane group k // 32 — i.e. byte j of lane group g takes the scale of lane group 2·(j >= 16) + g // 2
    kk = torch.arange(128)
    g_, j_ = kk // 32, kk % 32
    q = 2 * (j_ >= 16).long() + g_ // 2
    lane = torch.arange(16)[:, None] + 16 * q[None, :]  # [row, buffer position] -> lane of its scale
    A = _dec(a) * torch.pow(2.0, (sa[lane] - 127).double())
    B = _dec(b) * torch.pow(2.0, (sb[lane] - 127).double())
    ref = A @ B.t()
    mag = A.abs() @ B.abs().t()
    err = ((out - ref).abs() / mag.clamp(min=1e-300)).max().item()
    print(f"mx probe: max |out - ref| / sum|terms| = {err:.3g}")
    assert err <= 2.0 ** -15, err


def _emu_e4m3(v: torch.Tensor) -> torch.Tensor:
    return v.to(torch.float8_e4m3fn).to(torch.float64)


def _block_shift(m: torch.Tensor) -> torch.Tensor:
    e = torch.frexp(m.float())[1].long()
    s = (8 - e).clamp(-120, 120)
    return torch.where(m > 0, s, torch.zeros_like(s))


def _snap_ref(cb: torch.Tensor) -> torch.Tensor:
    """torch model of kmeans_mx_snap_kernel: per 32-element block, hi = e4m3(v·2^s), lo = e4m3(r·2^t)."""
    k, dp = cb.shape
    v = cb.double().reshape(k, dp // 32, 32)
    s = _block_shift(v.abs().amax(-1, keepdim=True))
    hi = _emu_e4m3(v * torch.pow(2.0, s.double())) * torch.pow(2.0, -s.double())
    r = v - hi
    t = _block_shift(r.abs().amax(-1, keepdim=True))
    lo = _emu_e4m3(r * torch.pow(2.0, t.double())) * torch.pow(2.0, -t.double())
    return (hi + lo).reshape(k, dp)


def test_mx_snap_grid():
    dev = torch.device("cuda", 0)
    g = torch.Generator(device="cpu").manual_seed(5)
    kc, kp, dp = 40, 48, 512
    c = torch.randn(kc, dp, generator=g, dtype=torch.float64) * torch.pow(
        2.0, torch.randint(-20, 4, (kc, dp), generator=g)).double()
    cb = torch.zeros(kp, dp, dtype=torch.bfloat16)
    cb[:kc] = c.to(torch.bfloat16)
    cbd = cb.to(dev)
    cn = torch.zeros(kp, dtype=torch.float32, device=dev)
    cn64 = torch.zeros(kp, dtype=torch.float64, device=dev)
    old = torch.zeros_like(cbd)
    drift = torch.zeros(kp, dtype=torch.float32, device=dev)
    K.mx_snap(cbd, kc, dp, cn, cn64=cn64, cb_old=old, drift=drift)
    got = cbd.cpu()
    ref = _snap_ref(cb[:kc])
    assert torch.equal(got[:kc].double(), ref), "snap != torch model of the e4m3 split"
    assert torch.equal(got[:kc].double(), got[:kc].to(torch.bfloat16).double())
    assert torch.equal(got[kc:], cb[kc:])
    # values within 2^-12 of their block's largest are untouched
    v = cb[:kc].double().reshape(kc, dp // 32, 32)
    near = (v.abs() >= v.abs().amax(-1, keepdim=True) * 2.0 ** -12).reshape(kc, dp)
    assert torch.equal(got[:kc].double()[near], cb[:kc].double()[near])
    assert (got[:kc].double() != cb[:kc].double()).any(), "the test data should exercise the lossy case"
    torch.testing.assert_close(cn64[:kc].cpu(), (got[:kc].double() ** 2).sum(1), rtol=1e-14, atol=0)
    torch.testing.assert_close(cn[:kc].cpu().double(), (got[:kc].double() ** 2).sum(1), rtol=1e-6, atol=0)
    assert (drift[:kc].cpu().double() >= got[:kc].double().norm(dim=1)).all()
    again = cbd.clone()
    K.mx_snap(again, kc, dp, cn)
    assert torch.equal(again, cbd), "snapping is idempotent"


def _fp8_blobs(n, d, k, seed, scale):
    g = torch.Generator(device="cuda")
    g.manual_seed(seed)
    cen = torch.randn(k, d, generator=g, device="cuda") * scale
    lab = torch.randint(0, k, (n,), generator=g, device="cuda")
    return (cen[lab] + torch.randn(n, d, generator=g, device="cuda")).clamp(-440, 440).to(torch.float8_e4m3fn)


@pytest.mark.parametrize("n,d,k", [(50_000, 512, 128), (40_000, 256, 200), (30_000, 512, 64)])
def test_mx_assign_matches_exact_within_band(n, d, k):
    """K9r on fp8 rows with MX arithmetic (default) against f64 distances to the snapped centres: the squared
    distance it reports is within tau·(|x|² + max|c|²) of the exact one, and its label is the exact argmin
    wherever the exact top-2 gap exceeds twice that; the bf16 widening pass (CML_KMEANS_FP8_MX=0) agrees
    with it outside the same band."""
    from clustermachinelearningforhospitalnetworks_apache_spark_amd.models.kmeans import LloydEngine, assign_gpu
    x8 = _fp8_blobs(n, d, k, seed=n, scale=0.4)
    init = x8[:k].double()
    assert K.fp8_mx_on()
    lab_mx, best_mx = assign_gpu(x8, d, d, init)
    eng = LloydEngine(x8, d, k, use_graph=False)
    assert eng._mx
    eng.set_centers(init)
    cb = eng.cb[:k, :d].double()
    xd = x8.double()
    d2 = (xd * xd).sum(1, keepdim=True) - 2.0 * xd @ cb.t() + (cb * cb).sum(1)[None, :]
    top = d2.topk(2, dim=1, largest=False)
    tau = eng._tau
    slack = tau * ((xd * xd).sum(1) + (cb * cb).sum(1).max())
    assert ((best_mx.double() - top.values[:, 0]).abs() <= slack).all()
    clear = (top.values[:, 1] - top.values[:, 0]) > 2 * slack
    assert clear.float().mean() > 0.5
    assert torch.equal(lab_mx.long()[clear], top.indices[:, 0][clear])
    prev = K.set_fp8_mx(False)
    try:
        lab_bf, _ = assign_gpu(x8, d, d, cb)  # the snapped centres, widening pass
    finally:
        K.set_fp8_mx(prev)
    assert torch.equal(lab_bf.long()[clear], lab_mx.long()[clear])
    print(f"MX vs bf16 pass: {(lab_bf != lab_mx).sum().item()} of {n} labels differ, all inside the band")


@pytest.mark.parametrize("n,d,k,scale", [(120_000, 512, 128, 0.5), (100_000, 256, 64, 1.0)])
def test_mx_pruned_step_equals_unpruned(n, d, k, scale):
    """Device pruned steps (K9r MX modes 1 and 2, snapped centres) against unpruned steps (MX mode 0): the same
    labels and centres at every step."""
    from clustermachinelearningforhospitalnetworks_apache_spark_amd.models.kmeans import LloydEngine
    x8 = _fp8_blobs(n, d, k, seed=n + d, scale=scale)
    init = x8[:k].float().double().cpu().numpy()
    a = LloydEngine(x8, d, k, prune=False, use_graph=False)
    b = LloydEngine(x8, d, k, prune=True, use_graph=False)
    assert a._mx and b._mx
    a.set_centers(init)
    b.set_centers(init)
    for _ in range(8):
        a.step()
        b.step()
        assert torch.equal(a.labels[:n].long(), b.labels[:n].long())
        torch.testing.assert_close(b.centers, a.centers, rtol=1e-12, atol=1e-12)
        assert torch.equal(a.cb, b.cb)
