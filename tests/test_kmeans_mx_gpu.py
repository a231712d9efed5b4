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


def test_mx_centres_split():
    dev = torch.device("cuda", 0)
    g = torch.Generator(device="cpu").manual_seed(5)
    kc, kp, dp = 40, 48, 256
    c = torch.randn(kc, dp, generator=g, dtype=torch.float64) * torch.pow(2.0, torch.randint(-12, 4, (kc, dp),
                                                                                           generator=g)).double()
    cb = torch.zeros(kp, dp, dtype=torch.bfloat16)
    cb[:kc] = c.to(torch.bfloat16)
    mc, ms, cn, stat = K.mx_centres(cb.to(dev), kc, kp, dp)
    mc, ms, cn, stat = mc.cpu(), ms.cpu(), cn.cpu(), stat.cpu()
    nb = dp // 128
    # rebuild -2·~c in the natural k order from the lane-ordered bytes and scales
    v = torch.zeros(kp, dp, dtype=torch.float64)
    for blk in range(nb):
        for q in range(4):  # lane group q: chunks 8·blk + q (bytes 0-15) and 8·blk + 4 + q (bytes 16-31)
            for h in range(2):
                ch = 8 * blk + q + 4 * h
                sc = ms[:, blk, (q + 4 * h) // 2]  # scale block of chunk ch: k // 32 within the MX block
                hi = _dec(mc[:, blk, q, 16 * h:16 * h + 16]) * torch.pow(2.0, ((sc & 255) - 127).double())[:, None]
                lo = _dec(mc[:, blk, q, 32 + 16 * h:48 + 16 * h]) * torch.pow(2.0, (((sc >> 8) & 255) - 127)
                                                                               .double())[:, None]
                v[:, 16 * ch:16 * ch + 16] = hi + lo
    ct = -0.5 * v[:kc]
    cbd = cb[:kc].double()
    e = (ct - cbd).norm(dim=1)
    assert (stat[:kc].double() >= e).all() and (stat[:kc].double() <= e * (1 + 1e-5) + 1e-29).all()
    assert (stat[kc:] == 0).all()
    torch.testing.assert_close(cn[:kc].double(), (ct * ct).sum(1), rtol=1e-6, atol=0)
    assert torch.isinf(cn[kc:]).all()
    # hi + lo keeps every bf16 value within 2^-8 of its block maximum exactly
    rel = ((ct - cbd).abs() / cbd.abs().clamp(min=1e-300))
    big = cbd.abs() >= cbd.abs().amax(dim=1, keepdim=True) * 2.0 ** -5
    assert (rel[big] == 0).all()


def _fp8_blobs(n, d, k, seed, scale):
    g = torch.Generator(device="cuda")
    g.manual_seed(seed)
    cen = torch.randn(k, d, generator=g, device="cuda") * scale
    lab = torch.randint(0, k, (n,), generator=g, device="cuda")
    return (cen[lab] + torch.randn(n, d, generator=g, device="cuda")).clamp(-440, 440).to(torch.float8_e4m3fn)


@pytest.mark.parametrize("n,d,k,scale,cap", [(120_000, 512, 128, 0.5, None), (100_000, 256, 64, 1.0, None),
                                             (60_000, 256, 32, 0.3, "0.001")])
def test_fp8_screen_step_equals_bf16_pass(n, d, k, scale, cap, monkeypatch):
    """The device pruned step on fp8 rows, whose full passes run the MX screen + bf16 re-check (or, past the
    list capacity, the bf16 pass), against the unpruned engine (bf16 widening pass): the same labels and
    centres at every step."""
    from clustermachinelearningforhospitalnetworks_apache_spark_amd.models.kmeans import LloydEngine
    if cap is not None:
        monkeypatch.setenv("CML_KMEANS_PRUNE_CAP", cap)
    x8 = _fp8_blobs(n, d, k, seed=n + d, scale=scale)
    init = x8[:k].float().double().cpu().numpy()
    a = LloydEngine(x8, d, k, prune=False, use_graph=False)
    b = LloydEngine(x8, d, k, prune=True, use_graph=False)
    a.set_centers(init)
    b.set_centers(init)
    screened = []
    for _ in range(8):
        a.step()
        b.step()
        assert torch.equal(a.labels[:n].long(), b.labels[:n].long())
        torch.testing.assert_close(b.centers, a.centers, rtol=1e-12, atol=1e-12)
        st = b.prune_stats()
        if "screen_rechecked" in st:
            screened.append(st["screen_rechecked"])
    assert b._pst.screen and screened, "no full step ran the screen"
    print(f"fp8 screen: rows re-checked by the bf16 pass per full step {screened} of {n}")
    if cap is None:
        assert min(screened) < n // 4  # the screen certifies most rows
    else:
        assert max(screened) > b._pst.cap_m  # the list overflowed: the bf16 fallback pass ran
