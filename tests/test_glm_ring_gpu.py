"""K13 (logistic / hinge / squared gradient) and K7 (column moments) on the U + 1 slot prefetch ring
(`_native/csrc/glm.hip`, profiles/r6/README.md §10): every forced depth against the f64 host reference, at row
counts that end inside the first group, inside the ring and mid-grid (rows past n re-read row n - 1 with weight 0),
with and without a weight column, and at widths whose last chunk is partial. Also: the same accumulation order at
every depth, so K7 gives the same bits at depth 1 and 2 for one grid."""
import pytest
import torch

from clustermachinelearningforhospitalnetworks_apache_spark_amd.ops import glm_ops

pytestmark = pytest.mark.gpu

SHAPES = [(torch.bfloat16, 256), (torch.float8_e4m3fn, 512), (torch.float32, 100), (torch.bfloat16, 37),
          (torch.float8_e4m3fn, 48)]
ROWS = [1, 63, 1000, 200_003]


def _data(n, d, dt, seed):
    g = torch.Generator().manual_seed(seed)
    x = torch.randn(n, d, generator=g)
    x = (x.to(torch.bfloat16) if dt == torch.float8_e4m3fn else x).to(dt)
    y = (torch.rand(n, generator=g) > 0.5).double()
    w = torch.rand(n, generator=g, dtype=torch.float64) + 0.5
    coef = torch.randn(d + 1, generator=g, dtype=torch.float64) * 0.05
    return x, y, w, coef


def _close(got, ref, rtol):
    scale = ref.abs().max().item() + 1e-30
    assert (got.cpu() - ref).abs().max().item() <= rtol * scale, (got.cpu() - ref).abs().max().item() / scale


@pytest.mark.parametrize("dt,d", SHAPES)
@pytest.mark.parametrize("n", ROWS)
def test_logreg_ring_depths_match_f64(dt, d, n):
    x, y, w, coef = _data(n, d, dt, seed=n + d)
    xc = x.cuda()
    try:
        for weight in (None, w):
            ref = glm_ops.logreg_grad(x, d, y, coef, weight)
            for u in (1, 2, 0):
                glm_ops.set_logreg_unroll(u)
                got = glm_ops.logreg_grad(xc, d, y.cuda(), coef.cuda(), None if weight is None else weight.cuda())
                _close(got, ref, 2e-5)
                assert abs(got[-1].item() - ref[-1].item()) <= 1e-6 * max(1.0, ref[-1].item())  # weight sum
    finally:
        glm_ops.set_logreg_unroll(0)


@pytest.mark.parametrize("loss", ["hinge", "squared"])
@pytest.mark.parametrize("dt,d", SHAPES[:3])
def test_loss_grad_ring_matches_f64(loss, dt, d):
    n = 70_001
    x, y, w, coef = _data(n, d, dt, seed=7)
    ref = glm_ops.loss_grad(x, d, y, coef, w, loss=loss)
    got = glm_ops.loss_grad(x.cuda(), d, y.cuda(), coef.cuda(), w.cuda(), loss=loss)
    _close(got, ref, 2e-5)


@pytest.mark.parametrize("dt,d", SHAPES)
@pytest.mark.parametrize("n", ROWS)
def test_moments_ring_depths_match_f64(dt, d, n):
    x, _, _, _ = _data(n, d, dt, seed=3 * n + d)
    ref = glm_ops.moments(x, d)
    xc = x.cuda()
    try:
        bits = None
        # x - shift is formed in f32 (exact for bf16 / e4m3 rows unless their exponents are ~16 apart)
        tol = 1e-6 if dt == torch.float32 else 1e-9
        for u in (1, 2):
            glm_ops.set_moments_unroll(u)
            cnt, s1, s2, shift = glm_ops.moments(xc, d)
            assert cnt == ref[0]
            _close(s1, ref[1], tol)
            _close(s2, ref[2], tol)
            cur = torch.cat([s1, s2])
            bits = cur if bits is None else bits
            assert torch.equal(cur, bits)  # one grid, the same per-lane order at either depth
    finally:
        glm_ops.set_moments_unroll(0)


@pytest.mark.parametrize("dt,code,d", [(torch.float8_e4m3fn, 3, 512), (torch.bfloat16, 0, 256)])
def test_logreg_kernel_empty_shard_writes_zero_partials(dt, code, d):
    """n = 0 straight into the kernel (the wrapper takes the host path): no load of row n - 1, zero partials."""
    from clustermachinelearningforhospitalnetworks_apache_spark_amd import _native

    x = torch.zeros(1, d, dtype=dt, device="cuda")
    y = torch.zeros(1, dtype=torch.float64, device="cuda")
    coef = torch.zeros(d + 1, dtype=torch.float64, device="cuda")
    out = torch.full((4, d + 3), float("nan"), dtype=torch.float64, device="cuda")
    st = _native.kernels().cml_logreg_grad(x.data_ptr(), 0, x.stride(0), d, code, y.data_ptr(), 0, coef.data_ptr(),
                                           out.data_ptr(), 4, 0, _native.stream_ptr())
    _native.check(st, "logreg_grad")
    torch.cuda.synchronize()
    assert torch.equal(out, torch.zeros_like(out))
