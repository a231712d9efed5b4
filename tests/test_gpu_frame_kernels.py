"""GPU numerics of the frame kernels (K2 assemble, K3 compact, K5 split, K22 Poisson, K6 binarize,
K23 metric sums, K4 fp8 quantisation) against the torch CPU paths of the same operations."""
import numpy as np
import pytest
import torch

from clustermachinelearningforhospitalnetworks_apache_spark_amd.ops import frame_ops as F
from clustermachinelearningforhospitalnetworks_apache_spark_amd.utils import rng
from clustermachinelearningforhospitalnetworks_apache_spark_amd.ml.evaluation import reg_sums_torch
from clustermachinelearningforhospitalnetworks_apache_spark_amd.ml.feature import VectorAssembler

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("n", [0, 1, 4095, 4096, 4097, 1_000_003])
@pytest.mark.parametrize("p", [0.0, 0.3, 1.0])
def test_compact_matches_nonzero(n, p):
    g = torch.Generator().manual_seed(n)
    m = torch.rand(n, generator=g) < p
    got = F.compact(m.cuda()).cpu()
    want = torch.nonzero(m).flatten()
    assert torch.equal(got, want)


def test_counter_rng_bit_exact():
    g = torch.Generator().manual_seed(0)
    rows = torch.randint(-(2**62), 2**62, (100_001,), generator=g, dtype=torch.int64)
    rows[:5] = torch.tensor([0, 1, -1, 2**40 + 7, 123456789])
    for seed, stream in [(42, 2), (7, 1003), (2**31 - 1, 21)]:
        assert torch.equal(rng.uniform(rows.cuda(), seed, stream).cpu(), rng.uniform(rows, seed, stream))
        assert torch.equal(rng.poisson1(rows.cuda(), seed, stream).cpu(), rng.poisson1(rows, seed, stream))
        cum = [0.0, 0.7, 1.0 + 1e-12]
        b = F.split_buckets(rows.cuda(), rng.key(seed, stream), cum).cpu().long()
        u = rng.uniform(rows, seed, stream)
        assert torch.equal(b, (u >= 0.7).long())


def test_random_split_gpu_equals_cpu():
    import pandas as pd
    from clustermachinelearningforhospitalnetworks_apache_spark_amd.sql import SparkSession
    rs = np.random.RandomState(3)
    pdf = pd.DataFrame({"a": rs.randn(5000), "b": rs.randint(0, 9, 5000)})
    outs = {}
    for master in ("mi355x", "local[1]"):
        spark = SparkSession.builder.appName("split").master(master).getOrCreate()
        df = spark.createDataFrame(pdf)
        parts = df.randomSplit([0.5, 0.3, 0.2], seed=11)
        outs[master] = [sorted(r.a for r in p.collect()) for p in parts]
        spark.stop()
    assert outs["mi355x"] == outs["local[1]"]


@pytest.mark.parametrize("out_dtype", [torch.float64, torch.float32, torch.bfloat16])
def test_assemble_matches_torch(out_dtype):
    n = 10_007
    g = torch.Generator().manual_seed(1)
    cols = [torch.randint(-100, 100, (n,), generator=g, dtype=torch.int32),
            torch.randn(n, generator=g, dtype=torch.float64),
            torch.randn(n, generator=g).to(torch.float32),
            torch.randint(0, 2, (n,), generator=g).to(torch.bool),
            torch.randn(n, 3, generator=g, dtype=torch.float64),
            torch.randint(-5, 5, (n,), generator=g, dtype=torch.int64)]
    cols[2][::97] = float("nan")
    valid = [None, torch.rand(n, generator=g) > 0.05, None, None, None, torch.rand(n, generator=g) > 0.01]

    class _CD:
        def __init__(self, v, m):
            self.values, self.valid = v, m

        def valid_mask(self):
            return self.valid if self.valid is not None else torch.ones(self.values.shape[0], dtype=torch.bool)

    class _DF:
        _nrows = n
        _device = torch.device("cpu")

    want, wbad = VectorAssembler._assemble_torch(_DF, [_CD(v, m) for v, m in zip(cols, valid)])
    got, gbad = F.assemble([(v.cuda(), None if m is None else m.cuda()) for v, m in zip(cols, valid)],
                           out_dtype=out_dtype)
    assert torch.equal(gbad.cpu(), wbad)
    np.testing.assert_array_equal(np.isnan(got.double().cpu().numpy()), np.isnan(want.numpy()))
    ok = ~torch.isnan(want)
    g_ok, w_ok = got.double().cpu()[ok], want.to(out_dtype).double()[ok]
    if out_dtype == torch.bfloat16:
        # torch rounds f64 -> f32 -> bf16 (twice); the GPU conversion rounds once, so values within
        # 2^-24 of a bf16 midpoint may land one ulp apart (always on the correctly rounded side).
        diff = (g_ok - w_ok).abs()
        ulp = w_ok.abs().clamp(min=1e-30) * 2.0 ** -7
        assert (diff <= ulp * 1.01).all() and (diff > 0).float().mean() < 1e-3
        exact = (want[ok] - g_ok).abs() <= (want[ok] - w_ok).abs()
        assert exact.all()
    else:
        assert torch.equal(g_ok, w_ok)


def test_binarize_and_metric_sums():
    n = 300_001
    g = torch.Generator().manual_seed(5)
    y = torch.randn(n, generator=g, dtype=torch.float64) * 3 + 5
    p = y + torch.randn(n, generator=g, dtype=torch.float64)
    w = torch.rand(n, generator=g, dtype=torch.float64)
    assert torch.equal(F.binarize(y.cuda(), 5.0).cpu(), (y > 5.0).double())
    for wt in (None, w):
        got = F.reg_metric_sums(y.cuda(), p.cuda(), None if wt is None else wt.cuda()).cpu()
        np.testing.assert_allclose(got.numpy(), reg_sums_torch(y, p, wt).numpy(), rtol=1e-10)
    yl = torch.randint(0, 4, (n,), generator=g)
    pl = torch.randint(0, 4, (n,), generator=g)
    cm = torch.zeros(16, dtype=torch.float64).index_add_(0, yl * 4 + pl, w).reshape(4, 4)
    np.testing.assert_allclose(F.confusion(yl.cuda(), pl.cuda(), 4, w.cuda()).cpu().numpy(), cm.numpy(),
                               rtol=1e-10)


@pytest.mark.parametrize("C", [2, 7, 33, 64])
def test_weighted_confusion_deterministic(C):
    """Fractional weights: the confusion counts are a fixed-order sum (no float atomics), bitwise equal
    across runs, and equal to the f64 oracle at 1e-12."""
    n = 2_000_003
    g = torch.Generator().manual_seed(C)
    yl = torch.randint(0, C, (n,), generator=g)
    pl = torch.where(torch.rand(n, generator=g) < 0.7, yl, torch.randint(0, C, (n,), generator=g))
    w = torch.rand(n, generator=g, dtype=torch.float64) * 3.3 + 1e-3
    a = F.confusion(yl.cuda(), pl.cuda(), C, w.cuda()).cpu()
    b = F.confusion(yl.cuda(), pl.cuda(), C, w.cuda()).cpu()
    assert torch.equal(a, b)
    cm = torch.zeros(C * C, dtype=torch.float64).index_add_(0, yl * C + pl, w).reshape(C, C)
    np.testing.assert_allclose(a.numpy(), cm.numpy(), rtol=1e-12)
    # out-of-range ids are skipped
    yl[:10] = -1
    pl[10:20] = C
    c = F.confusion(yl.cuda(), pl.cuda(), C, None).cpu()
    assert float(c.sum()) == n - 20


@pytest.mark.parametrize("src", [torch.float32, torch.bfloat16])
def test_fp8_quantisation(src):
    n, d = 4099, 37
    g = torch.Generator().manual_seed(9)
    x = (torch.randn(n, d, generator=g) * torch.logspace(-2, 2, d)).to(src)
    amax = F.col_absmax(x.cuda(), d).cpu()
    np.testing.assert_array_equal(amax.numpy(), x.float().abs().amax(0).numpy())
    scale = 448.0 / amax.clamp(min=1e-12)
    q = F.quant_fp8(x.cuda(), d, scale, ld=48).cpu()
    want = (x.float() * scale).clamp(-448, 448).to(torch.float8_e4m3fn)
    assert torch.equal(q[:, :d].view(torch.uint8), want.view(torch.uint8))
    assert (q[:, d:].view(torch.uint8) == 0).all()


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float32, torch.float64])
def test_has_nan(dtype):
    x = torch.randn(10_001, 40, dtype=torch.float64).to(dtype)
    xp = torch.zeros((10_001, 64), dtype=dtype)
    xp[:, :40] = x
    assert not F.has_nan(xp.cuda(), 40)
    xp[7777, 39] = float("nan")
    assert F.has_nan(xp.cuda(), 40)
    xp[7777, 39] = 0
    xp[5, 50] = float("nan")  # beyond d: ignored
    assert not F.has_nan(xp.cuda(), 40)


@pytest.mark.parametrize("out_dtype", [torch.float64, torch.float32, torch.bfloat16])
@pytest.mark.parametrize("ld", [0, 8, 7])
def test_assemble_scalar_fast_path(out_dtype, ld):
    """Scalar-only columns take the register-row / 16-byte-store kernel; padded and odd row widths too."""
    n = 20_011
    g = torch.Generator().manual_seed(3)
    cols = [torch.randint(-100, 100, (n,), generator=g, dtype=torch.int32),
            torch.randn(n, generator=g, dtype=torch.float64),
            torch.randn(n, generator=g).to(torch.float32),
            torch.randint(0, 2, (n,), generator=g).to(torch.bool),
            torch.randint(-5, 5, (n,), generator=g, dtype=torch.int64)]
    cols[1][::89] = float("nan")
    valid = [None, None, torch.rand(n, generator=g) > 0.05, None, torch.rand(n, generator=g) > 0.02]
    got, gbad = F.assemble([(v.cuda(), None if m is None else m.cuda()) for v, m in zip(cols, valid)],
                           out_dtype=out_dtype, ld=ld)
    want = torch.stack([c.double() for c in cols], 1)
    bad = torch.zeros(n, dtype=torch.bool)
    for j, m in enumerate(valid):
        if m is not None:
            want[~m, j] = float("nan")
    bad |= torch.isnan(want).any(1)
    assert torch.equal(gbad.cpu(), bad)
    width = max(ld, 5)
    assert got.shape == (n, width)
    g64 = got.double().cpu()
    np.testing.assert_array_equal(np.isnan(g64[:, :5].numpy()), np.isnan(want.numpy()))
    ok = ~torch.isnan(want)
    assert torch.equal(g64[:, :5][ok], want.to(out_dtype).double()[ok]) or out_dtype == torch.bfloat16
    if width > 5:
        assert (g64[:, 5:] == 0).all()


@pytest.mark.parametrize("src", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("d", [128, 256])
def test_fp8_quantisation_vector_paths(src, d):
    n = 9_001
    g = torch.Generator().manual_seed(11)
    x = (torch.randn(n, d, generator=g) * torch.logspace(-2, 2, d)).to(src)
    amax = F.col_absmax(x.cuda(), d).cpu()
    np.testing.assert_array_equal(amax.numpy(), x.float().abs().amax(0).numpy())
    scale = 448.0 / amax.clamp(min=1e-12)
    q = F.quant_fp8(x.cuda(), d, scale).cpu()
    want = (x.float() * scale).clamp(-448, 448).to(torch.float8_e4m3fn)
    assert torch.equal(q.view(torch.uint8), want.view(torch.uint8))
