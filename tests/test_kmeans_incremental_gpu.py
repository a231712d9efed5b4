"""Incremental-sums Lloyd step (kmeans.hip kmeans_delta_*) against the full re-accumulation.

The engine keeps the per-cluster sums of the current labels and, on steps where few labels change,
applies only the changed rows. On data whose f64 sums are exact (values on a 1/8 grid) the two
must agree bit for bit; on general data to f64 rounding.
"""
import numpy as np
import pytest
import torch

from clustermachinelearningforhospitalnetworks_apache_spark_amd.models.kmeans import LloydEngine

pytestmark = pytest.mark.gpu


@pytest.fixture(autouse=True)
def _full_steps_only(monkeypatch):
    """These tests target the full / incremental MFMA step machinery: pruned steps off by default, and
    f32/f64 rows take the bf16 path (not the source-precision one, tests/test_kmeans_exact_gpu.py)."""
    monkeypatch.setenv("CML_KMEANS_PRUNE", "0")
    monkeypatch.setenv("CML_KMEANS_PRECISION", "bf16")


def _blobs(n, d, k, seed, grid=True, dtype=torch.bfloat16):
    g = torch.Generator(device="cuda")
    g.manual_seed(seed)
    cen = torch.randn(k, d, device="cuda", generator=g) * 3
    x = cen[torch.randint(0, k, (n,), device="cuda", generator=g)] + torch.randn(n, d, device="cuda", generator=g)
    if grid:
        x = torch.round(x * 8) / 8  # exact in bf16, f64 sums exact
    return x.to(dtype)


def _run(x, d, k, init, steps, **kw):
    eng = LloydEngine(x, d, k, **kw)
    eng.set_centers(init)
    hist = []
    for _ in range(steps):
        eng.step()
        torch.cuda.synchronize()
        full = eng.delta.was_full() if eng.delta is not None else True
        ch = eng.delta.changed_rows() if eng.delta is not None else -1
        hist.append((eng.centers.clone(), eng.msgs.clone(), full, ch))
    return eng, hist


@pytest.mark.parametrize("n,d,k", [(200_000, 256, 256), (150_001, 128, 64), (60_000, 512, 40)])
def test_incremental_equals_full_bitwise(n, d, k):
    x = _blobs(n, d, k, seed=1)
    init = x[torch.randperm(n, generator=torch.Generator().manual_seed(0))[:k]].double().cpu().numpy()
    eng, inc = _run(x, d, k, init, 8, accum_mode="sort", use_graph=False)
    assert eng.delta is not None
    _, ful = _run(x, d, k, init, 8, accum_mode="sort", use_graph=False, incremental=False)
    assert inc[0][2], "first step must re-accumulate in full"
    assert any(not h[2] and h[3] > 0 for h in inc), "no step took the incremental path"
    for (ci, mi, _, _), (cf, mf, _, _) in zip(inc, ful):
        assert torch.equal(mi, mf)
        assert torch.equal(ci, cf)


def test_incremental_general_data_and_graph():
    """Unrounded Gaussian data (f64 rounding only) and the captured-graph step."""
    n, d, k = 120_000, 256, 128
    x = _blobs(n, d, k, seed=2, grid=False)
    init = x[:k].double().cpu().numpy()
    _, ful = _run(x, d, k, init, 6, accum_mode="sort", use_graph=False, incremental=False)
    for use_graph in (False, True):
        eng, inc = _run(x, d, k, init, 6, accum_mode="sort", use_graph=use_graph)
        assert any(not h[2] for h in inc)
        for (ci, mi, _, _), (cf, mf, _, _) in zip(inc, ful):
            np.testing.assert_allclose(mi.cpu().numpy(), mf.cpu().numpy(), rtol=1e-12, atol=1e-9)
            np.testing.assert_allclose(ci.cpu().numpy(), cf.cpu().numpy(), rtol=1e-12, atol=1e-12)


def test_incremental_falls_back_when_many_labels_change():
    """More changed rows than the change log holds: the step re-accumulates in full."""
    n, d, k = 100_000, 128, 64
    x = _blobs(n, d, k, seed=3)
    init = (x[:k].double() + 5.0).cpu().numpy()  # far-off start: many labels move for a few steps
    eng = LloydEngine(x, d, k, accum_mode="sort", use_graph=False)
    eng.delta.cap = 1500
    eng.set_centers(init)
    _, ful = _run(x, d, k, init, 6, accum_mode="sort", use_graph=False, incremental=False)
    modes = []
    for s in range(6):
        eng.step()
        torch.cuda.synchronize()
        modes.append(eng.delta.was_full())
        assert torch.equal(eng.msgs, ful[s][1])
    assert modes[0] and sum(modes) >= 2  # forced first step + at least one overflow fallback


def test_incremental_fp8_and_row_chunks():
    n, d, k = 90_000, 256, 96
    xb = _blobs(n, d, k, seed=4, grid=False, dtype=torch.float32)
    for x, chunks in ((xb.to(torch.float8_e4m3fn), 1), (xb.to(torch.bfloat16), 3)):
        init = x[:k].to(torch.float32).double().cpu().numpy()
        eng, inc = _run(x, d, k, init, 5, accum_mode="sort", use_graph=False, row_chunks=chunks)
        _, ful = _run(x, d, k, init, 5, accum_mode="sort", use_graph=False, row_chunks=chunks, incremental=False)
        assert eng.delta is not None and eng.row_chunks == chunks
        for (ci, mi, _, _), (cf, mf, _, _) in zip(inc, ful):
            np.testing.assert_allclose(mi.cpu().numpy(), mf.cpu().numpy(), rtol=1e-12, atol=1e-9)


def test_row_norm_cache_follows_tensor_version():
    """cached_row_sqnorm: reused for the same unmodified device matrix, recomputed after a write."""
    from clustermachinelearningforhospitalnetworks_apache_spark_amd.models.kmeans import (
        assign_gpu, cached_row_sqnorm, to_device_matrix)
    n, d, k = 40_000, 256, 32
    x = to_device_matrix(_blobs(n, d, k, seed=6), d)
    eng = LloydEngine(x, d, k, use_graph=False)
    xn0 = eng.xnorm  # computed on first use (or by the k-means|| first pass), then cached on the tensor
    assert eng.x is x and getattr(x, "_cml_xnorm")[2] is xn0
    assert cached_row_sqnorm(x, n, eng.dp) is eng.xnorm
    c = x[:k, :d].double()
    _, best0 = assign_gpu(x, eng.dp, d, c)
    scale = float(eng.xnorm[:k].max().item())
    assert float(best0[:k].abs().max().item()) <= 1e-5 * scale  # each of the first k rows is its own centre
    x[0].mul_(2.0)  # in-place write: the cached norms must not be reused
    xn = cached_row_sqnorm(x, n, eng.dp)
    assert xn is not eng.xnorm
    ref = x[:, :d].float().pow(2).sum(1)
    torch.testing.assert_close(xn, ref, rtol=1e-5, atol=1e-3)
    _, best1 = assign_gpu(x, eng.dp, d, c)
    ref0 = (x[0, :d].double() - c).pow(2).sum(1).min().item()
    assert abs(best1[0].item() - ref0) <= 1e-5 * 4 * scale + 1e-4 * ref0


def test_invalidate_forces_full_step():
    n, d, k = 50_000, 64, 16
    x = _blobs(n, d, k, seed=5)
    eng = LloydEngine(x, d, k, accum_mode="sort", use_graph=False)
    eng.set_centers(x[:k].double().cpu().numpy())
    for _ in range(3):
        eng.step()
    torch.cuda.synchronize()
    eng.delta.invalidate()
    eng.step()
    torch.cuda.synchronize()
    assert eng.delta.was_full()


def test_spherical_gpu_matches_cpu_engine():
    """distanceMeasure="cosine" on the MFMA path: unit bf16 rows, renormalised centres, vs the f64 CPU engine."""
    n, d, k = 60_000, 96, 24
    rs = np.random.RandomState(11)
    dirs = rs.randn(k, d)
    dirs /= np.linalg.norm(dirs, axis=1, keepdims=True)
    x = (dirs[rs.randint(0, k, n)] + 0.2 * rs.randn(n, d)) * rs.uniform(0.2, 30.0, (n, 1))
    u = x / np.linalg.norm(x, axis=1, keepdims=True)
    init = u[:k].copy()
    cpu = LloydEngine(torch.as_tensor(x), d, k, spherical=True)
    cpu.set_centers(init)
    gpu = LloydEngine(torch.as_tensor(x, dtype=torch.float32, device="cuda"), d, k, spherical=True)
    gpu.set_centers(init)
    for _ in range(8):
        cpu.step()
        gpu.step()
    torch.cuda.synchronize()
    cg = gpu.centers.cpu().numpy()
    np.testing.assert_allclose(np.linalg.norm(cg, axis=1), 1.0, rtol=1e-12)
    np.testing.assert_allclose(cg, cpu.centers.numpy(), atol=1e-2)  # bf16 unit rows vs f64 (2^-9 relative per element)
    lab_g = gpu.labels[:n].long().cpu().numpy()
    assert (lab_g == cpu.labels.numpy()).mean() > 0.995
    assert abs(gpu.training_cost() - cpu.training_cost()) <= 2e-2 * cpu.training_cost()
    assert gpu.delta is not None and gpu.converged(1.0)


@pytest.mark.parametrize("wide", [True, False])
def test_sum_grid_keeps_incremental_equal_to_full(wide):
    """Exactness guard of the incremental sums (models/kmeans.py _sum_grid): rows whose values span
    2^-30 .. 2^20 break the f64 window (log2 n + span + 8 > 53), so the rows are summed on a grid and
    the full, incremental and pruned fits stay equal bit for bit after 20 steps; a narrow span keeps
    plain f64 sums (no grid). A periodic full re-accumulation (refresh_interval) gives the same bits."""
    n, d, k = 200_000, 128, 16
    g = torch.Generator(device="cuda").manual_seed(3)
    if wide:
        mag = torch.exp2(torch.rand(n, d, device="cuda", generator=g) * 50 - 30)
        sgn = torch.where(torch.rand(n, d, device="cuda", generator=g) < 0.5, -1.0, 1.0)
        cen = torch.randn(k, d, device="cuda", generator=g) * 2 ** 18
        x = cen[torch.randint(0, k, (n,), device="cuda", generator=g)] + sgn * mag
    else:
        cen = torch.randn(k, d, device="cuda", generator=g) * 4
        x = cen[torch.randint(0, k, (n,), device="cuda", generator=g)] + torch.randint(
            -8, 9, (n, d), device="cuda", generator=g).float() / 4
    x = x.to(torch.bfloat16)
    init = x[:k].double().cpu().numpy()
    res = {}
    for name, kw in (("incremental", dict(prune=False)), ("full", dict(prune=False, incremental=False)),
                     ("pruned", dict(prune=True)), ("refresh", dict(prune=True, refresh_interval=3))):
        eng = LloydEngine(x, d, k, precision="bf16", accum_mode="sort", **kw)
        eng.set_centers(init)
        for _ in range(20):
            eng.step()
        torch.cuda.synchronize()
        res[name] = (eng.centers.cpu().numpy(), eng.sum_grid)
    assert np.array_equal(res["incremental"][0], res["full"][0])
    assert np.array_equal(res["pruned"][0], res["full"][0])
    assert np.array_equal(res["refresh"][0], res["full"][0])  # periodic full re-accumulation changes nothing
    assert (res["full"][1] is not None) == wide and (res["incremental"][1] is not None) == wide
