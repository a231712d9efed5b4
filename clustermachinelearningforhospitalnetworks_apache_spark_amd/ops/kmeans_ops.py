"""Python bindings of the KMeans kernels (K9–K11, ``_native/csrc/kmeans.hip``).

GPU tensors go to the gfx950 HIP kernels; there is no silent fallback — if the
kernel library is missing on a GPU box, the call raises.  CPU tensors use the
torch reference implementations below (the ``local[n]`` plumbing path and the
numerical oracle of the tests).
"""
from __future__ import annotations

import ctypes
from dataclasses import dataclass

import torch

from .. import _native
from ..utils.device import LDS_BUDGET, next_pow2, num_cus, round_up


@dataclass
class AssignPlan:
    n: int
    dp: int
    kp: int
    kc: int            # centres per launch (multiple of 32)
    grid: int


@dataclass
class AccumPlan:
    lpr: int
    dsl: int
    nsl: int
    gx: int


def plan_assign(n: int, dp: int, k: int, device_index: int = 0) -> AssignPlan:
    lib = _native.kernels()
    kp = round_up(max(k, 1), 32)
    kc = kp
    while kc > 32 and lib.cml_kmeans_assign_lds_bytes(kc, dp) > LDS_BUDGET:
        kc -= 32
    lds = lib.cml_kmeans_assign_lds_bytes(kc, dp)
    if lds > LDS_BUDGET:
        raise ValueError(f"feature width {dp} too large for the LDS-resident centroid tile")
    waves = lib.cml_kmeans_assign_threads() // 64
    per_cu = max(1, min(4, (160 * 1024) // max(lds, 1)))
    ntiles = (n + 31) // 32
    grid = max(1, min((ntiles + waves - 1) // waves, num_cus(device_index) * per_cu))
    return AssignPlan(n=n, dp=dp, kp=kp, kc=kc, grid=grid)


def plan_accum(n: int, dp: int, k: int, device_index: int = 0) -> AccumPlan:
    lpr = min(64, max(1, dp // 2))
    while lpr > 1 and k * 2 * lpr * 4 + 4 * k > 128 * 1024:
        lpr //= 2
    lpr = min(lpr, next_pow2(lpr))
    dsl = 2 * lpr
    nsl = (dp + dsl - 1) // dsl
    lds = k * dsl * 4 + 4 * k
    per_cu = max(1, min(2, (160 * 1024) // max(lds, 1)))
    rows_per_wg = 16 * (64 // lpr) * 4  # waves * rows/wave-iter * unroll
    want = max(1, (n + rows_per_wg - 1) // rows_per_wg)
    gx = max(1, min(want, (num_cus(device_index) * per_cu + nsl - 1) // nsl))
    return AccumPlan(lpr=lpr, dsl=dsl, nsl=nsl, gx=gx)


def assign_bf16(x: torch.Tensor, n: int, dp: int, cb: torch.Tensor, cnorm: torch.Tensor, plan: AssignPlan,
                labels: torch.Tensor, best: torch.Tensor, cost_part: torch.Tensor | None,
                stream=None) -> None:
    """K9: labels/best[i] = argmin/min_j ||x_i - c_j||² over all kp (padded) centres."""
    lib = _native.kernels()
    st = _native.stream_ptr(stream)
    nch = (plan.kp + plan.kc - 1) // plan.kc
    for ci in range(nch):
        c0 = ci * plan.kc
        kc = min(plan.kc, plan.kp - c0)
        status = lib.cml_kmeans_assign_bf16(
            x.data_ptr(), n, x.stride(0), dp,
            cb.data_ptr() + c0 * cb.stride(0) * 2, cb.stride(0), kc, c0,
            cnorm.data_ptr() + c0 * 4, labels.data_ptr(), best.data_ptr(),
            int(ci == 0), int(ci == nch - 1),
            cost_part.data_ptr() if (cost_part is not None and ci == nch - 1) else 0,
            plan.grid, st)
        _native.check(status, "kmeans_assign_bf16")


def accumulate_bf16(x: torch.Tensor, n: int, labels: torch.Tensor, k: int, plan: AccumPlan,
                    slab: torch.Tensor, cslab: torch.Tensor, stream=None) -> None:
    """K10: slab[sl][g][c][d] = Σ_{rows of WG g, label c} x[row, sl*dsl + d]."""
    lib = _native.kernels()
    status = lib.cml_kmeans_accum_bf16(x.data_ptr(), n, x.stride(0), labels.data_ptr(), k, plan.lpr,
                                       slab.data_ptr(), cslab.data_ptr(), plan.gx, plan.nsl,
                                       _native.stream_ptr(stream))
    _native.check(status, "kmeans_accum_bf16")


def reduce_slabs(slab, cslab, cost_part, ncost: int, k: int, d: int, plan: AccumPlan, out: torch.Tensor,
                 stream=None) -> None:
    """K10b: out = [Σx per (c,d) | count per c | cost] in f64, fixed summation order."""
    lib = _native.kernels()
    status = lib.cml_kmeans_reduce(slab.data_ptr(), cslab.data_ptr(), cost_part.data_ptr(), plan.gx, ncost, k,
                                   d, plan.dsl, out.data_ptr(), _native.stream_ptr(stream))
    _native.check(status, "kmeans_reduce")


def update_centers(msgs: torch.Tensor | None, k: int, d: int, cent: torch.Tensor, cb: torch.Tensor, dp: int,
                   kp: int, cnorm: torch.Tensor, shift2: torch.Tensor | None, stream=None) -> None:
    """K11: cent <- Σx/count (empty clusters keep their centre), cb <- bf16(cent), cnorm <- ||cb||²."""
    lib = _native.kernels()
    if msgs is not None:
        nbuf, bstride, mp = msgs.shape[0], msgs.stride(0), msgs.data_ptr()
    else:
        nbuf, bstride, mp = 0, 0, 0
    status = lib.cml_kmeans_update(mp, nbuf, bstride, k, d, cent.data_ptr(), cb.data_ptr(), cb.stride(0), dp, kp,
                                   cnorm.data_ptr(), shift2.data_ptr() if shift2 is not None else 0,
                                   _native.stream_ptr(stream))
    _native.check(status, "kmeans_update")


# ----------------------------------------------------------------------------------------------
# CPU reference implementations (torch, float64) — identical semantics, used by local[n] mode.
# ----------------------------------------------------------------------------------------------

def assign_reference(x: torch.Tensor, centers: torch.Tensor, chunk: int = 1 << 16):
    """Return (labels int64, min squared distance f64) with first-index tie breaking."""
    x = x.to(torch.float64)
    c = centers.to(torch.float64)
    cn = (c * c).sum(1)
    labels = torch.empty(x.shape[0], dtype=torch.int64)
    best = torch.empty(x.shape[0], dtype=torch.float64)
    for s in range(0, x.shape[0], chunk):
        xb = x[s:s + chunk]
        sc = cn[None, :] - 2.0 * xb @ c.T
        m, i = sc.min(1)
        labels[s:s + chunk] = i
        best[s:s + chunk] = torch.clamp((xb * xb).sum(1) + m, min=0.0)
    return labels, best


def sums_reference(x: torch.Tensor, labels: torch.Tensor, k: int):
    x = x.to(torch.float64)
    sums = torch.zeros(k, x.shape[1], dtype=torch.float64)
    sums.index_add_(0, labels, x)
    counts = torch.bincount(labels, minlength=k).to(torch.float64)
    return sums, counts
