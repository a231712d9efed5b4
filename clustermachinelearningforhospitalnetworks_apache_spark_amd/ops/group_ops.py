"""Host wrapper of K25 ``group_reduce`` (``_native/csrc/group.hip``): per-group sum / min / max of
one column with LDS-privatised accumulators, for the few-groups case of SQL group-by.

``group_reduce`` runs the HIP kernel for device tensors when the group count fits the LDS path
(G <= ``max_groups()``) and the torch scatter form otherwise (many groups: little contention) and
for CPU tensors (the oracle of the GPU tests).
"""
from __future__ import annotations

from typing import Optional

import torch

from .. import _native
from .._native import c_int, c_ll, c_vp

_native.register_kernel_sigs({
    "cml_group_reduce": (c_int, [c_vp, c_vp, c_int, c_vp, c_ll, c_int, c_int, c_int, c_int, c_ll, c_ll, c_vp,
                                 c_vp, c_vp]),
    "cml_group_reduce_max_groups": (c_int, []),
})

_OPS = {"sum": 0, "min": 1, "max": 2}
_VTYPES = {torch.float64: 0, torch.float32: 1, torch.int32: 2, torch.int64: 3, torch.uint8: 4, torch.bool: 4}
_MIN_ROWS = 1 << 14   # below this the launch pair costs more than the scatter
_ROWS_PER_BLOCK = 8192


def max_groups() -> int:
    return int(_native.kernels().cml_group_reduce_max_groups())


def _torch_reduce(gid: torch.Tensor, vals: Optional[torch.Tensor], G: int, op: str, mask, floating: bool,
                  n: int) -> torch.Tensor:
    dt = torch.float64 if floating else torch.int64
    v = torch.arange(n, device=gid.device, dtype=dt) if vals is None else vals.to(dt)
    g = gid.to(torch.int64)
    if op == "sum":
        if mask is not None:
            v = torch.where(mask.to(torch.bool), v, torch.zeros_like(v))
        return torch.zeros(G, dtype=dt, device=gid.device).index_add_(0, g, v)
    if floating:
        fill = float("inf") if op == "min" else float("-inf")
    else:
        fill = torch.iinfo(torch.int64).max if op == "min" else torch.iinfo(torch.int64).min
    if mask is not None:
        v = torch.where(mask.to(torch.bool), v, torch.full_like(v, fill))
    out = torch.full((G,), fill, dtype=dt, device=gid.device)
    return out.scatter_reduce_(0, g, v, "amin" if op == "min" else "amax", include_self=True)


def group_reduce(gid: torch.Tensor, vals: Optional[torch.Tensor], G: int, op: str,
                 mask: Optional[torch.Tensor] = None, floating: Optional[bool] = None,
                 ids_in_range: bool = False) -> torch.Tensor:
    """[G] per-group ``op`` ("sum" / "min" / "max") of ``vals`` (None = the row index) over rows whose
    ``mask`` is set. Accumulates in f64 for floating values (or ``floating=True``), else in i64.
    Empty groups hold the identity (0, +inf / -inf, int64 max / min). ``ids_in_range``: the caller
    guarantees 0 <= gid < G (e.g. KMeans labels), so the range check — a host read — is skipped."""
    n = int(gid.shape[0])
    if floating is None:
        floating = vals is not None and vals.is_floating_point()
    if not gid.is_cuda or G > 2048 or n < _MIN_ROWS or G <= 0:
        return _torch_reduce(gid, vals, G, op, mask, floating, n)
    gid32 = gid if gid.dtype == torch.int32 else gid.to(torch.int32)
    gid32 = gid32.contiguous()
    if not ids_in_range:
        lo, hi = torch.aminmax(gid32)
        if int(lo) < 0 or int(hi) >= G:  # the kernel indexes LDS by gid: never launch out of range
            raise ValueError(f"group_reduce: group ids outside [0, {G})")
    if vals is None:
        vt, vp = 5, None
    else:
        vals = vals.contiguous()
        if vals.dtype not in _VTYPES:
            vals = vals.to(torch.float64 if vals.is_floating_point() else torch.int64)
        vt, vp = _VTYPES[vals.dtype], vals.data_ptr()
        if vals.shape[0] != n:
            raise ValueError("group_reduce: gid and values differ in length")
    mp = None
    if mask is not None:
        mask = mask.contiguous()
        if mask.dtype == torch.bool:
            mask = mask.view(torch.uint8)
        elif mask.dtype != torch.uint8:
            mask = mask.to(torch.uint8)
        if mask.shape[0] != n:
            raise ValueError("group_reduce: gid and mask differ in length")
        mp = mask.data_ptr()
    return _launch(gid32, vp, vt, mp, n, 1, G, op, floating)


def _launch(gid32, vp, vt, mp, n: int, d: int, G: int, op: str, floating: bool) -> torch.Tensor:
    ne = n * d
    rpb = max(_ROWS_PER_BLOCK, -(-ne // 65535))
    nb = -(-ne // rpb)
    dt = torch.float64 if floating else torch.int64
    slots = G * d
    scratch = torch.empty(nb * slots, dtype=dt, device=gid32.device)
    out = torch.empty(slots, dtype=dt, device=gid32.device)
    stream = torch.cuda.current_stream(gid32.device).cuda_stream
    _native.check(_native.kernels().cml_group_reduce(gid32.data_ptr(), vp, vt, mp, n, d, slots, _OPS[op],
                                                     0 if floating else 1, rpb, nb, scratch.data_ptr(),
                                                     out.data_ptr(), stream), "group_reduce")
    return out


def group_sum_rows(gid: torch.Tensor, x: torch.Tensor, G: int, mask: Optional[torch.Tensor] = None) -> torch.Tensor:
    """[G, d] f64 per-group column sums of a row-major [n, d] matrix (class / cluster sums of the
    evaluators and NaiveBayes): K25 over the n*d elements when G*d fits the LDS path."""
    n, d = int(x.shape[0]), int(x.shape[1])
    if not x.is_cuda or G * d > 2048 or n * d < _MIN_ROWS or G <= 0 or d == 0:
        g = gid.to(torch.int64)
        v = x.to(torch.float64)
        if mask is not None:
            v = torch.where(mask.to(torch.bool)[:, None], v, torch.zeros_like(v))
        return torch.zeros(G, d, dtype=torch.float64, device=x.device).index_add_(0, g, v)
    gid32 = (gid if gid.dtype == torch.int32 else gid.to(torch.int32)).contiguous()
    lo, hi = torch.aminmax(gid32)
    if int(lo) < 0 or int(hi) >= G:
        raise ValueError(f"group_sum_rows: group ids outside [0, {G})")
    x = x.contiguous()
    if x.dtype not in (torch.float64, torch.float32):
        x = x.to(torch.float64)
    mp = None
    if mask is not None:
        mask = (mask.view(torch.uint8) if mask.dtype == torch.bool else mask.to(torch.uint8)).contiguous()
        mp = mask.data_ptr()
    return _launch(gid32, x.data_ptr(), _VTYPES[x.dtype], mp, n, d, G, "sum", True).view(G, d)
