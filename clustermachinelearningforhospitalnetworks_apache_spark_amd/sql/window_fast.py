"""Window functions on the device: ranking, offsets and frame aggregates over ``Window.partitionBy(..)
.orderBy(..)`` without a per-row Python loop (the call sites: per-hospital running counts and lags
over event time, ref.py:81 / ref.py:123-128 style analytics).

Plan: every partition / ordering key becomes an int64 code on the device (order-preserving ranks for
ordering keys, with Spark's null placement and NaN as the largest value); the codes are combined by
mixed radix with the partition id most significant, and ONE stable sort gives the window order.
Segment (partition) and peer (equal ordering key) boundaries are flags on the sorted key; running
maxima of their positions give each row its segment start / peer start, reversed running minima its
segment end / peer end. From those:

* row_number, rank, dense_rank, percent_rank, cume_dist, ntile are index arithmetic;
* lag / lead gather the shifted row when it stays in the segment;
* count / sum / avg over ROWS or RANGE frames (unbounded / current row / row offsets) are
  differences of segment prefix sums (int64 for integral sums, so exact), first / last gather the
  frame ends, min / max over whole partitions are segment reductions.

Distributed frames all-gather the needed device columns in rank order (the same global order as the
host path), evaluate on every rank and keep the rank's slice; string keys are factorised in value
order over the gathered values. Anything else (RANGE with value offsets, running min/max, stddev over
frames, ...) returns None and the caller uses the host implementation in window.py.
"""
from __future__ import annotations

from typing import List, Optional, Tuple

import numpy as np
import torch

from . import types as T
from .column import AggExpr, ColumnData, Expr

def _dense_codes(vals: torch.Tensor) -> Tuple[torch.Tensor, int]:
    """Order-preserving dense ranks (bincount + prefix sum for small integer ranges, else unique)."""
    if vals.is_floating_point():
        uniq, inv = torch.unique(vals, sorted=True, return_inverse=True)
        return inv.to(torch.int64), int(uniq.numel())
    from .relational_fast import _rerank
    return _rerank(vals.to(torch.int64))


def _gather(comm, t: torch.Tensor) -> torch.Tensor:
    return comm.allgather_cat(t.contiguous()) if comm.is_distributed else t


def _column(frame, e: Expr, comm):
    """(values, valid) device tensors of a key / argument, gathered over ranks; None if unsupported."""
    cd = e.eval(frame)
    if cd.is_host:
        if not isinstance(cd.dtype, T.StringType):
            return None
        import pandas as pd
        from .dataframe import column_to_python
        loc = column_to_python(cd)
        allv = [x for p in comm.allgather_object(loc) for x in p] if comm.is_distributed else loc
        codes, _ = pd.factorize(np.asarray(allv, dtype=object), sort=True)  # value-ordered codes, -1 = null
        v = torch.as_tensor(np.asarray(codes, dtype=np.int64), device=frame._device)
        return v, v >= 0, cd.dtype
    v = cd.values
    if v.dim() != 1:
        return None
    ok = cd.valid_mask().to(v.device)
    return _gather(comm, v), _gather(comm, ok), cd.dtype


def _order_code(v: torch.Tensor, ok: torch.Tensor, ascending: bool, nulls_first: bool) -> Tuple[torch.Tensor, int]:
    """Order-preserving int64 code in [0, C) with nulls first / last and NaN above every number."""
    if v.is_floating_point():
        x = v.to(torch.float64)
        nan = torch.isnan(x)
        x = torch.where(nan | ~ok, torch.zeros_like(x), x) + 0.0
        r, u = _dense_codes(x)
        r = torch.where(nan, torch.full_like(r, u), r)
        u = u + 1
    else:
        x = torch.where(ok, v.to(torch.int64), torch.zeros_like(v, dtype=torch.int64))
        r, u = _dense_codes(x)
    if not ascending:
        r = (u - 1) - r
    if nulls_first:
        return torch.where(ok, r + 1, torch.zeros_like(r)), u + 1
    return torch.where(ok, r, torch.full_like(r, u)), u + 1


def _next_start(flag: torch.Tensor) -> torch.Tensor:
    """For each i the smallest j > i with flag[j] (N when none)."""
    n = flag.numel()
    idx = torch.where(flag, torch.arange(n, device=flag.device), torch.full((n,), n, device=flag.device,
                                                                           dtype=torch.int64))
    shifted = torch.cat([idx[1:], torch.tensor([n], device=flag.device, dtype=torch.int64)])
    return torch.flip(torch.cummin(torch.flip(shifted, [0]), 0).values, [0])


def device_window(frame, func, spec) -> Optional[ColumnData]:
    from .window import WindowFunc, _UNB_FOLL, _UNB_PREC, _result_type
    comm = frame._comm
    dev = frame._device
    fn = func.fn
    rank_fns = ("row_number", "rank", "dense_rank", "percent_rank", "cume_dist", "ntile", "lag", "lead")
    agg_fns = ("count", "sum", "avg", "min", "max", "first", "last")
    if isinstance(func, WindowFunc):
        if fn not in rank_fns:
            return None
    elif isinstance(func, AggExpr):
        if fn not in agg_fns or getattr(func, "custom", False) or func.distinct:
            return None
        if getattr(func, "ignore_nulls", False):
            return None  # first / last ignoreNulls over a frame: host path
    else:
        return None
    frame_spec = spec._frame
    if frame_spec is not None and frame_spec[0] == "range":
        s, e = frame_spec[1], frame_spec[2]
        if s not in (_UNB_PREC, 0) or e not in (_UNB_FOLL, 0):
            return None  # RANGE with value offsets: host path
    n_local = frame._nrows
    counts = comm.allgather_object(n_local) if comm.is_distributed else [n_local]
    off = sum(counts[:comm.rank]) if comm.is_distributed else 0
    N = sum(counts)
    if N == 0:
        return None
    # ---- keys
    comp = torch.zeros(N, dtype=torch.int64, device=dev)
    radix = 1
    pid = torch.zeros(N, dtype=torch.int64, device=dev)
    for e in spec._partition:
        col = _column(frame, e, comm)
        if col is None:
            return None
        v, ok, _ = col
        if v.is_floating_point():
            x = torch.where(torch.isnan(v), torch.full_like(v, float("nan")), v).to(torch.float64) + 0.0
            x = x.view(torch.int64)
        else:
            x = v.to(torch.int64)
        code, card = _dense_codes(torch.where(ok, x, torch.zeros_like(x)))
        code = torch.where(ok, code + 1, torch.zeros_like(code))
        card += 1
        if radix * card >= (1 << 62):
            return None
        pid = pid * card + code
        radix *= card
    pid, pcard = _dense_codes(pid)
    comp = pid.clone()
    radix = pcard
    for o in spec._orders:
        col = _column(frame, o.expr, comm)
        if col is None:
            return None
        v, ok, _ = col
        code, card = _order_code(v, ok, o.ascending, o.nulls_first)
        if radix * card >= (1 << 62):
            return None
        comp = comp * card + code
        radix *= card
    # ---- window order and boundaries
    perm = torch.sort(comp, stable=True).indices
    cs = comp[perm]
    ps = pid[perm]
    ar = torch.arange(N, device=dev, dtype=torch.int64)
    seg_flag = torch.ones(N, dtype=torch.bool, device=dev)
    seg_flag[1:] = ps[1:] != ps[:-1]
    peer_flag = torch.ones(N, dtype=torch.bool, device=dev)
    peer_flag[1:] = cs[1:] != cs[:-1]
    seg_start = torch.cummax(torch.where(seg_flag, ar, torch.zeros_like(ar)), 0).values
    peer_start = torch.cummax(torch.where(peer_flag, ar, torch.zeros_like(ar)), 0).values
    seg_end = _next_start(seg_flag) - 1
    peer_end = _next_start(peer_flag) - 1
    m = seg_end - seg_start + 1
    # ---- argument
    child = func.child
    vals = valid = None
    in_type = None
    host_vals = None
    if child is not None:
        cd = child.eval(frame)
        in_type = cd.dtype
        if cd.is_host or cd.values.dim() != 1:
            if fn not in ("lag", "lead", "first", "last", "count"):
                return None
            from .dataframe import column_to_python
            loc = column_to_python(cd)
            allv = [x for p in comm.allgather_object(loc) for x in p] if comm.is_distributed else loc
            host_vals = np.empty(N, dtype=object)
            host_vals[:] = allv
            valid = torch.as_tensor(np.asarray([x is not None for x in allv], dtype=bool), device=dev)
        else:
            vals = _gather(comm, cd.values)
            valid = _gather(comm, cd.valid_mask().to(cd.values.device))
    res_valid = None
    out_type = _result_type(func, in_type)
    # ---- functions
    if fn == "row_number":
        res = ar - seg_start + 1
    elif fn == "rank":
        res = peer_start - seg_start + 1
    elif fn == "dense_rank":
        c = torch.cumsum(peer_flag.to(torch.int64), 0)
        res = c - c[seg_start] + 1
    elif fn == "percent_rank":
        rk = (peer_start - seg_start).to(torch.float64)
        res = torch.where(m > 1, rk / (m - 1).clamp(min=1).to(torch.float64), torch.zeros_like(rk))
    elif fn == "cume_dist":
        res = (peer_end - seg_start + 1).to(torch.float64) / m.to(torch.float64)
    elif fn == "ntile":
        k = int(func.arg)
        p = ar - seg_start
        base = torch.div(m, k, rounding_mode="floor")
        extra = m - base * k
        big = (base + 1) * extra
        res = torch.where(p < big, torch.div(p, base + 1, rounding_mode="floor"),
                          extra + torch.div(p - big, base.clamp(min=1), rounding_mode="floor")) + 1
    elif fn in ("lag", "lead"):
        shift = int(func.arg) * (-1 if fn == "lag" else 1)
        j = ar + shift
        inseg = (j >= seg_start) & (j <= seg_end)
        jc = j.clamp(0, N - 1)
        src = perm[jc]
        if host_vals is not None:
            hv = host_vals[src.cpu().numpy()]
            ins = inseg.cpu().numpy()
            outv = [v if i else func.default for v, i in zip(hv, ins)]
            return _scatter_host(outv, perm, off, n_local, out_type, frame)
        sv = vals[src]
        res_valid = torch.where(inseg, valid[src], torch.full_like(inseg, func.default is not None))
        if func.default is not None:
            res = torch.where(inseg, sv, torch.full_like(sv, func.default))
        else:
            res = sv
        out_type = in_type
    else:
        # frame aggregates: [lo, hi] positions in the sorted order
        if frame_spec is None:
            if spec._orders:
                lo, hi = seg_start, peer_end
            else:
                lo, hi = seg_start, seg_end
        elif frame_spec[0] == "rows":
            s, e = frame_spec[1], frame_spec[2]
            lo = seg_start if s <= _UNB_PREC else torch.maximum(seg_start, ar + s)
            hi = seg_end if e >= _UNB_FOLL else torch.minimum(seg_end, ar + e)
        else:
            s, e = frame_spec[1], frame_spec[2]
            lo = seg_start if s == _UNB_PREC else peer_start
            hi = seg_end if e == _UNB_FOLL else peer_end
        nonempty = hi >= lo
        vs = None if vals is None else vals[perm]
        ok = (valid[perm] if valid is not None else torch.ones(N, dtype=torch.bool, device=dev))
        if fn == "count" and child is None:
            ok = torch.ones(N, dtype=torch.bool, device=dev)
        cnt = torch.cat([torch.zeros(1, dtype=torch.int64, device=dev), torch.cumsum(ok.to(torch.int64), 0)])
        lo_c, hi_c = lo.clamp(0, N - 1), hi.clamp(-1, N - 1)
        fcount = torch.where(nonempty, cnt[hi_c + 1] - cnt[lo_c], torch.zeros_like(lo))
        if fn == "count":
            res = fcount
            out_type = T.LongType()
        elif fn in ("sum", "avg"):
            if vs is None:
                return None
            integral = not vs.is_floating_point() and vs.dtype != torch.bool
            x = torch.where(ok, vs.to(torch.int64 if (integral and fn == "sum") else torch.float64),
                            torch.zeros((), dtype=torch.int64 if (integral and fn == "sum") else torch.float64,
                                        device=dev))
            if vs.is_floating_point():
                x = torch.where(torch.isnan(vs) & ok, vs.to(torch.float64), x)
            pre = torch.cat([torch.zeros(1, dtype=x.dtype, device=dev), torch.cumsum(x, 0)])
            tot = torch.where(nonempty, pre[hi_c + 1] - pre[lo_c], torch.zeros_like(pre[lo_c]))
            res = tot if fn == "sum" else tot.to(torch.float64) / fcount.clamp(min=1).to(torch.float64)
            res_valid = fcount > 0
        elif fn in ("first", "last"):
            pos = lo_c if fn == "first" else hi_c.clamp(min=0)
            src = perm[pos]
            if host_vals is not None:
                hv = host_vals[src.cpu().numpy()]
                ne = nonempty.cpu().numpy()
                return _scatter_host([v if e_ else None for v, e_ in zip(hv, ne)], perm, off, n_local, out_type, frame)
            res = vals[src]
            res_valid = nonempty & valid[src]
            out_type = in_type
        elif fn in ("min", "max"):
            whole = (frame_spec is None and not spec._orders) or (
                frame_spec is not None and frame_spec[1] <= _UNB_PREC and frame_spec[2] >= _UNB_FOLL)
            if not whole or vs is None:
                return None
            sid = torch.cumsum(seg_flag.to(torch.int64), 0) - 1
            nseg = int(sid[-1]) + 1
            x = vs.to(torch.float64) if vs.is_floating_point() else vs.to(torch.int64)
            if x.is_floating_point():
                okx = ok & ~torch.isnan(x)
                fill = float("inf") if fn == "min" else float("-inf")
            else:
                okx = ok
                fill = torch.iinfo(torch.int64).max if fn == "min" else torch.iinfo(torch.int64).min
            from ..ops.group_ops import group_reduce
            red = group_reduce(sid, x, nseg, fn, mask=okx)  # K25 on the GPU for few partitions
            has = group_reduce(sid, okx.to(torch.uint8), nseg, "sum", floating=False) > 0
            res = red[sid].to(vs.dtype)
            res_valid = has[sid]
            out_type = in_type
        else:
            return None
    # ---- back to row order, this rank's slice
    full = torch.empty_like(res)
    full[perm] = res
    loc = full[off:off + n_local]
    lv = None
    if res_valid is not None:
        fv = torch.empty_like(res_valid)
        fv[perm] = res_valid
        lv = fv[off:off + n_local]
        if bool(lv.all()):
            lv = None
    if out_type is not None and out_type.torch_dtype is not None and loc.dtype != out_type.torch_dtype:
        loc = loc.to(out_type.torch_dtype)
    return ColumnData(loc.contiguous(), lv, out_type)


def _scatter_host(outv: List, perm: torch.Tensor, off: int, n_local: int, dtype, frame) -> ColumnData:
    from .builder import column_from_values
    p = perm.cpu().numpy()
    full = np.empty(len(outv), dtype=object)
    full[p] = np.asarray(outv, dtype=object) if outv else np.empty(0, dtype=object)
    return column_from_values(list(full[off:off + n_local]), dtype, frame._device)


__all__ = ["device_window"]
