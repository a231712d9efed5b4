"""Device-side group-by: the per-group partial aggregates of ``group.local_partials`` computed
with dense group ids and segmented reductions on the rank's device instead of a per-row Python
loop (reference call sites: the per-hospital ``groupBy(...).agg(count, avg, max)`` of ref.py
:150-160 and the streaming window counts of ref.py:84-92).

Group ids: every key becomes a dense int64 code on the device — numeric / timestamp / date /
boolean keys through ``torch.unique`` on their (NaN- and -0.0-canonicalised) bit patterns,
string keys through the ingest dictionary codes (``ColumnData.codes``, native CSV dictionary
encoding) or one ``pandas.factorize`` pass, a tumbling or sliding ``window()`` key through its
bucket start computed on the device (sliding windows expand rows exactly as Spark's
TimeWindowing does). The codes are combined by mixed radix into one id, ranked, and ordered by
first appearance so the result is identical (order included) to the row-loop path.

Aggregates: count / sum / avg / variance / stddev (Chan partials ``(n, Σ, mean, M2)`` from two
``index_add_`` passes), min / max (``scatter_reduce`` amin/amax), first / last (first / last
row index per group), and the custom-aggregate protocol (``ml.stat.Summarizer``) with per-group
row lists. Partials keep the exact shapes ``group._partial`` produces, so the cross-rank merge,
streaming state and final projection are shared with the row-loop path, which still handles
what this path declines (distinct counts, collect_*, percentile, string min/max, ...).
"""
from __future__ import annotations

from typing import Any, List, Optional

import numpy as np
import torch

from . import types as T
from ..ops.group_ops import group_reduce
from .column import AggExpr, ColRef, ColumnData

_FAST_FNS = {"count", "sum", "avg", "min", "max", "stddev", "stddev_pop", "variance", "var_pop", "first", "last"}
_MOM_FNS = {"sum", "avg", "stddev", "stddev_pop", "variance", "var_pop"}
_MIN_ROWS = 64  # below this the row loop is as fast and keeps tiny frames off the device
ENABLED = True  # tests flip this to compare against the row-loop path


def _numeric(dt) -> bool:
    return isinstance(dt, (T.ByteType, T.ShortType, T.IntegerType, T.LongType, T.FloatType, T.DoubleType,
                           T.TimestampType, T.DateType))


def _dense(v: torch.Tensor, bound: Optional[int] = None):
    """(dense ids in [0, k), k) of non-negative int64 values; a presence bincount + prefix sum when
    the value range is small (O(n)), a sort-based unique otherwise."""
    if bound is None and v.numel():
        bound = int(v.max()) + 1
    if bound is not None and bound <= max(4 * v.numel(), 1 << 20):
        present = torch.bincount(v, minlength=bound) > 0
        remap = torch.cumsum(present, 0) - 1
        return remap[v], int(remap[-1]) + 1 if bound else 0
    uniq, inv = torch.unique(v, return_inverse=True)
    return inv, int(uniq.numel())


def _key_codes(cd: ColumnData, dev):
    """(dense int64 codes in [0, card), card) for one key column; null is its own code 0."""
    if cd.is_host:
        if not isinstance(cd.dtype, T.StringType):
            return None
        if cd.codes is not None:
            raw = np.asarray(cd.codes, dtype=np.int64)
        else:
            import pandas as pd
            raw = np.asarray(pd.factorize(cd.values, use_na_sentinel=True)[0], dtype=np.int64)
        if cd.valid is not None:
            raw = np.where(np.asarray(cd.valid, dtype=bool), raw, -1)
        code = torch.as_tensor(raw + 1, device=dev)
        return code, int(raw.max(initial=-1)) + 2
    v = cd.values
    if v.dim() != 1 or not (_numeric(cd.dtype) or isinstance(cd.dtype, T.BooleanType)):
        return None
    if v.is_floating_point():
        v = v.to(torch.float64) + 0.0  # -0.0 -> 0.0
        v = torch.where(torch.isnan(v), torch.full_like(v, float("nan")), v).view(torch.int64)
        inv, k = _dense(v, bound=1 << 62)  # bit patterns: always the sort path
    else:
        v = v.to(torch.int64)
        lo, hi = (int(v.min()), int(v.max())) if v.numel() else (0, 0)
        inv, k = _dense(v - lo, bound=hi - lo + 1) if hi - lo < (1 << 62) else _dense(v, bound=1 << 62)
    code = inv + 1
    if cd.valid is not None:
        code = torch.where(cd.valid.to(v.device), code, torch.zeros_like(code))
    return code, k + 1


def _window_expand(tw, df, dev):
    """(src row index, bucket start) per expanded entry, row-major and earliest window first."""
    cd = tw.child.eval(df)
    if not isinstance(cd.dtype, T.TimestampType) or cd.is_host:
        raise TypeError("window() needs a timestamp column")
    t = cd.values.to(torch.int64)
    last = t - torch.remainder(t - tw.start, tw.slide)
    nwin = -(-tw.dur // tw.slide)
    if nwin == 1 and cd.valid is None:
        return None, last.to(dev)  # tumbling window, no nulls: one bucket per row, no expansion
    vm = cd.valid_mask().to(t.device)
    j = torch.arange(nwin - 1, -1, -1, device=t.device, dtype=torch.int64)
    s0 = last[:, None] - j[None, :] * tw.slide                     # [n, nwin]
    ok = (s0 + tw.dur > t[:, None]) & vm[:, None]
    rows = torch.arange(t.shape[0], device=t.device)[:, None].expand(-1, nwin)
    return rows[ok].to(dev), s0[ok].to(dev)


def _python_values(cd: ColumnData) -> List[Any]:
    from .dataframe import column_to_python
    return column_to_python(cd)


class TensorPartials:
    """Per-group partial aggregates of one rank as device tensors (group g = g-th group in first-
    appearance order): ``parts[j]`` is None for a key spec, else a dict with ``kind`` and tensors
    ("n": cnt; "min"/"max": cnt, val; "first"/"last": cnt, rows; "isum": cnt, sum; "mom": cnt, sum,
    mu, m2; "custom": computed from the group row lists)."""

    def __init__(self, **kw):
        self.__dict__.update(kw)


def fast_local_partials(df, keys, exprs):
    """Same result as ``group.local_partials`` or None when this path does not apply."""
    tp = tensor_partials(df, keys, exprs)
    if tp is None:
        return None
    return tp.specs, tp.key_types, _to_python(tp, df)


def tensor_partials(df, keys, exprs) -> Optional[TensorPartials]:
    """The device stage of ``fast_local_partials``; None when this path does not apply."""
    from .group import _agg_name, _unwrap
    from .window import _WINDOW_TYPE, TimeWindow
    n = df._nrows
    if n < _MIN_ROWS:
        return None
    dev = df._device
    key_names = [k.name() for k in keys]
    tws = [k for k in keys if isinstance(k, TimeWindow)]
    if len(tws) > 1:
        return None
    src: Optional[torch.Tensor] = None  # expanded entry -> row (None = identity)
    win_start = None
    if tws:
        src, win_start = _window_expand(tws[0], df, dev)
    m = n if src is None else int(src.shape[0])
    if m == 0:
        return None
    # ---- aggregate specs (decline before any key work when unsupported)
    specs, agg_inputs = [], []
    for e in exprs:
        alias, inner = _unwrap(e)
        if not isinstance(inner, AggExpr):
            if isinstance(inner, ColRef) and inner.col in key_names:
                specs.append(("key", alias or inner.col, key_names.index(inner.col), None))
                agg_inputs.append(None)
                continue
            raise ValueError(f"expression {e} is neither an aggregate nor a grouping column")
        name = alias or _agg_name(inner)
        if getattr(inner, "custom", False):
            specs.append(("agg", name, inner, None, None))  # prepared once the keys are accepted
            agg_inputs.append(("custom", None))
            continue
        if inner.fn not in _FAST_FNS or inner.distinct:
            return None
        if inner.child is None:
            specs.append(("agg", name, inner, None, T.LongType()))
            agg_inputs.append(("star", None))
            continue
        cd = inner.child.eval(df)
        if inner.fn in ("first", "last") and not inner.ignore_nulls and cd.valid is not None:
            return None  # first/last ROW with nulls present (Spark's default): the row-loop merge
        if inner.fn in ("first", "last") and (cd.is_host or cd.values.dim() == 1):
            pass  # positions are computed on the device, values taken from the column as stored
        elif inner.fn != "count" and (cd.is_host or not _numeric(cd.dtype) or cd.values.dim() != 1):
            return None
        if inner.fn in _MOM_FNS and isinstance(cd.dtype, (T.TimestampType, T.DateType)):
            return None
        specs.append(("agg", name, inner, None, cd.dtype))
        agg_inputs.append(("col", cd))
    # ---- keys -> one dense group id per expanded entry
    key_types, key_codes = [], []
    key_cols: List[Optional[ColumnData]] = []
    for k in keys:
        if isinstance(k, TimeWindow):
            lo = int(win_start.min())
            inv, k = _dense(torch.div(win_start - lo, tws[0].slide, rounding_mode="floor"))
            key_codes.append((inv, k))
            key_types.append(_WINDOW_TYPE)
            key_cols.append(None)
            continue
        cd = k.eval(df)
        kc = _key_codes(cd, dev)
        if kc is None:
            return None
        code, card = kc
        if src is not None:
            code = code[src]
        key_codes.append((code, card))
        key_types.append(cd.dtype)
        key_cols.append(cd)
    if key_codes:
        radix = 1
        for _, card in key_codes:
            radix *= max(card, 1)
        if radix < (1 << 62):
            comb = torch.zeros(m, dtype=torch.int64, device=dev)
            for code, card in key_codes:
                comb = comb * card + code
            inv, _ = _dense(comb, bound=radix)
        else:
            _, inv = torch.unique(torch.stack([c for c, _ in key_codes], 1), dim=0, return_inverse=True)
        G = int(inv.max()) + 1
        first = group_reduce(inv, None, G, "min", floating=False)  # first entry of every group
        order = torch.argsort(first)
        rank = torch.empty_like(order)
        rank[order] = torch.arange(G, device=dev)
        gid = rank[inv]
        first = first[order]
    else:
        G = 1
        gid = torch.zeros(m, dtype=torch.int64, device=dev)
        first = torch.zeros(1, dtype=torch.int64, device=dev)
    specs = [("agg", sp[1], sp[2], sp[2].prepare(df), None) if inp is not None and inp[0] == "custom" else sp
             for sp, inp in zip(specs, agg_inputs)]
    first_rows = first if src is None else src[first]
    # ---- per-group partials (tensors)
    parts: List[Optional[dict]] = []
    all_count = None
    for sp, inp in zip(specs, agg_inputs):
        if sp[0] == "key":
            parts.append(None)
            continue
        agg = sp[2]
        kind = inp[0]
        if kind == "custom":
            parts.append({"kind": "custom"})
            continue
        if kind == "star":
            if all_count is None:
                all_count = torch.bincount(gid, minlength=G)
            parts.append({"kind": "n", "cnt": all_count})
            continue
        cd = inp[1]
        fn = agg.fn
        # validity as a mask (None = every entry counts); no boolean-mask gathers below — the
        # reductions run over all entries with neutral values where the mask is off
        vm = None
        if cd.valid is not None:
            vm = torch.as_tensor(np.asarray(cd.valid, dtype=bool)) if cd.is_host else cd.valid
            vm = vm.to(dev)
            vm = vm if src is None else vm[src]
        vals = None
        if not cd.is_host and fn != "count":
            vals = cd.values if src is None else cd.values[src]
            if vals.is_floating_point():
                nn = ~torch.isnan(vals)
                vm = nn if vm is None else vm & nn
        # per-group reductions: K25 group_reduce (LDS-privatised, few groups) on the GPU, torch
        # scatter otherwise; masked-off entries (nulls, NaN) are skipped
        if vm is None:
            if all_count is None:
                all_count = torch.bincount(gid, minlength=G)
            cnt = all_count
        else:
            cnt = group_reduce(gid, vm.to(torch.uint8), G, "sum", floating=False)
        if fn == "count":
            parts.append({"kind": "n", "cnt": cnt})
            continue
        if fn in ("min", "max"):
            out = group_reduce(gid, vals, G, fn, mask=vm)
            if out.dtype != vals.dtype:
                if not vals.is_floating_point():
                    info = torch.iinfo(vals.dtype)
                    out = out.clamp(info.min, info.max)
                out = out.to(vals.dtype)
            parts.append({"kind": fn, "cnt": cnt, "val": out, "cd": cd})
            continue
        if fn in ("first", "last"):
            pick = group_reduce(gid, None, G, "min" if fn == "first" else "max", mask=vm, floating=False)
            pick = pick.clamp(0, m - 1)
            parts.append({"kind": fn, "cnt": cnt, "rows": pick if src is None else src[pick], "cd": cd})
            continue
        # sum / avg / variance family
        if fn == "sum" and T.is_integral(cd.dtype):
            parts.append({"kind": "isum", "cnt": cnt, "sum": group_reduce(gid, vals, G, "sum", mask=vm,
                                                                          floating=False)})
            continue
        s = group_reduce(gid, vals, G, "sum", mask=vm, floating=True)
        mu = s / cnt.clamp(min=1).to(torch.float64)
        d = vals.to(torch.float64) - mu[gid]
        m2 = group_reduce(gid, d * d, G, "sum", mask=vm, floating=True)
        parts.append({"kind": "mom", "cnt": cnt, "sum": s, "mu": mu, "m2": m2})
    return TensorPartials(specs=specs, key_types=key_types, keys=keys, key_cols=key_cols, G=G, gid=gid,
                          first=first, first_rows=first_rows, src=src, win_start=win_start, n=n, m=m, parts=parts)


def _to_python(tp: TensorPartials, df):
    """{key tuple: [partial per spec]} in the shapes ``group._partial`` produces."""
    G, dev = tp.G, df._device
    # ---- key tuples (python values of each group's first entry, as the row loop sees them)
    key_lists = []
    for k, cd in zip(tp.keys, tp.key_cols):
        if cd is None:
            from .column import micros_to_datetime
            from .types import Row
            s0 = tp.win_start[tp.first].cpu().tolist()
            key_lists.append([Row(start=micros_to_datetime(s), end=micros_to_datetime(s + k.dur)) for s in s0])
        else:
            key_lists.append(_python_values(cd.take(tp.first_rows)))
    group_keys = [tuple(kl[g] for kl in key_lists) for g in range(G)]
    per_spec: List[Optional[List[Any]]] = []
    rows_of_group = None
    for sp, pt in zip(tp.specs, tp.parts):
        if pt is None:
            per_spec.append(None)
            continue
        kind = pt["kind"]
        if kind == "custom":
            if rows_of_group is None:
                srows = (torch.arange(tp.n, device=dev) if tp.src is None else tp.src)
                perm = torch.argsort(tp.gid, stable=True)
                counts = torch.bincount(tp.gid, minlength=G).cpu().tolist()
                flat = srows[perm].cpu().tolist()
                rows_of_group, at = [], 0
                for c in counts:
                    rows_of_group.append(flat[at:at + c])
                    at += c
            per_spec.append([sp[2].partial(sp[3], rows_of_group[g]) for g in range(G)])
            continue
        cnt_l = pt["cnt"].cpu().tolist()
        if kind == "n":
            per_spec.append([("n", c) for c in cnt_l])
        elif kind in ("min", "max"):
            py = _python_values(ColumnData(pt["val"], None, pt["cd"].dtype))
            per_spec.append([(kind, py[g] if cnt_l[g] else None) for g in range(G)])
        elif kind in ("first", "last"):
            py = _python_values(pt["cd"].take(pt["rows"]))
            per_spec.append([(kind, py[g] if cnt_l[g] else None, bool(cnt_l[g])) for g in range(G)])
        elif kind == "isum":
            per_spec.append([("isum", c, int(x)) if c else ("mom", 0, 0.0, 0.0, 0.0)
                             for c, x in zip(cnt_l, pt["sum"].cpu().tolist())])
        else:
            st = torch.stack([pt["sum"], pt["mu"], pt["m2"]]).cpu().tolist()
            per_spec.append([("mom", c, st[0][g], st[1][g], st[2][g]) if c else ("mom", 0, 0.0, 0.0, 0.0)
                             for g, c in enumerate(cnt_l)])
    local = {}
    for g, key in enumerate(group_keys):
        local[key] = [None if ps is None else ps[g] for ps in per_spec]
    return local
