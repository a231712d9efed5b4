"""Device relational operators: ``orderBy`` / ``sort``, ``dropDuplicates`` / ``distinct``,
``repartition`` and equi-joins (``DataFrame.join`` and SQL ``JOIN ... ON / USING``) without
gathering every row into Python lists.

The reference runs these as Spark SQL shuffles (sort of per-hospital results before ``show``,
ref.py:150-160; ``dropna``/``distinct`` cleaning, ref.py:57; the hospital-record joins of the
streaming job). Here:

* **sort** — every ordering key becomes an order-preserving int64 code (Spark's null placement,
  NaN above every number, strings in code-point order); keys are folded most-significant-first
  and re-ranked after each fold, so the composite never overflows. ONE stable sort gives the
  global permutation. On one rank the frame is gathered by it; across ranks only the keys are
  all-gathered, every rank derives the same permutation, and the payload moves once through a
  variable all-to-all (``Communicator.alltoallv``) into contiguous, balanced output slices — the
  placement the row-loop path produces, ids included.
* **dropDuplicates** — equality codes per key column (NaN == NaN, -0.0 == 0.0, null == null, as
  Spark's grouping), first occurrence per code via ``scatter_reduce(amin)``; duplicates are
  first dropped rank-locally, then only the surviving keys are all-gathered to resolve
  cross-rank duplicates in global order. Rows stay on their rank.
* **join** — left and right keys are coded jointly (one ``torch.unique`` over both sides; null
  keys never match), the right side is sorted by code and per-code counts / prefix sums give
  every left row's match range; ``repeat_interleave`` expands the pairs in (left row, right row) order.
  inner / left / right / full / semi / anti / cross are index arithmetic on those ranges; the
  right side is broadcast to every rank (the reference's tables are small dimensions), the
  unmatched right rows of right / full joins are emitted once, by rank 0.

Each entry point returns None when a key has no device code (vectors, arrays, maps, decimals)
and the caller runs its row-loop implementation.
"""
from __future__ import annotations

from typing import Dict, List, Optional, Sequence, Tuple

import numpy as np
import torch

from . import types as T
from .column import ColumnData, DictColumnData

ENABLED = True  # tests flip this to compare against the row-loop paths


# ------------------------------------------------------------------------------------------------ codes
def _rerank(v: torch.Tensor) -> Tuple[torch.Tensor, int]:
    """Order-preserving dense ranks of int64 values: a presence bincount + prefix sum when the value
    range is small (O(n + range), no sort), a sort-based unique otherwise."""
    n = v.numel()
    if n == 0:
        return v.to(torch.int64), 0
    lo, hi = int(v.min()), int(v.max())
    if hi - lo < max(4 * n, 1 << 20):
        x = v - lo
        present = torch.bincount(x, minlength=hi - lo + 1) > 0
        remap = torch.cumsum(present, 0) - 1
        return remap[x], int(remap[-1]) + 1
    uniq, inv = torch.unique(v, sorted=True, return_inverse=True)
    return inv.to(torch.int64), int(uniq.numel())


_I64_MASK = 0x7FFFFFFFFFFFFFFF


def _order_key(v: torch.Tensor, ok: Optional[torch.Tensor], ascending: bool, nulls_first: bool):
    """Order-preserving int64 sort keys of one column: a list of (key, range) to sort by, most
    significant first; ``range`` (keys in [0, range)) is None for full-width keys. Floats map to
    their total-order bit pattern (NaN canonical and largest, -0.0 == 0.0), descending is the bitwise
    complement, nulls go below / above every value."""
    if v.is_floating_point():
        x = v.to(torch.float64) + 0.0
        x = torch.where(torch.isnan(x), torch.full_like(x, float("nan")), x)
        b = x.view(torch.int64)
        k = b ^ ((b >> 63) & _I64_MASK)
    else:
        k = v.to(torch.int64)
    if not ascending:
        k = ~k
    has_null = ok is not None and not bool(ok.all())
    valid = k[ok] if has_null else k
    if valid.numel() == 0:
        return [(torch.zeros_like(k), 1)]
    lo, hi = int(valid.min()), int(valid.max())
    span = hi - lo + 1 + (1 if has_null else 0)
    if span < (1 << 62):
        key = k - lo + (1 if has_null and nulls_first else 0)
        if has_null:
            key = torch.where(ok, key, torch.full_like(key, 0 if nulls_first else hi - lo + 1))
        return [(key, span)]
    if not has_null:
        return [(k, None)]
    flag = (ok if nulls_first else ~ok).to(torch.int64)  # 0 sorts first
    return [(flag, 2), (torch.where(ok, k, torch.zeros_like(k)), None)]


def _lex_perm(keys: List[Tuple[torch.Tensor, Optional[int]]], n: int, dev) -> torch.Tensor:
    """Stable lexicographic permutation: bounded keys are packed by mixed radix into as few int64
    words as fit, then one stable sort per word, least significant word first."""
    words, cur, radix = [], None, 1
    for key, rng in keys:
        if rng is None:
            if cur is not None:
                words.append(cur)
            words.append(key)
            cur, radix = None, 1
            continue
        if cur is not None and radix * rng < (1 << 62):
            cur, radix = cur * rng + key, radix * rng
        else:
            if cur is not None:
                words.append(cur)
            cur, radix = key, rng
    if cur is not None:
        words.append(cur)
    perm = None
    for w in reversed(words):
        if perm is None:
            perm = torch.sort(w, stable=True).indices
        else:
            perm = perm[torch.sort(w[perm], stable=True).indices]
    return perm if perm is not None else torch.arange(n, device=dev)


def _fold(parts: List[Tuple[torch.Tensor, int]]) -> torch.Tensor:
    """Lexicographic (most significant first) combination of dense codes into one dense code."""
    comp, card = parts[0]
    for code, c in parts[1:]:
        comp, card = _rerank(comp * c + code)
    return comp


def _host_values(cd: ColumnData) -> np.ndarray:
    vals = np.asarray(cd.values, dtype=object)
    if cd.valid is not None:
        vals = np.where(np.asarray(cd.valid, dtype=bool), vals, None)
    return vals


def _str_parts(cd: ColumnData) -> Tuple[np.ndarray, np.ndarray]:
    """(int64 codes with -1 = null, distinct strings) of a host string column: the ingest
    dictionary when the column has one, one ``pandas.factorize`` otherwise."""
    if isinstance(cd, DictColumnData):
        codes = cd.codes.astype(np.int64)
        if cd.valid is not None:
            codes = np.where(np.asarray(cd.valid, dtype=bool), codes, -1)
        return codes, np.asarray(cd.dictionary[:-1], dtype=object)
    import pandas as pd
    codes, uniq = pd.factorize(_host_values(cd), use_na_sentinel=True)
    return codes.astype(np.int64), np.asarray(uniq, dtype=object)


def _merge_str(blocks: List[ColumnData]) -> Tuple[np.ndarray, np.ndarray]:
    """Codes of several string blocks against one merged dictionary: only the (small)
    dictionaries are factorised together, the per-row codes are remapped by a gather."""
    import pandas as pd
    parts = [_str_parts(c) for c in blocks]
    if len(parts) == 1:
        return parts[0]
    alld = np.concatenate([d for _, d in parts]) if parts else np.zeros(0, dtype=object)
    gmap, guniq = pd.factorize(alld)
    out, off = [], 0
    for codes, d in parts:
        m = gmap[off:off + len(d)]
        out.append(np.where(codes >= 0, m[np.clip(codes, 0, None)] if len(d) else -1, -1))
        off += len(d)
    return (np.concatenate(out) if out else np.zeros(0, dtype=np.int64)), np.asarray(guniq, dtype=object)


def _dict_column(codes: np.ndarray, uniq: np.ndarray, dtype) -> ColumnData:
    dictionary = np.empty(len(uniq) + 1, dtype=object)
    dictionary[:-1] = uniq
    dictionary[-1] = None
    ok = codes >= 0
    return DictColumnData(codes.astype(np.int32), dictionary, None if ok.all() else ok, dtype)


def _numeric_like(dt) -> bool:
    return isinstance(dt, (T.ByteType, T.ShortType, T.IntegerType, T.LongType, T.FloatType, T.DoubleType,
                           T.TimestampType, T.DateType, T.BooleanType))


def _eq_bits(v: torch.Tensor, as_float: bool) -> torch.Tensor:
    """int64 equality key of a numeric column: canonical NaN, -0.0 folded into 0.0."""
    if as_float or v.is_floating_point():
        x = v.to(torch.float64) + 0.0
        x = torch.where(torch.isnan(x), torch.full_like(x, float("nan")), x)
        return x.view(torch.int64)
    return v.to(torch.int64)


def _key_kind(cd: ColumnData) -> Optional[str]:
    if cd.is_host:
        return "str" if isinstance(cd.dtype, T.StringType) else None
    if cd.values.dim() != 1 or not _numeric_like(cd.dtype):
        return None
    return "num"


def _eq_codes(cols: List[ColumnData], dev) -> Optional[Tuple[torch.Tensor, int]]:
    """Joint equality codes of one key over several row blocks (same key, different frames or
    ranks): (codes over the concatenation, -1 = null; cardinality)."""
    kinds = {_key_kind(c) for c in cols}
    if len(kinds) != 1 or None in kinds:
        return None
    if kinds == {"str"}:
        codes, uniq = _merge_str(cols)
        return torch.as_tensor(codes, device=dev), len(uniq)
    as_float = any(c.values.is_floating_point() for c in cols)
    bits = torch.cat([_eq_bits(c.values.to(dev), as_float) for c in cols])
    ok = torch.cat([c.valid_mask().to(dev) for c in cols])
    code, card = _rerank(torch.where(ok, bits, torch.zeros_like(bits)))
    return torch.where(ok, code, torch.full_like(code, -1)), card


def _tuple_codes(keycols: List[List[ColumnData]], dev, null_equal: bool) -> Optional[torch.Tensor]:
    """Dense code of the key tuple per row over the concatenated blocks. ``null_equal``: a null is
    an ordinary key value (grouping / dedup); otherwise any null key gives -1 (join)."""
    parts, anynull = [], None
    for blocks in keycols:
        r = _eq_codes(blocks, dev)
        if r is None:
            return None
        code, card = r
        isnull = code < 0
        anynull = isnull if anynull is None else anynull | isnull
        parts.append((code + 1, card + 1))
    comp = _fold(parts)
    if not null_equal:
        comp = torch.where(anynull, torch.full_like(comp, -1), comp)
    return comp


def _order_codes(cd: ColumnData, comm, dev, ascending: bool, nulls_first: bool):
    """Sort keys (``_order_key``) of a column over all ranks in rank order, or None."""
    if cd.is_host:
        if not isinstance(cd.dtype, T.StringType):
            return None
        codes, uniq = _merge_str(_blocks(cd, comm, dev))
        rank = np.empty(len(uniq), dtype=np.int64)
        rank[np.argsort(uniq, kind="stable")] = np.arange(len(uniq))  # code-point (= UTF-8 byte) order
        v = torch.as_tensor(np.where(codes >= 0, rank[np.clip(codes, 0, None)] if len(uniq) else 0, -1),
                            device=dev)
        ok = v >= 0
    else:
        if cd.values.dim() != 1 or not _numeric_like(cd.dtype):
            return None
        v = _gather(comm, cd.values.to(dev))
        ok = _gather(comm, cd.valid_mask().to(dev)) if (cd.valid is not None or comm.is_distributed) else None
    return _order_key(v, ok, ascending, nulls_first)


def _gather(comm, t: torch.Tensor) -> torch.Tensor:
    return comm.allgather_cat(t.contiguous()) if comm.is_distributed else t


def _counts(comm, n: int) -> List[int]:
    return comm.allgather_object(n) if comm.is_distributed else [n]


# ------------------------------------------------------------------------------------------------ row movement
def _exchange(df, perm: torch.Tensor, counts: List[int]):
    """Frame whose rank-r slice is rows ``perm[shard_range(N, r, W)]`` of the global (rank-order)
    row sequence: one alltoallv per device column, an object exchange for host columns."""
    from .builder import shard_range
    comm = df._comm
    W, me = comm.world_size, comm.rank
    dev = df._device
    if not comm.is_distributed:
        return df._take_rows(perm)
    N = int(perm.numel())
    offs = torch.tensor(np.cumsum([0] + counts), dtype=torch.int64, device=dev)
    starts = [shard_range(N, r, W)[0] for r in range(W)] + [N]
    src_rank = torch.bucketize(perm, offs[1:], right=True)           # owner of every sorted position
    mine = src_rank == me
    send_pos = torch.nonzero(mine).flatten()                          # ascending destination position
    send_idx = perm[send_pos] - offs[me]
    bounds = torch.tensor(starts, dtype=torch.int64, device=dev)
    dest = torch.bucketize(send_pos, bounds[1:], right=True)
    send_counts = torch.bincount(dest, minlength=W).tolist()
    a, b = starts[me], starts[me + 1]
    # receive layout: grouped by source rank, ascending position inside each group
    order = torch.sort(src_rank[a:b], stable=True).indices
    inv = torch.empty_like(order)
    inv[order] = torch.arange(order.numel(), device=dev)
    return _move(df, send_idx, send_counts, inv)


def shuffle_to(df, dest: torch.Tensor):
    """Send every local row to rank ``dest[i]``; a rank's result holds what it received in source-rank
    order, each source's rows in their original order (the exchange of applyInPandas)."""
    comm = df._comm
    if not comm.is_distributed:
        return df
    dest = dest.to(df._device)
    send_idx = torch.sort(dest, stable=True).indices
    send_counts = torch.bincount(dest, minlength=comm.world_size).tolist()
    return _move(df, send_idx, send_counts, None)


def _move(df, send_idx: torch.Tensor, send_counts: List[int], inv: Optional[torch.Tensor]):
    """Row exchange: local rows ``send_idx`` (grouped by destination, ``send_counts`` per rank) go out,
    the received rows (source-rank order) are permuted by ``inv`` when given."""
    comm = df._comm
    W, me = comm.world_size, comm.rank
    dev = df._device
    inv_np = None if inv is None else inv.cpu().numpy()

    def perm_np(a):
        return a if inv_np is None else a[inv_np]

    def perm_t(t):
        return t if inv is None else t[inv]
    cols = {}
    for name, cd in df._cols.items():
        if cd.is_host and isinstance(cd.dtype, T.StringType):
            codes, uniq = _str_parts(cd)
            codes = codes[send_idx.cpu().numpy()]
            cut = np.cumsum([0] + send_counts)
            parts = comm.allgather_object(([codes[cut[r]:cut[r + 1]] for r in range(W)], uniq))
            blocks = [_dict_column(p[0][me], p[1], cd.dtype) for p in parts]
            rc, ru = _merge_str(blocks)
            cols[name] = _dict_column(perm_np(rc), ru, cd.dtype)
        elif cd.is_host:
            vals = _host_values(cd)[send_idx.cpu().numpy()]
            cut = np.cumsum([0] + send_counts)
            parts = comm.allgather_object([vals[cut[r]:cut[r + 1]] for r in range(W)])
            recv = np.concatenate([p[me] for p in parts]) if parts else np.zeros(0, dtype=object)
            out = perm_np(recv)
            ok = np.asarray([x is not None for x in out], dtype=bool)
            cols[name] = ColumnData(out, None if ok.all() else ok, cd.dtype)
        else:
            v = perm_t(comm.alltoallv(cd.values[send_idx], send_counts))
            ok = perm_t(comm.alltoallv(cd.valid_mask().to(dev)[send_idx], send_counts))
            cols[name] = ColumnData(v, None if cd.valid is None and bool(ok.all()) else ok, cd.dtype)
    ids = perm_t(comm.alltoallv(df._row_ids.to(dev)[send_idx], send_counts))
    return df._new(df._schema, cols, int(ids.numel()), ids)


def device_rebalance(df):
    if not ENABLED:
        return None
    counts = _counts(df._comm, df._nrows)
    return _exchange(df, torch.arange(sum(counts), device=df._device), counts)


# ------------------------------------------------------------------------------------------------ sort
def device_sort(df, orders) -> Optional[object]:
    """``orderBy`` / ``sort`` on device codes; None when an ordering key has no code."""
    if not ENABLED or not orders:
        return None
    comm, dev = df._comm, df._device
    counts = _counts(comm, df._nrows)
    N = sum(counts)
    if N == 0:
        return df
    keys = []
    for o in orders:
        r = _order_codes(o.expr.eval(df), comm, dev, o.ascending, o.nulls_first)
        if r is None:
            return None
        keys += r
    return _exchange(df, _lex_perm(keys, N, dev), counts)


# ------------------------------------------------------------------------------------------------ dedup
def _first_of(code: torch.Tensor, key: torch.Tensor) -> torch.Tensor:
    """Bool mask of the rows holding the smallest ``key`` of their code."""
    n = code.numel()
    card = int(code.max()) + 1 if n else 0
    from ..ops.group_ops import group_reduce
    best = group_reduce(code, key.to(torch.int64), card, "min", floating=False)
    return best[code] == key


def device_dedup(df, subset: Optional[Sequence[str]]):
    """``dropDuplicates`` keeping each key's first row in global (rank) order; None if unsupported."""
    if not ENABLED:
        return None
    comm, dev = df._comm, df._device
    names = df.columns if subset is None else list(subset)
    cds = [df._cols[n] for n in names]
    if any(_key_kind(c) is None for c in cds):
        ok_local = False
    else:
        ok_local = True
    if comm.is_distributed:
        ok_local = all(comm.allgather_object(ok_local))
    if not ok_local:
        return None
    n = df._nrows
    local = torch.arange(n, dtype=torch.int64, device=dev)
    if n:
        code = _tuple_codes([[c] for c in cds], dev, null_equal=True)
        keep = _first_of(code, local)
    else:
        keep = torch.zeros(0, dtype=torch.bool, device=dev)
    if comm.is_distributed:
        counts = _counts(comm, n)
        off = sum(counts[:comm.rank])
        surv = torch.nonzero(keep).flatten()
        # every rank codes the same concatenation of survivors (rank order)
        blocks = [_blocks(c.take(surv), comm, dev) for c in cds]
        gidx = _gather(comm, surv + off)
        if gidx.numel():
            gcode = _tuple_codes(blocks, dev, null_equal=True)
            gkeep = _first_of(gcode, gidx)
        else:
            gkeep = torch.zeros(0, dtype=torch.bool, device=dev)
        scounts = _counts(comm, int(surv.numel()))
        s0 = sum(scounts[:comm.rank])
        mine = gkeep[s0:s0 + int(surv.numel())]
        keep = torch.zeros(n, dtype=torch.bool, device=dev)
        keep[surv[mine]] = True
    if bool(keep.all()):
        return df
    return df._mask_rows(keep)


def _blocks(cd: ColumnData, comm, dev) -> List[ColumnData]:
    """The column's per-rank blocks (rank order), on every rank."""
    if not comm.is_distributed:
        return [cd]
    if cd.is_host and isinstance(cd.dtype, T.StringType):
        return [_dict_column(c, u, cd.dtype) for c, u in comm.allgather_object(_str_parts(cd))]
    if cd.is_host:
        return [ColumnData(v, None, cd.dtype) for v in comm.allgather_object(_host_values(cd))]
    vs = comm.allgather(cd.values.to(dev).contiguous())
    oks = comm.allgather(cd.valid_mask().to(dev).contiguous())
    return [ColumnData(v, o, cd.dtype) for v, o in zip(vs, oks)]


def _occurrence(code: torch.Tensor) -> torch.Tensor:
    """0-based rank of every row among the earlier rows with the same code."""
    n = code.numel()
    srt, perm = torch.sort(code, stable=True)
    pos = torch.arange(n, device=code.device)
    start = torch.ones(n, dtype=torch.bool, device=code.device)
    start[1:] = srt[1:] != srt[:-1]
    first = torch.cummax(torch.where(start, pos, torch.zeros_like(pos)), 0).values
    occ = torch.empty_like(pos)
    occ[perm] = pos - first
    return occ


def device_set_op(left, right, kind: str):
    """``intersect`` / ``subtract`` (distinct) and ``intersectAll`` / ``exceptAll`` (multiset) on
    whole-row equality codes (nulls equal, as Spark's set operations); the kept rows are this
    rank's left rows, in order. None when a column has no device code."""
    if not ENABLED or len(left.columns) != len(right.columns):
        return None
    comm, dev = left._comm, left._device
    lc = [left._cols[n] for n in left.columns]
    rc = [right._cols[n] for n in right.columns]
    ok = all(_key_kind(a) is not None and _key_kind(a) == _key_kind(b) for a, b in zip(lc, rc))
    if comm.is_distributed:
        ok = all(comm.allgather_object(ok))
    if not ok:
        return None
    lcounts = _counts(comm, left._nrows)
    NL = sum(lcounts)
    if NL == 0:
        return left
    code = _tuple_codes([_blocks(a, comm, dev) + _blocks(b, comm, dev) for a, b in zip(lc, rc)], dev,
                        null_equal=True)
    lcode, rcode = code[:NL], code[NL:]
    rcnt = torch.bincount(rcode, minlength=int(code.max()) + 1)[lcode]
    occ = _occurrence(lcode)
    keep = {"intersect": (occ == 0) & (rcnt > 0), "subtract": (occ == 0) & (rcnt == 0),
            "intersectAll": occ < rcnt, "exceptAll": occ >= rcnt}[kind]
    off = sum(lcounts[:comm.rank])
    mine = keep[off:off + left._nrows]
    return left if bool(mine.all()) else left._mask_rows(mine)


# ------------------------------------------------------------------------------------------------ join
def _gather_frame(df) -> Tuple[Dict[str, ColumnData], int]:
    """Every column of ``df`` over all ranks (rank order) on this rank."""
    comm = df._comm
    if not comm.is_distributed:
        return dict(df._cols), df._nrows
    out = {}
    for name, cd in df._cols.items():
        if cd.is_host and isinstance(cd.dtype, T.StringType):
            out[name] = _dict_column(*_merge_str(_blocks(cd, comm, df._device)), cd.dtype)
        elif cd.is_host:
            vals = np.concatenate(comm.allgather_object(_host_values(cd)))
            ok = np.asarray([x is not None for x in vals], dtype=bool)
            out[name] = ColumnData(vals, None if ok.all() else ok, cd.dtype)
        else:
            out[name] = ColumnData(comm.allgather_cat(cd.values.contiguous()),
                                   comm.allgather_cat(cd.valid_mask().to(cd.values.device).contiguous()), cd.dtype)
    return out, sum(_counts(comm, df._nrows))


def _take_nullable(cd: ColumnData, idx: torch.Tensor) -> ColumnData:
    """Rows ``idx`` of ``cd``; ``idx < 0`` gives null."""
    miss = idx < 0
    safe = torch.clamp(idx, min=0)
    if len(cd) == 0:
        if cd.is_host:
            return ColumnData(np.full(idx.numel(), None, dtype=object), np.zeros(idx.numel(), dtype=bool), cd.dtype)
        shape = (idx.numel(),) + tuple(cd.values.shape[1:])
        return ColumnData(torch.zeros(shape, dtype=cd.values.dtype, device=cd.values.device),
                          torch.zeros(idx.numel(), dtype=torch.bool, device=cd.values.device), cd.dtype)
    if isinstance(cd, DictColumnData):
        codes, uniq = _str_parts(cd)
        c = codes[safe.cpu().numpy()]
        c[miss.cpu().numpy()] = -1
        return _dict_column(c, uniq, cd.dtype)
    if cd.is_host:
        ii = safe.cpu().numpy()
        mm = miss.cpu().numpy()
        vals = _host_values(cd)[ii]
        vals[mm] = None
        ok = ~mm if cd.valid is None else (np.asarray(cd.valid, dtype=bool)[ii] & ~mm)
        return ColumnData(vals, None if ok.all() else ok, cd.dtype)
    d = cd.values.device
    safe, miss = safe.to(d), miss.to(d)
    v = cd.values[safe]
    ok = cd.valid_mask().to(d)[safe] & ~miss
    return ColumnData(v, None if (cd.valid is None and not bool(miss.any())) else ok, cd.dtype)


def _coalesce_cols(a: ColumnData, b: ColumnData, use_b: torch.Tensor) -> ColumnData:
    """``b`` where ``use_b`` else ``a`` (the key columns of unmatched right rows)."""
    if a.is_host or b.is_host:
        av, bv = _host_values(a) if a.is_host else np.asarray(_py(a), dtype=object), \
            _host_values(b) if b.is_host else np.asarray(_py(b), dtype=object)
        m = use_b.cpu().numpy()
        out = np.where(m, bv, av)
        ok = np.asarray([x is not None for x in out], dtype=bool)
        return ColumnData(out, None if ok.all() else ok, a.dtype)
    d = a.values.device
    m = use_b.to(d)
    shape = (-1,) + (1,) * (a.values.dim() - 1)
    v = torch.where(m.view(shape), b.values.to(d).to(a.values.dtype), a.values)
    ok = torch.where(m, b.valid_mask().to(d), a.valid_mask().to(d))
    return ColumnData(v, ok, a.dtype)


def _py(cd):
    from .dataframe import column_to_python
    return column_to_python(cd)


def join_indices(left, rcols: Dict[str, ColumnData], n_right: int, lkeys: List[str], rkeys: List[str],
                 how: str):
    """(li, ri, unmatched-right mask or None): output row t pairs local left row ``li[t]`` (-1 =
    none) with global right row ``ri[t]`` (-1 = none). None when a key has no device code."""
    comm, dev = left._comm, left._device
    n_left = left._nrows
    if how == "cross":
        li = torch.repeat_interleave(torch.arange(n_left, device=dev), n_right)
        ri = torch.arange(n_right, device=dev).repeat(n_left)
        return li, ri
    ok = all(_key_kind(left._cols[a]) is not None and _key_kind(rcols[b]) is not None
             for a, b in zip(lkeys, rkeys))
    if comm.is_distributed:
        ok = all(comm.allgather_object(ok))
    if not ok or not lkeys:
        return None
    code = _tuple_codes([[left._cols[a], rcols[b]] for a, b in zip(lkeys, rkeys)], dev, null_equal=False)
    if code is None:
        return None
    lc, rc = code[:n_left], code[n_left:]
    # codes are dense: per-code counts and starts of the code-sorted right side replace a binary search
    # (at least one code slot: with every key null, or an empty side, the lookups below still index slot 0)
    card = max(int(code.max()) + 2 if code.numel() else 0, 2)
    rperm = torch.sort(rc, stable=True).indices
    rcount = torch.bincount(rc + 1, minlength=card)[1:]           # slot 0 = null keys
    rstart = torch.cumsum(rcount, 0) - rcount + int((rc < 0).sum())  # null right keys sort first
    lsafe = torch.clamp(lc, min=0)
    lo = rstart[lsafe]
    cnt = torch.where(lc >= 0, rcount[lsafe], torch.zeros_like(lo))
    if how in ("leftsemi", "leftanti"):
        keep = cnt > 0 if how == "leftsemi" else cnt == 0
        li = torch.nonzero(keep).flatten()
        return li, None
    outer_left = how in ("left", "full")
    emit = torch.clamp(cnt, min=1) if outer_left else cnt
    total = int(emit.sum()) if n_left else 0
    li = torch.repeat_interleave(torch.arange(n_left, device=dev), emit)
    first = torch.cumsum(emit, 0) - emit
    k = torch.arange(total, device=dev) - first[li]
    hit = cnt[li] > 0
    ri = torch.where(hit, rperm[torch.clamp(lo[li] + k, max=max(n_right - 1, 0))] if n_right else
                     torch.full_like(li, -1), torch.full_like(li, -1))
    if how in ("right", "full"):
        matched = torch.zeros(n_right, dtype=torch.int32, device=dev)
        if ri.numel():
            matched[ri[ri >= 0]] = 1
        if comm.is_distributed:
            comm.allreduce_(matched, "max")
        if comm.rank == comm.world_size - 1:
            extra = torch.nonzero(matched == 0).flatten()
            li = torch.cat([li, torch.full_like(extra, -1)])
            ri = torch.cat([ri, extra])
    return li, ri


def build_join(left, rcols, li, ri, l_out: List[Tuple[str, str]], r_out: List[Tuple[str, str]],
               key_fill: List[Tuple[str, str]], schema):
    """Output frame: left columns ``l_out`` (out name, left name) at ``li``, right columns ``r_out``
    at ``ri``; for rows without a left side the left key columns take the right key (``key_fill``).
    Rows stay on this rank with ids continuing the rank-order numbering."""
    from .dataframe import DataFrame
    comm, dev = left._comm, left._device
    cols = {}
    fill = dict(key_fill)
    for oname, lname in l_out:
        cd = _take_nullable(left._cols[lname], li)
        if lname in fill and ri is not None and bool((li < 0).any()):
            cd = _coalesce_cols(cd, _take_nullable(rcols[fill[lname]], ri), li < 0)
        cols[oname] = cd
    if ri is not None:
        for oname, rname in r_out:
            cols[oname] = _take_nullable(rcols[rname], ri)
    n = int(li.numel())
    counts = _counts(comm, n)
    off = sum(counts[:comm.rank])
    ids = torch.arange(off, off + n, dtype=torch.int64, device=dev)
    return DataFrame(left._session, schema, cols, n, ids, dev)


def device_join(left, right, keys: List[str], how: str, out_names, schema):
    """``DataFrame.join(right, on=keys, how)``: output columns are left's, then right's non-key
    columns named by ``out_names``; None when unsupported."""
    if not ENABLED:
        return None
    rcols, n_right = _gather_frame(right)
    r = join_indices(left, rcols, n_right, keys, keys, how)
    if r is None:
        return None
    li, ri = r
    lnames = left.columns
    l_out = [(n, n) for n in lnames]
    r_extra = [n for n in right.columns if n not in keys]
    r_out = list(zip(out_names[len(lnames):], r_extra)) if ri is not None else []
    return build_join(left, rcols, li, ri, l_out, r_out, [(k, k) for k in keys], schema)
