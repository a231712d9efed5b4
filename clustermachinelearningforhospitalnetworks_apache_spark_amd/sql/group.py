"""Global (cross-shard) relational operators: aggregation, grouping, sort, distinct,
describe, join, rebalance.

Aggregation computes partial statistics per group on each rank (count, Σ,
mean/M2 for Chan's parallel variance merge, min, max), all-gathers the small
partials and merges them; results are placed on ranks round-robin so
``count()``/``collect()`` see every group exactly once.  Sort / distinct / join
gather to the host — they serve reference-scale analytics, not the hot path.
"""
from __future__ import annotations

import math
from typing import Any, Dict, List, Optional, Sequence

import numpy as np
import torch

from . import types as T
from .builder import rows_contiguous, rows_round_robin
from .column import AggExpr, Alias, ColRef, Column, ColumnData, Expr, SortOrder, _to_host
from .dataframe import DataFrame, _as_expr, column_to_python


def _agg_name(e: Expr) -> str:
    return e.name()


def _result_type(fn: str, in_type: Optional[T.DataType], arg=None) -> T.DataType:
    if fn == "count":
        return T.LongType()
    if fn in ("collect_list", "collect_set"):
        return T.ArrayType(in_type or T.StringType())
    if fn == "percentile" and isinstance(arg, (list, tuple)):
        return T.ArrayType(in_type or T.DoubleType())
    if fn in ("avg", "stddev", "stddev_pop", "variance", "var_pop"):
        return T.DoubleType()
    if fn in ("sum", "try_sum"):
        return T.LongType() if in_type is not None and T.is_integral(in_type) else T.DoubleType()
    if fn == "try_avg":
        return T.DoubleType()
    return in_type or T.DoubleType()


def _unwrap(e: Expr):
    alias = None
    if isinstance(e, Alias):
        alias, e = e.alias, e.child
    return alias, e


def _partial(values: List[Any], fn: str, distinct: bool, ignore_nulls: bool = True):
    if fn in ("first", "last"):
        # (kind, value, rows seen): without ignoreNulls the first / last ROW decides, null or not
        vals = values if not ignore_nulls else [v for v in values if v is not None]
        if not vals:
            return (fn, None, False)
        return (fn, vals[0] if fn == "first" else vals[-1], True)
    vals = [v for v in values if v is not None and not (isinstance(v, float) and math.isnan(v) and fn != "count")]
    if fn == "count":
        return ("set", set(vals)) if distinct else ("n", len(vals))
    if fn in ("collect_list", "collect_set", "percentile"):
        return ("list", [_hashable(v) for v in values if v is not None])
    if fn in ("min", "max"):
        if not vals:
            return (fn, None)
        return (fn, min(vals) if fn == "min" else max(vals))
    nums = [float(v) for v in vals]
    if fn in ("sum", "try_sum") and vals and \
            all(isinstance(v, (int, np.integer)) and not isinstance(v, bool) for v in vals):
        # exact (unbounded) integer sum: the merge wraps it to 64 bits (sum, Spark's non-ANSI
        # overflow) or turns an out-of-range total into null (try_sum)
        return ("isum", len(nums), sum(int(v) for v in vals))
    if not nums:
        return ("mom", 0, 0.0, 0.0, 0.0)
    a = np.asarray(nums, dtype=np.float64)
    mu = float(a.mean())
    return ("mom", len(nums), float(a.sum()), mu, float(((a - mu) ** 2).sum()))


def _merge(parts, fn: str):
    kind = parts[0][0]
    if kind == "n":
        return sum(p[1] for p in parts)
    if kind == "set":
        s = set()
        for p in parts:
            s |= p[1]
        return len(s)
    if kind == "first":
        for p in parts:
            if p[2]:
                return p[1]
        return None
    if kind == "last":
        for p in reversed(parts):
            if p[2]:
                return p[1]
        return None
    if kind == "list":
        vals = [v for p in parts for v in p[1]]
        if fn == "collect_list":
            return vals
        if fn == "collect_set":
            out, seen = [], set()
            for v in vals:
                if v not in seen:
                    seen.add(v)
                    out.append(v)
            return out
        return vals  # percentile: finished by _percentile with the requested fractions
    if kind in ("min", "max"):
        vals = [p[1] for p in parts if p[1] is not None]
        if not vals:
            return None
        return min(vals) if kind == "min" else max(vals)
    if kind == "isum" or all(p[0] == "isum" for p in parts):
        n = sum(p[1] for p in parts if p[0] == "isum")
        s = sum(p[2] for p in parts if p[0] == "isum") + sum(p[2] for p in parts if p[0] == "mom")
        if not n:
            return None
        if fn == "try_sum":
            return s if -2 ** 63 <= s < 2 ** 63 else None
        return (s + 2 ** 63) % 2 ** 64 - 2 ** 63  # two's-complement wrap, as Spark's LongType sum
    # Chan et al. parallel merge of (count, mean, M2)
    n, mean, m2, s = 0, 0.0, 0.0, 0.0
    for p in parts:
        if p[0] != "mom" or p[1] == 0:
            continue
        nb, sb, mb, m2b = p[1], p[2], p[3], p[4]
        delta = mb - mean
        tot = n + nb
        mean = mean + delta * nb / tot
        m2 = m2 + m2b + delta * delta * n * nb / tot
        n = tot
        s += sb
    if n == 0:
        return None
    if fn in ("sum", "try_sum"):
        return s
    if fn in ("avg", "try_avg"):
        return s / n
    var_pop = max(m2 / n, 0.0)
    if fn in ("var_pop", "stddev_pop"):
        return var_pop if fn == "var_pop" else math.sqrt(var_pop)
    if n < 2:
        return None
    var = var_pop * n / (n - 1)
    return var if fn == "variance" else math.sqrt(var)


def local_partials(df: DataFrame, keys: List[Expr], exprs: List[Expr]):
    """This rank's per-group partial aggregates: (specs, key_types, {key tuple: [partial per spec]}).
    A spec is ("key", name, key index, None) or ("agg", name, AggExpr, values, input type)."""
    from . import group_fast
    from .window import _WINDOW_TYPE, TimeWindow
    if group_fast.ENABLED:
        fast = group_fast.fast_local_partials(df, keys, exprs)
        if fast is not None:
            return fast
    key_names = [k.name() for k in keys]
    # time-window keys (functions.window) may put a row into several buckets: expand rows first
    src = list(range(df._nrows))
    key_vals, key_types = [], []
    for k in keys:
        if isinstance(k, TimeWindow):
            key_vals.append(("tw", k.buckets(df)))
            key_types.append(_WINDOW_TYPE)
        else:
            cd = k.eval(df)
            key_vals.append(("col", column_to_python(cd)))
            key_types.append(cd.dtype)
    if any(kind == "tw" for kind, _ in key_vals):
        # expanded row list: one entry per (row, bucket) of the first time-window key
        tw = next(v for kind, v in key_vals if kind == "tw")
        src = [i for i in range(df._nrows) for _ in tw[i]]
        which = []
        for i in range(df._nrows):
            which += list(range(len(tw[i])))
        key_vals = [[v[i] for i in src] if kind == "col" else [v[i][w] for i, w in zip(src, which)]
                    for kind, v in key_vals]
    else:
        key_vals = [v for _, v in key_vals]
    specs = []
    for e in exprs:
        alias, inner = _unwrap(e)
        if not isinstance(inner, AggExpr):
            if isinstance(inner, ColRef) and inner.col in key_names:
                specs.append(("key", alias or inner.col, key_names.index(inner.col), None))
                continue
            raise ValueError(f"expression {e} is neither an aggregate nor a grouping column")
        if getattr(inner, "custom", False):
            # device-side aggregate (e.g. ml.stat.Summarizer): prepare / partial / merge hooks
            specs.append(("agg", alias or _agg_name(inner), inner, inner.prepare(df), None))
            continue
        if inner.child is None:
            vals = [1] * len(src)
            itype = T.LongType()
        else:
            cd = inner.child.eval(df)
            vals = column_to_python(cd)
            vals = [vals[i] for i in src] if len(src) != df._nrows or src != list(range(df._nrows)) else vals
            itype = cd.dtype
        specs.append(("agg", alias or _agg_name(inner), inner, vals, itype))
    groups: Dict[tuple, List[Any]] = {}
    order: List[tuple] = []
    for i in range(len(src)):
        key = tuple(kv[i] for kv in key_vals)
        if key not in groups:
            groups[key] = []
            order.append(key)
        groups[key].append(i)
    if not keys and not groups:
        groups[()] = []
        order.append(())
    local = {}
    for key in order:
        idx = groups[key]
        parts = []
        for sp in specs:
            if sp[0] == "key":
                parts.append(None)
            else:
                _, _, agg, vals, _ = sp
                if getattr(agg, "custom", False):
                    parts.append(agg.partial(vals, [src[i] for i in idx]))
                else:
                    parts.append(_partial([vals[i] for i in idx], agg.fn, agg.distinct,
                                          getattr(agg, "ignore_nulls", False)))
        local[key] = parts
    return specs, key_types, local


def gather_partials(comm, local, nspecs: int):
    """All ranks' partials per group, in first-seen (rank, local) order: ({key: [[partials] per spec]}, keys)."""
    merged: Dict[tuple, List[List[Any]]] = {}
    morder: List[tuple] = []
    for part in comm.allgather_object(local):
        for key, parts in part.items():
            if key not in merged:
                merged[key] = [[] for _ in range(nspecs)]
                morder.append(key)
            for j, p in enumerate(parts):
                if p is not None:
                    merged[key][j].append(p)
    return merged, morder


def final_row(key: tuple, parts: List[List[Any]], specs) -> List[Any]:
    row = []
    for j, sp in enumerate(specs):
        if sp[0] == "key":
            row.append(key[sp[2]])
        elif getattr(sp[2], "custom", False):
            row.append(sp[2].merge(parts[j]))
        else:
            v = _merge(parts[j], sp[2].fn)
            if sp[2].fn == "percentile":
                v = _percentile(v, getattr(sp[2], "arg", 0.5))
            row.append(v)
    return row


def result_schema(specs, key_types) -> T.StructType:
    fields = []
    for sp in specs:
        if sp[0] == "key":
            fields.append(T.StructField(sp[1], key_types[sp[2]], True))
        elif getattr(sp[2], "custom", False):
            fields.append(T.StructField(sp[1], sp[2].result_type(), True))
        else:
            fields.append(T.StructField(sp[1], _result_type(sp[2].fn, sp[4], getattr(sp[2], "arg", None)), True))
    return T.StructType(fields)


def fix_long_columns(schema: T.StructType, rows: List[List[Any]]) -> None:
    for j, f in enumerate(schema.fields):
        if isinstance(f.dataType, T.LongType):
            for r in rows:
                if r[j] is not None:
                    r[j] = int(r[j])


def combine_partials(parts: List[Any], fn: str):
    """Several partials of one built-in aggregate -> one partial of the same kind (streaming state)."""
    if not parts:
        return None
    kind = parts[0][0]
    if kind == "n":
        return ("n", sum(p[1] for p in parts))
    if kind == "set":
        out = set()
        for p in parts:
            out |= p[1]
        return ("set", out)
    if kind in ("first", "last"):
        rows = any(p[2] for p in parts)
        return (kind, _merge(parts, fn), rows)
    if kind == "list":
        return ("list", [v for p in parts for v in p[1]])
    if kind in ("min", "max"):
        return (kind, _merge(parts, fn))
    live = [p for p in parts if not (p[0] == "mom" and p[1] == 0)]
    if not live:
        return ("mom", 0, 0.0, 0.0, 0.0)
    if all(p[0] == "isum" for p in live):
        return ("isum", sum(p[1] for p in live), sum(p[2] for p in live))
    n, mean, m2, s = 0, 0.0, 0.0, 0.0
    for p in live:
        if p[0] == "isum":
            nb, sb = p[1], float(p[2])
            mb, m2b = (sb / nb if nb else 0.0), 0.0
        else:
            nb, sb, mb, m2b = p[1], p[2], p[3], p[4]
        delta = mb - mean
        tot = n + nb
        mean = mean + delta * nb / tot
        m2 = m2 + m2b + delta * delta * n * nb / tot
        n = tot
        s += sb
    return ("mom", n, s, mean, m2)


def aggregate(df: DataFrame, keys: List[Expr], exprs: List[Expr]) -> DataFrame:
    from .window import SessionWindow, materialize_sessions
    if any(isinstance(k, SessionWindow) for k in keys):
        # sessions depend on the other keys: materialise them as a column, then group by it
        df, keys, _ = materialize_sessions(df, keys)
    from .aggregate_fast import device_aggregate
    out = device_aggregate(df, keys, exprs)
    if out is not None:
        return out
    specs, key_types, local = local_partials(df, keys, exprs)
    merged, morder = gather_partials(df._comm, local, len(specs))
    rows = [final_row(key, merged[key], specs) for key in morder]
    schema = result_schema(specs, key_types)
    fix_long_columns(schema, rows)
    return rows_round_robin(df._session, schema, rows)


def _as_key_exprs(cols) -> List[Expr]:
    from .dataframe import _as_expr
    if len(cols) == 1 and isinstance(cols[0], (list, tuple)):
        cols = tuple(cols[0])
    return [_as_expr(c) for c in cols]


class GroupedData:
    def __init__(self, df: DataFrame, keys: List[Expr]):
        self.df = df
        self.keys = keys

    def pivot(self, pivot_col, values=None):
        from .dataframe_more import PivotedData
        return PivotedData(self.df, self.keys, pivot_col, list(values) if values is not None else None)

    def applyInPandas(self, func, schema):
        from .dataframe_more import apply_in_pandas
        return apply_in_pandas(self, func, schema)

    def agg(self, *exprs) -> DataFrame:
        if len(exprs) == 1 and isinstance(exprs[0], dict):
            from . import functions as F
            exprs = tuple(getattr(F, fn if fn != "mean" else "avg")(c).alias(f"{fn}({c})")
                          for c, fn in exprs[0].items())
        es = [ColRef(k.name()) for k in self.keys] + [_as_expr(e) for e in exprs]
        if self.df.isStreaming:
            return self.df._lazy("_stream_aggregate", self.keys, es)
        return aggregate(self.df, self.keys, es)

    def _simple(self, fn: str, cols) -> DataFrame:
        from . import functions as F
        if not cols:
            cols = [f.name for f in self.df.schema.fields
                    if T.is_numeric(f.dataType) and f.name not in [k.name() for k in self.keys]]
        return self.agg(*[getattr(F, fn)(c).alias(f"{fn}({c})") for c in cols])

    def count(self) -> DataFrame:
        from . import functions as F
        return self.agg(F.count("*").alias("count"))

    def sum(self, *cols): return self._simple("sum", cols)
    def avg(self, *cols): return self._simple("avg", cols)
    mean = avg
    def min(self, *cols): return self._simple("min", cols)
    def max(self, *cols): return self._simple("max", cols)


def _sort_key(v, ascending: bool, nulls_first: bool):
    if v is None:
        return (0 if nulls_first else 2, 0)
    return (1, v if ascending else _Neg(v))


class _Neg:
    __slots__ = ("v",)

    def __init__(self, v):
        self.v = v

    def __lt__(self, o):
        return self.v > o.v

    def __gt__(self, o):
        return self.v < o.v

    def __eq__(self, o):
        return self.v == o.v


def sort_frame(df: DataFrame, orders: List[SortOrder]) -> DataFrame:
    from .relational_fast import device_sort
    out = device_sort(df, orders)
    if out is not None:
        return out
    names, rows, ids = df._gather_host()
    keyvals = []
    for o in orders:
        kcol = column_to_python(o.expr.eval(df))
        keyvals.append(df._comm.allgather_object(kcol))
    flat_keys = [[v for part in kv for v in part] for kv in keyvals]
    perm = sorted(range(len(rows)), key=lambda i: tuple(
        _sort_key(flat_keys[j][i], o.ascending, o.nulls_first) for j, o in enumerate(orders)))
    rows = [rows[i] for i in perm]
    ids = [ids[i] for i in perm]
    return rows_contiguous(df._session, df.schema, rows, ids)


def drop_duplicates(df: DataFrame, subset: Optional[Sequence[str]]) -> DataFrame:
    from .relational_fast import device_dedup
    out = device_dedup(df, subset)
    if out is not None:
        return out
    names, rows, ids = df._gather_host()
    cols = list(range(len(names))) if subset is None else [names.index(c) for c in subset]
    seen = set()
    keep_rows, keep_ids = [], []
    for r, i in zip(rows, ids):
        key = tuple(_hashable(r[c]) for c in cols)
        if key in seen:
            continue
        seen.add(key)
        keep_rows.append(r)
        keep_ids.append(i)
    return rows_contiguous(df._session, df.schema, keep_rows, keep_ids)


def _percentile(vals: List[Any], p):
    """Smallest value whose rank reaches ceil(p·n) (Spark percentile_approx's exact limit)."""
    if not vals:
        return None
    srt = sorted(vals)

    def one(q):
        q = float(q)
        if not 0.0 <= q <= 1.0:
            raise ValueError("percentage must be in [0, 1]")
        i = max(int(math.ceil(q * len(srt))) - 1, 0)
        return srt[i]
    if isinstance(p, (list, tuple)):
        return [one(q) for q in p]
    return one(p)


def _hashable(v):
    if hasattr(v, "toArray"):
        return tuple(v.toArray().tolist())
    return v


def describe(df: DataFrame, cols: List[str]) -> DataFrame:
    from . import functions as F
    if not cols:
        cols = [f.name for f in df.schema.fields if T.is_numeric(f.dataType) or isinstance(f.dataType, T.StringType)]
    stats = ["count", "mean", "stddev", "min", "max"]
    out_rows = [[s] for s in stats]
    for c in cols:
        is_num = T.is_numeric(df.schema[c].dataType)
        exprs = [F.count(c)]
        if is_num:
            exprs += [F.avg(c), F.stddev(c)]
        exprs += [F.min(c), F.max(c)]
        vals = df.agg(*exprs).collect()[0]
        if is_num:
            cnt, mean, sd, mn, mx = vals
        else:
            cnt, mn, mx = vals
            mean = sd = None
        for r, v in zip(out_rows, [cnt, mean, sd, mn, mx]):
            r.append(None if v is None else str(v))
    schema = T.StructType([T.StructField("summary", T.StringType())] + [T.StructField(c, T.StringType()) for c in cols])
    return rows_round_robin(df._session, schema, out_rows)


def join_frames(left: DataFrame, right: DataFrame, on, how: str) -> DataFrame:
    """Equi-join on column names. Device path: relational_fast (joint key codes, sorted right side,
    per-code count and prefix-sum match ranges); the row loop below (broadcast hash join, right side gathered to
    every rank) handles keys without device codes. Null keys never match (Spark equality).
    Right non-key columns whose names clash with left ones get an ``_r`` suffix."""
    how = how.lower().replace("_", "")
    how = {"leftouter": "left", "rightouter": "right", "fullouter": "full", "outer": "full",
           "semi": "leftsemi", "anti": "leftanti"}.get(how, how)
    lnames = left.columns
    if on is None:
        keys = []
    elif isinstance(on, str):
        keys = [on]
    elif isinstance(on, (list, tuple)) and all(isinstance(k, str) for k in on):
        keys = list(on)
    else:
        raise NotImplementedError("join supports column-name keys")
    if not keys and how != "cross":
        how = "cross"
    r_extra = [n for n in right.columns if n not in keys]
    semi = how in ("leftanti", "leftsemi")
    out_names = lnames if semi else lnames + [n + "_r" if n in lnames else n for n in r_extra]
    fields = [T.StructField(n, left.schema[n].dataType) for n in lnames]
    if not semi:
        fields += [T.StructField(o, right.schema[n].dataType) for o, n in zip(out_names[len(lnames):], r_extra)]
    schema = T.StructType(fields)
    from .relational_fast import device_join
    out = device_join(left, right, keys, how, out_names, schema)
    if out is not None:
        return out
    rnames, rrows, _ = right._gather_host()
    lcols = left._local_rows_host()
    index: Dict[tuple, List[int]] = {}
    for j, r in enumerate(rrows):
        key = tuple(_hashable(r[rnames.index(k)]) for k in keys)
        if any(v is None for v in key):
            continue
        index.setdefault(key, []).append(j)
    r_out_idx = [rnames.index(n) for n in r_extra]
    out_rows = []
    matched_right = set()
    for i in range(left._nrows):
        lrow = [lcols[n][i] for n in lnames]
        key = tuple(_hashable(lcols[k][i]) for k in keys)
        hits = list(range(len(rrows))) if how == "cross" else index.get(key, [])
        if semi:
            if bool(hits) == (how == "leftsemi"):
                out_rows.append(lrow)
            continue
        if hits:
            for j in hits:
                matched_right.add(j)
                out_rows.append(lrow + [rrows[j][t] for t in r_out_idx])
        elif how in ("left", "full"):
            out_rows.append(lrow + [None] * len(r_out_idx))
    if how in ("right", "full"):
        allm = left._comm.allgather_object(sorted(matched_right))
        m = set()
        for a in allm:
            m |= set(a)
        if left._comm.rank == left._comm.world_size - 1:
            for j, r in enumerate(rrows):
                if j not in m:
                    lrow = [r[rnames.index(n)] if n in keys else None for n in lnames]
                    out_rows.append(lrow + [r[t] for t in r_out_idx])
    # gather-free placement: keep this rank's output rows local
    from .builder import frame_from_pycolumns
    pycols = {f.name: [r[j] for r in out_rows] for j, f in enumerate(schema.fields)}
    counts = left._comm.allgather_object(len(out_rows))
    off = sum(counts[: left._comm.rank])
    return frame_from_pycolumns(left._session, schema, pycols, list(range(off, off + len(out_rows))))


def rebalance(df: DataFrame) -> DataFrame:
    from .relational_fast import device_rebalance
    out = device_rebalance(df)
    if out is not None:
        return out
    names, rows, ids = df._gather_host()
    return rows_contiguous(df._session, df.schema, rows, ids)
