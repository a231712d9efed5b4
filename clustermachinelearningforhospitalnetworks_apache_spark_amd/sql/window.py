"""Window functions: ``pyspark.sql.Window`` / ``WindowSpec`` and ``Column.over``.

Beyond the reference (which only filters a time range, ref.py:123-128), these are what a
hospital-operations job over the unbounded event table reaches for next: per-hospital running
occupancy, the previous reading of the same hospital (``lag``), a rank of admissions within a day.

Semantics follow Spark SQL:

* ranking functions (``row_number``, ``rank``, ``dense_rank``, ``percent_rank``, ``cume_dist``,
  ``ntile``) and offsets (``lag``, ``lead``) need an ``orderBy`` and ignore the frame;
* aggregates (``sum``, ``avg``, ``count``, ``min``, ``max``, ``first``, ``last``, ``stddev``, ...)
  run over the frame. Default frame: ``RANGE BETWEEN UNBOUNDED PRECEDING AND CURRENT ROW`` (peers
  of the current row included) with an ``orderBy``, the whole partition without one;
* ``rowsBetween(start, end)`` counts rows, ``rangeBetween(start, end)`` offsets the (single,
  numeric) ordering value; ``Window.unboundedPreceding`` / ``unboundedFollowing`` / ``currentRow``;
* ordering puts nulls first ascending and last descending, nulls are skipped by aggregates.

Execution: partitions may span ranks, so a window expression gathers its partition keys, ordering
keys and argument (host values) over the communicator, evaluates every partition with vectorised
numpy (lexicographic sort, segment boundaries, prefix sums for sliding sums/counts), and keeps this
rank's rows. Reference-scale analytics, like ``orderBy``/``join`` (``group.py``), not the GPU hot path.
"""
from __future__ import annotations

import math
import sys
from typing import Any, Dict, List, Optional, Sequence

import numpy as np
import torch

from . import types as T
from .column import AggExpr, ColRef, Column, ColumnData, Expr, SortOrder, _expr

DEVICE_WINDOWS = True  # window_fast.device_window first; tests flip this to compare with the host path
_UNB_PREC = -sys.maxsize - 1
_UNB_FOLL = sys.maxsize


def _order(x) -> SortOrder:
    if isinstance(x, SortOrder):
        return x
    if isinstance(x, str):
        return SortOrder(ColRef(x), True)
    return SortOrder(_expr(x), True)


class WindowSpec:
    def __init__(self, partition: Sequence[Expr] = (), orders: Sequence[SortOrder] = (), frame=None):
        self._partition = list(partition)
        self._orders = list(orders)
        self._frame = frame  # None | ("rows" | "range", start, end)

    def partitionBy(self, *cols) -> "WindowSpec":
        if len(cols) == 1 and isinstance(cols[0], (list, tuple)):
            cols = tuple(cols[0])
        return WindowSpec([ColRef(c) if isinstance(c, str) else _expr(c) for c in cols], self._orders, self._frame)

    def orderBy(self, *cols) -> "WindowSpec":
        if len(cols) == 1 and isinstance(cols[0], (list, tuple)):
            cols = tuple(cols[0])
        return WindowSpec(self._partition, [_order(c) for c in cols], self._frame)

    def rowsBetween(self, start: int, end: int) -> "WindowSpec":
        return WindowSpec(self._partition, self._orders, ("rows", int(start), int(end)))

    def rangeBetween(self, start: int, end: int) -> "WindowSpec":
        return WindowSpec(self._partition, self._orders, ("range", start, end))

    def __repr__(self):
        return f"WindowSpec(partition={len(self._partition)}, order={len(self._orders)}, frame={self._frame})"


class Window:
    unboundedPreceding = _UNB_PREC
    unboundedFollowing = _UNB_FOLL
    currentRow = 0

    @staticmethod
    def partitionBy(*cols) -> WindowSpec:
        return WindowSpec().partitionBy(*cols)

    @staticmethod
    def orderBy(*cols) -> WindowSpec:
        return WindowSpec().orderBy(*cols)

    @staticmethod
    def rowsBetween(start: int, end: int) -> WindowSpec:
        return WindowSpec().rowsBetween(start, end)

    @staticmethod
    def rangeBetween(start: int, end: int) -> WindowSpec:
        return WindowSpec().rangeBetween(start, end)


# ------------------------------------------------------------------------------------------------ expressions

class WindowFunc(Expr):
    """A ranking / offset function that is only valid with ``.over(window)``."""

    def __init__(self, fn: str, child: Optional[Expr] = None, arg: Any = None, default: Any = None):
        self.fn, self.child, self.arg, self.default = fn, child, arg, default

    def refs(self):
        return self.child.refs() if self.child is not None else []

    def __str__(self):
        inner = "" if self.child is None else str(self.child)
        if self.fn in ("lag", "lead"):
            inner += f", {self.arg}, {self.default}"
        elif self.fn == "ntile":
            inner = str(self.arg)
        elif self.fn == "nth_value":
            inner += f", {self.arg}" + (", true" if self.default else "")
        return f"{self.fn}({inner})"

    def eval(self, frame):
        raise ValueError(f"window function {self} needs .over(Window...)")


class WindowExpr(Expr):
    def __init__(self, func: Expr, spec: WindowSpec):
        if not isinstance(func, (WindowFunc, AggExpr)):
            raise ValueError(f"{func} is not a window or aggregate function")
        if isinstance(func, AggExpr) and func.distinct:
            raise NotImplementedError("DISTINCT aggregates over a window")
        self.func, self.spec = func, spec

    def refs(self):
        out = list(self.func.refs())
        for e in self.spec._partition:
            out += e.refs()
        for o in self.spec._orders:
            out += o.expr.refs()
        return out

    def __str__(self):
        parts = []
        if self.spec._partition:
            parts.append("PARTITION BY " + ", ".join(str(e) for e in self.spec._partition))
        if self.spec._orders:
            parts.append("ORDER BY " + ", ".join(f"{o.expr} {'ASC' if o.ascending else 'DESC'}"
                                                 for o in self.spec._orders))
        return f"{self.func} OVER ({' '.join(parts)})"

    def eval(self, frame) -> ColumnData:
        from .builder import column_from_values
        from .dataframe import column_to_python
        if DEVICE_WINDOWS:
            from .window_fast import device_window
            fast = device_window(frame, self.func, self.spec)
            if fast is not None:
                return fast
        comm = frame._comm
        child = self.func.child
        pk = [column_to_python(e.eval(frame)) for e in self.spec._partition]
        ok = [column_to_python(o.expr.eval(frame)) for o in self.spec._orders]
        cd = child.eval(frame) if child is not None else None
        arg = column_to_python(cd) if cd is not None else None
        n = frame._nrows
        if comm.is_distributed:
            parts = comm.allgather_object((pk, ok, arg, n))
            off = sum(p[3] for p in parts[: comm.rank])
            pk = [[v for p in parts for v in p[0][j]] for j in range(len(pk))]
            ok = [[v for p in parts for v in p[1][j]] for j in range(len(ok))]
            arg = None if arg is None else [v for p in parts for v in p[2]]
            total = sum(p[3] for p in parts)
        else:
            off, total = 0, n
        out = _evaluate(self.func, self.spec, pk, ok, arg, total)
        dtype = _result_type(self.func, cd.dtype if cd is not None else None)
        return column_from_values(out[off:off + n], dtype, frame._device)


def over(col: Column, spec: WindowSpec) -> Column:
    return Column(WindowExpr(col._expr, spec))


def _result_type(func, in_type: Optional[T.DataType]) -> T.DataType:
    fn = func.fn
    if fn in ("row_number", "rank", "dense_rank", "ntile"):
        return T.IntegerType()
    if fn in ("percent_rank", "cume_dist", "avg", "try_avg", "stddev", "stddev_pop", "variance", "var_pop"):
        return T.DoubleType()
    if fn == "count":
        return T.LongType()
    if fn in ("sum", "try_sum"):
        return T.LongType() if in_type is not None and T.is_integral(in_type) else T.DoubleType()
    return in_type or T.DoubleType()


# ------------------------------------------------------------------------------------------------ evaluation

def _sort_perm(pk: List[list], ok: List[list], orders: List[SortOrder], n: int) -> np.ndarray:
    """Stable order of all rows by (partition keys, ordering keys with Spark's null placement)."""
    keys = []  # np.lexsort: last key is primary
    for vals, o in reversed(list(zip(ok, orders))):
        codes, nulls = _codes(vals)
        if not o.ascending:
            codes = -codes
        null_rank = np.where(nulls, 0 if o.nulls_first else 2, 1)
        keys.append(codes)
        keys.append(null_rank)
    for vals in reversed(pk):
        codes, nulls = _codes(vals)
        keys.append(codes)
        keys.append(nulls.astype(np.int64))
    if not keys:
        return np.arange(n)
    return np.lexsort(keys)


def _codes(vals: list):
    """Order-preserving integer codes of arbitrary comparable values (nulls -> code 0 + flag)."""
    n = len(vals)
    nulls = np.array([v is None for v in vals], dtype=bool)
    present = [v for v in vals if v is not None]
    if not present:
        return np.zeros(n, dtype=np.int64), nulls
    uniq = sorted(set(present))
    index = {v: i + 1 for i, v in enumerate(uniq)}
    return np.array([0 if v is None else index[v] for v in vals], dtype=np.int64), nulls


def _evaluate(func, spec: WindowSpec, pk, ok, arg, n: int) -> list:
    out: list = [None] * n
    if n == 0:
        return out
    perm = _sort_perm(pk, ok, spec._orders, n)
    # partition boundaries in sorted order
    pkey = [tuple(col[i] for col in pk) for i in perm] if pk else [()] * n
    okey = [tuple(col[i] for col in ok) for i in perm] if ok else [()] * n
    starts = [0] + [i for i in range(1, n) if pkey[i] != pkey[i - 1]] + [n]
    fn = func.fn
    for a, b in zip(starts[:-1], starts[1:]):
        idx = perm[a:b]
        ov = okey[a:b]
        m = b - a
        if isinstance(func, WindowFunc) and fn == "nth_value":
            res = _nth_value(func, spec, ov, [arg[i] for i in idx], m)
        elif isinstance(func, WindowFunc):
            res = _rank_like(func, ov, [arg[i] for i in idx] if arg is not None else None, m)
        else:
            res = _frame_agg(fn, spec, ov, [arg[i] for i in idx] if arg is not None else [1] * m, m,
                             count_star=func.child is None, ignore_nulls=getattr(func, "ignore_nulls", False))
        for j, i in enumerate(idx):
            out[i] = res[j]
    return out


def _nth_value(func: WindowFunc, spec: WindowSpec, ov: list, vals: list, m: int) -> list:
    """``nth_value(col, k[, ignoreNulls])``: the k-th (non-null) value of each row's frame."""
    k, skip_nulls = int(func.arg), bool(func.default)
    lo, hi = _frame_bounds(spec, ov, m)
    out = []
    for i in range(m):
        if skip_nulls:
            seen = [v for v in vals[lo[i]:hi[i] + 1] if v is not None]
            out.append(seen[k - 1] if len(seen) >= k else None)
        else:
            j = lo[i] + k - 1
            out.append(vals[j] if j <= hi[i] else None)
    return out


def _peer_bounds(ov: list, m: int):
    """first/last index of each row's peer group (equal ordering key)."""
    first = [0] * m
    last = [0] * m
    s = 0
    for i in range(1, m + 1):
        if i == m or ov[i] != ov[i - 1]:
            for j in range(s, i):
                first[j], last[j] = s, i - 1
            s = i
    return first, last


def _rank_like(func: WindowFunc, ov: list, vals: Optional[list], m: int) -> list:
    fn = func.fn
    if fn == "row_number":
        return list(range(1, m + 1))
    if fn in ("rank", "dense_rank", "percent_rank", "cume_dist"):
        first, last = _peer_bounds(ov, m)
        if fn == "rank":
            return [f + 1 for f in first]
        if fn == "percent_rank":
            return [0.0 if m == 1 else f / (m - 1) for f in first]
        if fn == "cume_dist":
            return [(l + 1) / m for l in last]
        out, d = [], 0
        for i in range(m):
            if i == 0 or first[i] == i:
                d += 1
            out.append(d)
        return out
    if fn == "ntile":
        k = int(func.arg)
        base, extra = divmod(m, k)
        out = []
        for b in range(k):
            out += [b + 1] * (base + (1 if b < extra else 0))
        return out[:m]
    if fn in ("lag", "lead"):
        off = int(func.arg) * (-1 if fn == "lag" else 1)
        return [vals[i + off] if 0 <= i + off < m else func.default for i in range(m)]
    raise ValueError(f"unknown window function {fn}")


def _frame_bounds(spec: WindowSpec, ov: list, m: int):
    frame = spec._frame
    if frame is None:
        if not spec._orders:
            return [0] * m, [m - 1] * m
        frame = ("range", _UNB_PREC, 0)
    kind, s, e = frame
    if kind == "rows":
        lo = [0 if s <= _UNB_PREC else max(0, i + s) for i in range(m)]
        hi = [m - 1 if e >= _UNB_FOLL else min(m - 1, i + e) for i in range(m)]
        return lo, hi
    first, last = _peer_bounds(ov, m)
    if s in (_UNB_PREC, 0) and e in (_UNB_FOLL, 0):
        lo = [0 if s == _UNB_PREC else first[i] for i in range(m)]
        hi = [m - 1 if e == _UNB_FOLL else last[i] for i in range(m)]
        return lo, hi
    if len(spec._orders) != 1:
        raise ValueError("rangeBetween with value offsets needs exactly one ordering column")
    sign = 1 if spec._orders[0].ascending else -1
    v = np.array([x[0] if x[0] is not None else np.nan for x in ov], dtype=np.float64) * sign
    lo, hi = [], []
    for i in range(m):
        if math.isnan(v[i]):  # null ordering value: its frame is its (null) peer group
            lo.append(first[i])
            hi.append(last[i])
            continue
        a = 0 if s == _UNB_PREC else int(np.searchsorted(v, v[i] + s, side="left"))
        z = m - 1 if e == _UNB_FOLL else int(np.searchsorted(v, v[i] + e, side="right")) - 1
        lo.append(a)
        hi.append(z)
    return lo, hi


def _frame_agg(fn: str, spec: WindowSpec, ov: list, vals: list, m: int, count_star: bool,
               ignore_nulls: bool = False) -> list:
    lo, hi = _frame_bounds(spec, ov, m)
    present = np.array([v is not None for v in vals], dtype=bool)
    try_sum = fn == "try_sum"
    fn = {"try_sum": "sum", "try_avg": "avg"}.get(fn, fn)
    if fn in ("sum", "avg", "count"):
        if count_star:
            present = np.ones(m, dtype=bool)
        cnt = np.concatenate([[0], np.cumsum(present)])
        if fn == "count":
            return [int(cnt[h + 1] - cnt[l]) if h >= l else 0 for l, h in zip(lo, hi)]
        integral = all(isinstance(v, (int, np.integer)) and not isinstance(v, bool) for v in vals if v is not None)
        if fn == "sum" and integral:
            # exact prefix sums (Python ints); sum wraps to 64 bits, try_sum turns overflow into null
            acc = [0]
            for v in vals:
                acc.append(acc[-1] + (int(v) if v is not None else 0))
            out = []
            for l, h in zip(lo, hi):
                if h < l or cnt[h + 1] - cnt[l] == 0:
                    out.append(None)
                    continue
                t = acc[h + 1] - acc[l]
                if try_sum:
                    out.append(t if -2 ** 63 <= t < 2 ** 63 else None)
                else:
                    out.append((t + 2 ** 63) % 2 ** 64 - 2 ** 63)
            return out
        x = np.array([float(v) if v is not None else 0.0 for v in vals], dtype=np.float64)
        out = []
        for l, h in zip(lo, hi):
            c = int(cnt[h + 1] - cnt[l]) if h >= l else 0
            if c == 0:
                out.append(None)
                continue
            s = float(x[l:h + 1].sum())  # exact-order sum of the frame (no prefix-sum cancellation)
            out.append(s if fn == "sum" else s / c)
        return out
    out = []
    for l, h in zip(lo, hi):
        seg = [v for v in vals[l:h + 1] if v is not None] if h >= l else []
        if fn in ("first", "last") and ignore_nulls:
            out.append((seg[0] if fn == "first" else seg[-1]) if seg else None)
        elif fn == "first":
            out.append(vals[l] if h >= l else None)
        elif fn == "last":
            out.append(vals[h] if h >= l else None)
        elif not seg:
            out.append(None)
        elif fn == "min":
            out.append(min(seg))
        elif fn == "max":
            out.append(max(seg))
        elif fn in ("stddev", "variance", "stddev_pop", "var_pop"):
            a = np.asarray(seg, dtype=np.float64)
            pop = fn.endswith("_pop")
            if len(a) < (1 if pop else 2):
                out.append(None)
                continue
            var = float(a.var(ddof=0 if pop else 1))
            out.append(math.sqrt(var) if fn.startswith("stddev") else var)
        else:
            raise ValueError(f"aggregate {fn} is not supported over a window")
    return out


# ------------------------------------------------------------------------------------------------ time windows

_WINDOW_TYPE = T.StructType([T.StructField("start", T.TimestampType(), True),
                             T.StructField("end", T.TimestampType(), True)])


class TimeWindow(Expr):
    """``functions.window(timeColumn, windowDuration, slideDuration, startTime)``: the event-time
    bucket(s) of each row as ``struct<start: timestamp, end: timestamp>``. Tumbling windows
    (slide = duration) give one bucket per row; sliding windows give ceil(duration / slide), and
    ``groupBy(window(...))`` counts the row in each of them (Spark's expand)."""

    def __init__(self, child: Expr, dur_us: int, slide_us: int, start_us: int):
        if dur_us <= 0 or slide_us <= 0 or slide_us > dur_us:
            raise ValueError("window needs 0 < slideDuration <= windowDuration")
        self.child, self.dur, self.slide, self.start = child, dur_us, slide_us, start_us % slide_us

    def refs(self):
        return self.child.refs()

    def name(self):
        return "window"

    def __str__(self):
        return f"window({self.child}, {self.dur}us, {self.slide}us, {self.start}us)"

    def buckets(self, frame) -> List[list]:
        """Per row: the list of Row(start, end) windows containing its timestamp ([] for null)."""
        from .column import micros_to_datetime
        from .types import Row
        cd = self.child.eval(frame)
        if not isinstance(cd.dtype, T.TimestampType) or cd.is_host:
            raise TypeError("window() needs a timestamp column")
        t = cd.values.cpu().numpy().astype(np.int64)
        vm = cd.valid_mask().cpu().numpy()
        # last window start <= t, aligned to startTime modulo slide (Spark TimeWindowing)
        last = t - ((t - self.start) % self.slide)
        nwin = -(-self.dur // self.slide)
        out = []
        for i in range(len(t)):
            if not vm[i]:
                out.append([])
                continue
            ws = []
            for j in range(nwin - 1, -1, -1):  # earliest window first
                s0 = int(last[i]) - j * self.slide
                if s0 + self.dur > t[i]:
                    ws.append(Row(start=micros_to_datetime(s0), end=micros_to_datetime(s0 + self.dur)))
            out.append(ws)
        return out

    def eval(self, frame) -> ColumnData:
        from .builder import column_from_values
        b = self.buckets(frame)
        if self.slide != self.dur:
            raise ValueError("a sliding window() yields several buckets per row: use it in groupBy")
        return column_from_values([w[0] if w else None for w in b], _WINDOW_TYPE, frame._device)


class SessionWindow(Expr):
    """``functions.session_window(timeColumn, gapDuration)``: per group of the other grouping keys,
    events closer than ``gap`` form one session [first event, last event + gap). Sessions can span
    ranks, so the (key, event time) pairs are gathered, swept in time order once, and every rank
    maps its rows to their session (``materialize``, called by GroupedData before aggregating)."""

    def __init__(self, child: Expr, gap_us: int):
        if gap_us <= 0:
            raise ValueError("session_window needs a positive gap duration")
        self.child, self.gap = child, gap_us

    def refs(self):
        return self.child.refs()

    def name(self):
        return "session_window"

    def __str__(self):
        return f"session_window({self.child}, {self.gap}us)"

    def eval(self, frame) -> ColumnData:
        raise ValueError("session_window() is only supported as a groupBy key")

    def materialize(self, frame, other_keys: List[Expr], prior=None):
        """Session column of ``frame``. ``prior`` ({other-key tuple: [(start_us, end_us), ...]}) are
        sessions already held in a streaming state store: this batch's events merge with them (an
        event can extend a session or bridge two). Returns the column, and with ``prior`` also the
        {(key, (start, end)) -> (start', end')} remap of the prior sessions."""
        from .builder import column_from_values
        from .column import micros_to_datetime
        from .dataframe import column_to_python
        from .types import Row
        cd = self.child.eval(frame)
        if not isinstance(cd.dtype, T.TimestampType) or cd.is_host:
            raise TypeError("session_window() needs a timestamp column")
        ts = cd.values.to(torch.int64).cpu().tolist()
        vm = cd.valid_mask().cpu().tolist()
        kv = [column_to_python(k.eval(frame)) for k in other_keys]
        keys = [tuple(_hashable_key(k[i]) for k in kv) for i in range(len(ts))]
        local = sorted({(k, t) for k, t, ok in zip(keys, ts, vm) if ok}, key=lambda x: (repr(x[0]), x[1]))
        spans: Dict[tuple, List[tuple]] = {}
        for part in frame._comm.allgather_object(local):
            for k, t in part:
                spans.setdefault(k, []).append((t, t + self.gap, "e"))
        for k, lst in (prior or {}).items():
            for s_, e_ in lst:
                spans.setdefault(k, []).append((s_, e_, "p"))
        session: Dict[tuple, tuple] = {}
        remap: Dict[tuple, tuple] = {}
        for k, sl in spans.items():
            sl = sorted(set(sl))
            cur = None
            members: List[tuple] = []

            def close():
                for s_, e_, kind in members:
                    if kind == "e":
                        session[(k, s_)] = cur
                    else:
                        remap[(k, (s_, e_))] = cur
            for s_, e_, kind in sl:
                if cur is not None and s_ < cur[1]:
                    cur = (cur[0], max(cur[1], e_))
                    members.append((s_, e_, kind))
                    continue
                if cur is not None:
                    close()
                cur, members = (s_, e_), [(s_, e_, kind)]
            if cur is not None:
                close()
        vals = []
        for k, t, ok in zip(keys, ts, vm):
            if not ok:
                vals.append(None)
                continue
            a, b = session[(k, t)]
            vals.append(Row(start=micros_to_datetime(a), end=micros_to_datetime(b)))
        col = column_from_values(vals, _WINDOW_TYPE, frame._device)
        return col if prior is None else (col, remap)


def materialize_sessions(df, keys: List[Expr], prior=None):
    """Replace a ``session_window`` grouping key by a materialised ``session_window`` column:
    (frame with the column, keys referring to it, prior-session remap or None)."""
    from .column import ColRef
    out_keys, remap = [], None
    for k in keys:
        if isinstance(k, SessionWindow):
            others = [o for o in keys if o is not k]
            r = k.materialize(df, others, prior) if prior is not None else (k.materialize(df, others), None)
            cd, remap = r
            df = df._from_columns(list(df.columns) + ["session_window"], [df._cols[c] for c in df.columns] + [cd])
            out_keys.append(ColRef("session_window"))
        else:
            out_keys.append(k)
    return df, out_keys, remap


def _hashable_key(v):
    if isinstance(v, list):
        return tuple(_hashable_key(x) for x in v)
    if isinstance(v, dict):
        return tuple(sorted((k, _hashable_key(x)) for k, x in v.items()))
    return v


def parse_duration_us(s) -> int:
    """'10 minutes', '1 hour', '30 seconds', '2 days', '500 milliseconds' -> microseconds."""
    if isinstance(s, (int, float)):
        return int(s)
    units = {"microsecond": 1, "millisecond": 1000, "second": 10 ** 6, "minute": 60 * 10 ** 6,
             "hour": 3600 * 10 ** 6, "day": 86400 * 10 ** 6, "week": 7 * 86400 * 10 ** 6}
    toks = str(s).strip().lower().split()
    if len(toks) % 2:
        raise ValueError(f"cannot parse duration {s!r}")
    total = 0
    for q, u in zip(toks[::2], toks[1::2]):
        u = u.rstrip("s")
        if u not in units:
            raise ValueError(f"unknown time unit in {s!r}")
        total += int(float(q) * units[u])
    return total
