"""Column expressions evaluated column-at-a-time on the rank's device.

Covers what the reference builds with pyspark Column objects — ``when(...).
otherwise(...)`` on ``length_of_stay > threshold`` (ref.py:176-177),
``current_timestamp()`` (ref.py:82) — plus the usual arithmetic, comparison,
boolean (SQL three-valued logic), null tests, ``between``, ``isin``, ``cast``
and ``alias``.  An expression evaluates to a :class:`ColumnData` — a torch
tensor (HBM-resident on GPU ranks) or a host numpy array for strings — plus a
validity mask, so nulls propagate exactly like Spark SQL.
"""
from __future__ import annotations

import datetime as _dt
import math
import operator
from dataclasses import dataclass
from typing import Any, Callable, List, Optional, Sequence, Tuple, Union

import numpy as np
import torch

from . import types as T


@dataclass
class ColumnData:
    values: Any                      # torch.Tensor (device) or np.ndarray (host, object/str)
    valid: Any                       # None (all valid) | bool torch.Tensor | bool np.ndarray
    dtype: T.DataType
    # dictionary codes of a host string column (int32, -1 = null; values[i] is the codes[i]-th
    # distinct string, shared objects) — set by ingest, kept by row subsets, used by group-by
    codes: Any = None

    @property
    def is_host(self) -> bool:
        return isinstance(self.values, np.ndarray)

    def __len__(self):
        return int(self.values.shape[0])

    def valid_mask(self):
        n = len(self)
        if self.valid is not None:
            return self.valid
        if self.is_host:
            return np.ones(n, dtype=bool)
        return torch.ones(n, dtype=torch.bool, device=self.values.device)

    def _vals(self):
        """The values without running a deferred check (NanCheckedColumnData overrides this)."""
        return self.values

    def take(self, idx) -> "ColumnData":
        """Row subset by index tensor (device) / array."""
        if self.is_host:
            ii = idx.cpu().numpy() if isinstance(idx, torch.Tensor) else np.asarray(idx)
            return ColumnData(self.values[ii], None if self.valid is None else self.valid[ii], self.dtype,
                              None if self.codes is None else self.codes[ii])
        v = self._vals()
        ti = idx if isinstance(idx, torch.Tensor) else torch.as_tensor(idx, device=v.device)
        ti = ti.to(v.device)
        return self._keep_checks(ColumnData(v[ti], None if self.valid is None else self.valid[ti], self.dtype))

    def mask(self, m) -> "ColumnData":
        if self.is_host:
            mm = m.cpu().numpy() if isinstance(m, torch.Tensor) else np.asarray(m, dtype=bool)
            return ColumnData(self.values[mm], None if self.valid is None else self.valid[mm], self.dtype,
                              None if self.codes is None else self.codes[mm])
        v = self._vals()
        mm = m if isinstance(m, torch.Tensor) else torch.as_tensor(m, device=v.device)
        mm = mm.to(v.device)
        return self._keep_checks(ColumnData(v[mm], None if self.valid is None else self.valid[mm], self.dtype))

    def _keep_checks(self, out: "ColumnData") -> "ColumnData":
        """A row subset inherits a deferred NaN check (VectorAssembler handleInvalid="error")."""
        pend = getattr(self, "nan_pending", None)
        if pend:
            return NanCheckedColumnData(out.values, out.valid, out.dtype, pend, getattr(self, "_comm", None))
        return out


class NanCheckedColumnData(ColumnData):
    """A vector column whose handleInvalid="error" NaN check is deferred to its first reader (Spark's
    VectorAssembler raises when the assembled rows are consumed). ``values`` runs the check
    on this rank's rows before handing them out — any consumer (Binarizer, a second VectorAssembler,
    collect / show / write) raises on a NaN row. ``DataFrame._feature_matrix`` runs the rank-agreed form
    first (fits are collectives), and a consumer whose own pass exposes NaNs (StandardScaler's moments)
    takes the check over through ``_vals()`` and clears it."""

    def __init__(self, values, valid, dtype, msg: str, comm=None):
        self._raw = values
        self.valid = valid
        self.dtype = dtype
        self.codes = None
        self.nan_pending = msg
        # the session communicator: the check's verdict is agreed over every rank — every consumer
        # of a multi-rank frame (collect, toPandas, show, write, a fit) is itself a collective, so all ranks
        # reach it together and fail together, instead of NaN-free ranks blocking in the consumer's
        # collective until its timeout while a NaN rank has raised
        self._comm = comm

    def _vals(self):
        return self._raw

    @property
    def is_host(self) -> bool:
        return False

    def __len__(self):
        return int(self._raw.shape[0])

    @property
    def values(self):
        if self.nan_pending:
            x = self._raw
            bad = False
            if x.numel():
                if x.is_cuda:
                    from ..ops import frame_ops
                    bad = bool(frame_ops.has_nan(x))
                else:
                    bad = bool(torch.isnan(x).any().item())
            comm = self._comm
            if comm is not None and comm.is_distributed:
                bad = comm.max_scalar(1.0 if bad else 0.0) > 0
            if bad:
                raise ValueError(self.nan_pending)
            self.nan_pending = None
        return self._raw

    @values.setter
    def values(self, v):
        self._raw = v


class LazyColumnData(ColumnData):
    """A device column computed on first access of its values (Spark evaluates ``transform`` lazily): a
    Pipeline stage's prediction column that no later stage reads — KMeansModel's cluster ids before a
    LogisticRegression — is never computed. ``thunk()`` returns (values tensor, valid or None); the row
    count is known up front, so schema work, row counts and column projections never trigger it."""

    def __init__(self, thunk, n: int, dtype: T.DataType):
        self._thunk = thunk
        self._n = int(n)
        self.dtype = dtype
        self.codes = None
        self._values = None
        self._valid = None

    def _force(self):
        if self._thunk is not None:
            v, ok = self._thunk()
            self._values, self._valid, self._thunk = v, ok, None

    @property
    def values(self):
        self._force()
        return self._values

    @values.setter
    def values(self, v):
        self._thunk, self._values = None, v

    @property
    def valid(self):
        self._force()
        return self._valid

    @valid.setter
    def valid(self, v):
        self._force()
        self._valid = v

    @property
    def is_host(self) -> bool:
        return False

    @property
    def computed(self) -> bool:
        return self._thunk is None

    def __len__(self):
        return self._n


class DictColumnData(ColumnData):
    """A dictionary-encoded host string column: int32 ``codes`` (-1 = null) into
    ``dictionary`` (distinct strings followed by a trailing None). Row subsets gather the codes only;
    the object array of values is built on first access and cached."""

    def __init__(self, codes, dictionary, valid, dtype):
        self.codes = np.asarray(codes, dtype=np.int32)
        self.dictionary = dictionary
        self.valid = valid
        self.dtype = dtype
        self._values = None

    @property
    def values(self):
        if self._values is None:
            self._values = self.dictionary[self.codes]
        return self._values

    @values.setter
    def values(self, v):
        self._values = v

    @property
    def is_host(self) -> bool:
        return True

    def __len__(self):
        return int(self.codes.shape[0])

    def take(self, idx) -> "ColumnData":
        ii = idx.cpu().numpy() if isinstance(idx, torch.Tensor) else np.asarray(idx)
        return DictColumnData(self.codes[ii], self.dictionary, None if self.valid is None else self.valid[ii],
                              self.dtype)

    def mask(self, m) -> "ColumnData":
        mm = m.cpu().numpy() if isinstance(m, torch.Tensor) else np.asarray(m, dtype=bool)
        return DictColumnData(self.codes[mm], self.dictionary, None if self.valid is None else self.valid[mm],
                              self.dtype)


# ------------------------------------------------------------------------------------------------
# conversion helpers
# ------------------------------------------------------------------------------------------------

def ts_to_micros(v) -> int:
    if isinstance(v, (int, np.integer)):
        return int(v)
    if isinstance(v, np.datetime64):
        return int(v.astype("datetime64[us]").astype(np.int64))
    if isinstance(v, _dt.datetime):
        if v.tzinfo is None:
            v = v.replace(tzinfo=_dt.timezone.utc)
        return int(round(v.timestamp() * 1e6))
    if isinstance(v, _dt.date):
        return ts_to_micros(_dt.datetime(v.year, v.month, v.day))
    if isinstance(v, str):
        s = v.strip().replace("T", " ")
        if s.endswith("Z"):
            s = s[:-1]
        for fmt in ("%Y-%m-%d %H:%M:%S.%f", "%Y-%m-%d %H:%M:%S", "%Y-%m-%d %H:%M", "%Y-%m-%d"):
            try:
                return ts_to_micros(_dt.datetime.strptime(s, fmt))
            except ValueError:
                continue
        raise ValueError(f"cannot parse timestamp {v!r}")
    raise TypeError(f"not a timestamp: {v!r}")


def micros_to_datetime(us: int) -> _dt.datetime:
    return _dt.datetime(1970, 1, 1) + _dt.timedelta(microseconds=int(us))


def _device_of(data: ColumnData, default):
    return data.values.device if not data.is_host else default


def _and_valid(a, b):
    if a is None:
        return b
    if b is None:
        return a
    return a & b


def _to_host(cd: ColumnData) -> ColumnData:
    if cd.is_host:
        return cd
    vals = cd.values.cpu().numpy()
    if isinstance(cd.dtype, T.TimestampType):
        vals = np.array([micros_to_datetime(v) for v in vals], dtype=object)
    valid = None if cd.valid is None else cd.valid.cpu().numpy()
    return ColumnData(vals.astype(object) if vals.dtype != object else vals, valid, cd.dtype)


# ------------------------------------------------------------------------------------------------
# expression tree
# ------------------------------------------------------------------------------------------------

class Expr:
    def eval(self, frame) -> ColumnData:
        raise NotImplementedError

    def name(self) -> str:
        return str(self)

    def refs(self) -> List[str]:
        return []

    def is_aggregate(self) -> bool:
        return False


class ColRef(Expr):
    def __init__(self, name: str):
        self.col = name

    def eval(self, frame) -> ColumnData:
        return frame._column_data(self.col)

    def name(self):
        return self.col

    def refs(self):
        return [self.col]

    def __str__(self):
        return self.col


class Lit(Expr):
    def __init__(self, value):
        self.value = value

    def dtype(self) -> T.DataType:
        v = self.value
        if v is None:
            return T.NullType()
        if isinstance(v, bool):
            return T.BooleanType()
        if isinstance(v, (int, np.integer)):
            return T.IntegerType() if -2**31 <= int(v) < 2**31 else T.LongType()
        if isinstance(v, (float, np.floating)):
            return T.DoubleType()
        if isinstance(v, _dt.datetime):
            return T.TimestampType()
        return T.StringType()

    def eval(self, frame) -> ColumnData:
        n = frame._nrows
        dt = self.dtype()
        if isinstance(dt, (T.StringType, T.NullType)):
            vals = np.empty(n, dtype=object)
            vals[:] = self.value
            valid = None if self.value is not None else np.zeros(n, dtype=bool)
            cd = ColumnData(vals, valid, dt)
            cd.scalar = (self.value,)  # a broadcast literal: consumers may use the one value
            return cd
        v = ts_to_micros(self.value) if isinstance(dt, T.TimestampType) else self.value
        t = torch.full((n,), v, dtype=dt.torch_dtype, device=frame._device)
        return ColumnData(t, None, dt)

    def name(self):
        return str(self.value)

    def __str__(self):
        return str(self.value)


class Alias(Expr):
    def __init__(self, child: Expr, alias: str):
        self.child = child
        self.alias = alias

    def eval(self, frame):
        return self.child.eval(frame)

    def name(self):
        return self.alias

    def refs(self):
        return self.child.refs()

    def is_aggregate(self):
        return self.child.is_aggregate()

    def __str__(self):
        return f"{self.child} AS {self.alias}"


_NUM_RANK = [T.ByteType, T.ShortType, T.IntegerType, T.LongType, T.FloatType, T.DoubleType]


def _promote(a: T.DataType, b: T.DataType) -> T.DataType:
    ra = next((i for i, c in enumerate(_NUM_RANK) if isinstance(a, c)), None)
    rb = next((i for i, c in enumerate(_NUM_RANK) if isinstance(b, c)), None)
    if ra is None or rb is None:
        if isinstance(a, T.TimestampType) or isinstance(b, T.TimestampType):
            return T.TimestampType()
        if isinstance(a, T.BooleanType) and isinstance(b, T.BooleanType):
            return T.BooleanType()
        return T.DoubleType()
    return _NUM_RANK[max(ra, rb)]()


def _coerce_pair(a: ColumnData, b: ColumnData, frame):
    """Make both operands comparable: timestamps vs string literals, strings on host, numeric promotion."""
    if isinstance(a.dtype, T.TimestampType) and b.is_host and isinstance(b.dtype, T.StringType):
        b = _parse_ts_column(b, frame)
    if isinstance(b.dtype, T.TimestampType) and a.is_host and isinstance(a.dtype, T.StringType):
        a = _parse_ts_column(a, frame)
    if a.is_host or b.is_host:
        return _to_host(a), _to_host(b), True
    if isinstance(a.dtype, T.NullType) or isinstance(b.dtype, T.NullType):
        return a, b, False
    pt = _promote(a.dtype, b.dtype)
    if pt.torch_dtype is not None:
        av = a.values.to(pt.torch_dtype) if a.values.dtype != pt.torch_dtype else a.values
        bv = b.values.to(pt.torch_dtype) if b.values.dtype != pt.torch_dtype else b.values
        a = ColumnData(av, a.valid, pt)
        b = ColumnData(bv, b.valid, pt)
    return a, b, False


def _parse_ts_column(cd: ColumnData, frame) -> ColumnData:
    """Host strings -> timestamp micros. Each distinct string is parsed once (a broadcast literal
    such as the reference's BETWEEN bounds, ref.py:126-127, is one parse, not one per row)."""
    dev = frame._device
    n = len(cd)
    lit = getattr(cd, "scalar", None)
    if lit is not None and isinstance(lit[0], str):  # a string literal (BETWEEN bounds): one parse, no row scan
        try:
            us = ts_to_micros(lit[0])
        except (TypeError, ValueError):
            return ColumnData(torch.zeros(n, dtype=torch.int64, device=dev),
                              torch.zeros(n, dtype=torch.bool, device=dev), T.TimestampType())
        return ColumnData(torch.full((n,), us, dtype=torch.int64, device=dev), None, T.TimestampType())
    valid = cd.valid_mask().copy()
    if n and valid.all() and all(v is cd.values[0] for v in (cd.values[0], cd.values[n // 2], cd.values[-1])) \
            and isinstance(cd.values[0], str):
        first = cd.values[0]
        if all(v is first for v in cd.values):  # identity check only: a literal column
            try:
                us = ts_to_micros(first)
            except (TypeError, ValueError):
                return ColumnData(torch.zeros(n, dtype=torch.int64, device=dev),
                                  torch.zeros(n, dtype=torch.bool, device=dev), T.TimestampType())
            return ColumnData(torch.full((n,), us, dtype=torch.int64, device=dev), None, T.TimestampType())
    vals = np.zeros(n, dtype=np.int64)
    cache = {}
    for i, v in enumerate(cd.values):
        if valid[i] and v is not None:
            r = cache.get(v)
            if r is None:
                try:
                    r = ts_to_micros(v)
                except (TypeError, ValueError):
                    r = False
                cache[v] = r
            if r is False:
                valid[i] = False
            else:
                vals[i] = r
        else:
            valid[i] = False
    return ColumnData(torch.as_tensor(vals, device=dev), torch.as_tensor(valid, device=dev), T.TimestampType())


_CMP = {"==": operator.eq, "!=": operator.ne, "<": operator.lt, "<=": operator.le, ">": operator.gt,
        ">=": operator.ge}
_ARITH = {"+": operator.add, "-": operator.sub, "*": operator.mul, "/": operator.truediv, "%": operator.mod}


class BinOp(Expr):
    def __init__(self, op: str, left: Expr, right: Expr):
        self.op, self.left, self.right = op, left, right

    def refs(self):
        return self.left.refs() + self.right.refs()

    def is_aggregate(self):
        return self.left.is_aggregate() or self.right.is_aggregate()

    def __str__(self):
        return f"({self.left} {self.op} {self.right})"

    def eval(self, frame) -> ColumnData:
        a = self.left.eval(frame)
        b = self.right.eval(frame)
        if self.op in ("and", "or"):
            return _logic(self.op, a, b, frame)
        a, b, host = _coerce_pair(a, b, frame)
        valid = _and_valid(a.valid, b.valid)
        if host:
            va, vb = a.values, b.values
            vm = np.ones(len(va), dtype=bool) if valid is None else valid.copy()
            out = np.empty(len(va), dtype=object)
            fn = _CMP.get(self.op) or _ARITH.get(self.op)
            for i in range(len(va)):
                if vm[i] and va[i] is not None and vb[i] is not None:
                    try:
                        out[i] = fn(va[i], vb[i])
                    except Exception:
                        out[i] = None
                        vm[i] = False
                else:
                    vm[i] = False
            if self.op in _CMP:
                dev = frame._device
                return ColumnData(torch.as_tensor(np.where(vm, out, False).astype(bool), device=dev),
                                  torch.as_tensor(vm, device=dev), T.BooleanType())
            return ColumnData(out, vm, T.StringType() if self.op == "+" else T.DoubleType())
        if self.op in _CMP:
            return ColumnData(_CMP[self.op](a.values, b.values), valid, T.BooleanType())
        if self.op == "/":
            av = a.values.to(torch.float64)
            bv = b.values.to(torch.float64)
            zero = bv == 0
            out = av / torch.where(zero, torch.ones_like(bv), bv)
            v2 = ~zero if valid is None else valid & ~zero  # Spark: x / 0 -> null
            return ColumnData(out, v2, T.DoubleType())
        if self.op == "%":
            bv = b.values
            zero = bv == 0
            out = torch.fmod(a.values, torch.where(zero, torch.ones_like(bv), bv))  # Java/Spark remainder
            v2 = ~zero if valid is None else valid & ~zero
            return ColumnData(out, v2, a.dtype)
        return ColumnData(_ARITH[self.op](a.values, b.values), valid, a.dtype)


def _logic(op, a: ColumnData, b: ColumnData, frame) -> ColumnData:
    dev = frame._device
    av = a.values if not a.is_host else torch.as_tensor(np.asarray(a.values, dtype=bool), device=dev)
    bv = b.values if not b.is_host else torch.as_tensor(np.asarray(b.values, dtype=bool), device=dev)
    am = a.valid_mask() if not a.is_host else torch.as_tensor(a.valid_mask(), device=dev)
    bm = b.valid_mask() if not b.is_host else torch.as_tensor(b.valid_mask(), device=dev)
    av = av.to(torch.bool)
    bv = bv.to(torch.bool)
    if op == "and":
        # Kleene: false if either is a known false; null if any null otherwise
        known_false = (am & ~av) | (bm & ~bv)
        val = av & bv & am & bm
        valid = known_false | (am & bm)
        return ColumnData(val & ~known_false, valid, T.BooleanType())
    known_true = (am & av) | (bm & bv)
    valid = known_true | (am & bm)
    return ColumnData(known_true | (av & bv & am & bm), valid, T.BooleanType())


class Unary(Expr):
    def __init__(self, op: str, child: Expr):
        self.op, self.child = op, child

    def refs(self):
        return self.child.refs()

    def is_aggregate(self):
        return self.child.is_aggregate()

    def __str__(self):
        return f"{self.op}({self.child})"

    def eval(self, frame) -> ColumnData:
        c = self.child.eval(frame)
        dev = frame._device
        if self.op in ("isnull", "isnotnull"):
            m = c.valid_mask()
            if c.is_host:
                m = m & np.array([v is not None for v in c.values], dtype=bool)
                m = torch.as_tensor(m, device=dev)
            res = ~m if self.op == "isnull" else m
            return ColumnData(res, None, T.BooleanType())
        if self.op == "isnan":
            if c.is_host or not c.values.is_floating_point():
                return ColumnData(torch.zeros(len(c), dtype=torch.bool, device=dev), c.valid, T.BooleanType())
            return ColumnData(torch.isnan(c.values), c.valid, T.BooleanType())
        if self.op == "not":
            return ColumnData(~c.values.to(torch.bool), c.valid, T.BooleanType())
        if self.op == "neg":
            return ColumnData(-c.values, c.valid, c.dtype)
        fn = _MATH.get(self.op)
        if fn is not None:
            v = c.values.to(torch.float64)
            out = fn(v)
            valid = c.valid
            if self.op in ("log", "sqrt", "log10", "log2"):
                bad = ~torch.isfinite(out)
                valid = ~bad if valid is None else valid & ~bad
            return ColumnData(out, valid, T.DoubleType())
        if self.op in ("upper", "lower", "trim", "length"):
            h = _to_host(c)
            f = {"upper": lambda s: s.upper(), "lower": lambda s: s.lower(), "trim": lambda s: s.strip(),
                 "length": len}[self.op]
            out = np.array([f(str(v)) if v is not None else None for v in h.values], dtype=object)
            if self.op == "length":
                vm = h.valid_mask() & np.array([v is not None for v in out])
                return ColumnData(torch.as_tensor(np.where(vm, out, 0).astype(np.int32), device=dev),
                                  torch.as_tensor(vm, device=dev), T.IntegerType())
            return ColumnData(out, h.valid, T.StringType())
        if self.op in ("year", "month", "dayofmonth", "hour", "minute", "second", "dayofweek"):
            us = c.values.to(torch.int64)
            if isinstance(c.dtype, T.DateType):  # dates hold days since the epoch, not microseconds
                us = us * 86_400_000_000
            if self.op in ("hour", "minute", "second"):
                secs = torch.div(us, 1_000_000, rounding_mode="floor")
                val = {"hour": torch.remainder(torch.div(secs, 3600, rounding_mode="floor"), 24),
                       "minute": torch.remainder(torch.div(secs, 60, rounding_mode="floor"), 60),
                       "second": torch.remainder(secs, 60)}[self.op]
                return ColumnData(val.to(torch.int32), c.valid, T.IntegerType())
            days = torch.div(us, 86_400_000_000, rounding_mode="floor").cpu().numpy()
            dates = days.astype("datetime64[D]")
            if self.op == "year":
                out = dates.astype("datetime64[Y]").astype(np.int64) + 1970
            elif self.op == "month":
                out = dates.astype("datetime64[M]").astype(np.int64) % 12 + 1
            elif self.op == "dayofweek":
                out = (days + 4) % 7 + 1  # 1 = Sunday (Spark)
            else:
                out = (dates - dates.astype("datetime64[M]")).astype(np.int64) + 1
            return ColumnData(torch.as_tensor(out.astype(np.int32), device=dev), c.valid, T.IntegerType())
        raise ValueError(f"unknown unary op {self.op}")


_MATH = {"abs": torch.abs, "sqrt": torch.sqrt, "exp": torch.exp, "log": torch.log, "log10": torch.log10,
         "log2": torch.log2, "floor": torch.floor, "ceil": torch.ceil, "sin": torch.sin, "cos": torch.cos,
         "tanh": torch.tanh, "sigmoid": torch.sigmoid, "signum": torch.sign}


class Cast(Expr):
    def __init__(self, child: Expr, to: T.DataType):
        self.child, self.to = child, to

    def refs(self):
        return self.child.refs()

    def __str__(self):
        return f"CAST({self.child} AS {self.to.simpleString()})"

    def name(self):
        return self.child.name() if isinstance(self.child, ColRef) else str(self)

    def eval(self, frame) -> ColumnData:
        c = self.child.eval(frame)
        dev = frame._device
        to = self.to
        if isinstance(to, T.StringType):
            if isinstance(c.dtype, (T.DateType, T.TimestampType)) and not c.is_host:
                # device dates / timestamps hold days / microseconds: format the calendar values
                from .dataframe import column_to_python
                vals = column_to_python(c)
                return ColumnData(np.array([None if v is None else _fmt_datetime(v) for v in vals], dtype=object),
                                  None if c.valid is None else c.valid_mask().cpu().numpy(), to)
            h = _to_host(c)
            return ColumnData(np.array([None if v is None else _fmt(v) for v in h.values], dtype=object),
                              h.valid, to)
        if isinstance(to, T.DateType) and (c.is_host or isinstance(c.dtype, T.TimestampType)):
            ts = _parse_ts_column(c, frame) if c.is_host else c
            days = torch.div(ts.values, 86_400_000_000, rounding_mode="floor").to(torch.int32)
            return ColumnData(days, ts.valid, to)
        if isinstance(to, T.TimestampType) and not c.is_host and isinstance(c.dtype, T.DateType):
            return ColumnData(c.values.to(torch.int64) * 86_400_000_000, c.valid, to)
        if c.is_host:
            if isinstance(to, T.TimestampType):
                return _parse_ts_column(c, frame)
            vm = c.valid_mask().copy()
            out = np.zeros(len(c), dtype=np.float64)
            for i, v in enumerate(c.values):
                if not vm[i] or v is None:
                    vm[i] = False
                    continue
                try:
                    out[i] = float(v)
                except (TypeError, ValueError):
                    vm[i] = False
            t = torch.as_tensor(out, device=dev)
            if T.is_integral(to):
                t = torch.trunc(t)
            return ColumnData(t.to(to.torch_dtype), torch.as_tensor(vm, device=dev), to)
        v = c.values
        if T.is_integral(to) and v.is_floating_point():
            v = torch.trunc(v)
        return ColumnData(v.to(to.torch_dtype), c.valid, to)


def _fmt_datetime(v):
    """Spark's string form: 2024-05-17 for dates, 2024-05-17 10:20:30[.fraction without trailing zeros]."""
    import datetime as _dt
    if isinstance(v, _dt.datetime):
        out = v.strftime("%Y-%m-%d %H:%M:%S")
        return out + ("." + f"{v.microsecond:06d}".rstrip("0") if v.microsecond else "")
    if isinstance(v, _dt.date):
        return f"{v.year:04d}-{v.month:02d}-{v.day:02d}"
    return str(v)


def _fmt(v):
    if isinstance(v, float):
        return repr(v)
    if isinstance(v, bool):
        return "true" if v else "false"
    return str(v)


class When(Expr):
    def __init__(self, branches: List[Tuple[Expr, Expr]], otherwise: Optional[Expr] = None):
        self.branches = branches
        self.other = otherwise

    def refs(self):
        out = []
        for c, v in self.branches:
            out += c.refs() + v.refs()
        return out + (self.other.refs() if self.other else [])

    def __str__(self):
        s = "CASE " + " ".join(f"WHEN {c} THEN {v}" for c, v in self.branches)
        return s + (f" ELSE {self.other}" if self.other is not None else "") + " END"

    def eval(self, frame) -> ColumnData:
        dev = frame._device
        n = frame._nrows
        vals = [v.eval(frame) for _, v in self.branches]
        other = self.other.eval(frame) if self.other is not None else None
        all_cols = vals + ([other] if other is not None else [])
        typed = [x for x in all_cols if not isinstance(x.dtype, T.NullType)]
        if typed and not any(x.is_host for x in typed):
            # NULL literal branches (when(c, None)) take the device type of the others
            def _dev(x):
                if not isinstance(x.dtype, T.NullType):
                    return x
                return ColumnData(torch.zeros(n, dtype=torch.float64, device=dev),
                                  torch.zeros(n, dtype=torch.bool, device=dev), x.dtype)
            vals = [_dev(v) for v in vals]
            other = None if other is None else _dev(other)
            all_cols = vals + ([other] if other is not None else [])
        if any(x.is_host for x in all_cols):
            out = np.empty(n, dtype=object)
            vm = np.zeros(n, dtype=bool)
            done = np.zeros(n, dtype=bool)
            for (cond, _), v in zip(self.branches, vals):
                cd = cond.eval(frame)
                hit = (cd.values & cd.valid_mask()).cpu().numpy() & ~done
                hv = _to_host(v)
                out[hit] = hv.values[hit]
                vm[hit] = hv.valid_mask()[hit]
                done |= hit
            if other is not None:
                ho = _to_host(other)
                rest = ~done
                out[rest] = ho.values[rest]
                vm[rest] = ho.valid_mask()[rest]
            return ColumnData(out, vm, T.StringType())
        dt = vals[0].dtype
        for x in all_cols[1:]:
            if not isinstance(x.dtype, T.NullType):
                dt = _promote(dt, x.dtype) if not isinstance(dt, T.NullType) else x.dtype
        tdt = dt.torch_dtype or torch.float64
        if other is not None:
            out = other.values.to(tdt).clone()
            vm = other.valid_mask().clone()
        else:
            out = torch.zeros(n, dtype=tdt, device=dev)
            vm = torch.zeros(n, dtype=torch.bool, device=dev)
        # apply branches in reverse so the first matching branch wins
        for (cond, _), v in reversed(list(zip(self.branches, vals))):
            cd = cond.eval(frame)
            hit = cd.values.to(torch.bool) & cd.valid_mask()
            out = torch.where(hit, v.values.to(tdt), out)
            vm = torch.where(hit, v.valid_mask(), vm)
        return ColumnData(out, vm, dt)


class Func(Expr):
    """Generic function node evaluated by a callable (frame, [ColumnData]) -> ColumnData."""

    def __init__(self, fname: str, args: Sequence[Expr], impl: Callable):
        self.fname = fname
        self.args = list(args)
        self.impl = impl

    def refs(self):
        out = []
        for a in self.args:
            out += a.refs()
        return out

    def is_aggregate(self):
        return any(a.is_aggregate() for a in self.args)

    def __str__(self):
        label = getattr(self, "label", None)
        if label is not None:
            return label
        parts = [str(a) for a in self.args] + [str(p) for p in getattr(self, "params", ())]
        return f"{self.fname}({', '.join(parts)})"

    def eval(self, frame):
        return self.impl(frame, [a.eval(frame) for a in self.args])


class AggExpr(Expr):
    """Aggregate (count/sum/avg/min/max/stddev/variance/count_distinct) — evaluated by groupBy/agg."""

    def __init__(self, fn: str, child: Optional[Expr], distinct: bool = False, ignore_nulls: bool = False):
        self.fn, self.child, self.distinct = fn, child, distinct
        self.ignore_nulls = bool(ignore_nulls)  # first / last: Spark's ignoreNulls (default False)

    def is_aggregate(self):
        return True

    def refs(self):
        return self.child.refs() if self.child is not None else []

    def __str__(self):
        inner = "*" if self.child is None else str(self.child)
        if self.fn == "count" and self.child is not None and isinstance(self.child, Lit):
            inner = str(self.child.value)
        return f"{self.fn}({'DISTINCT ' if self.distinct else ''}{inner})"

    def eval(self, frame):
        raise ValueError(f"aggregate {self} used outside of an aggregation")


class SortOrder:
    def __init__(self, expr: Expr, ascending: bool = True, nulls_first: Optional[bool] = None):
        self.expr, self.ascending = expr, ascending
        self.nulls_first = ascending if nulls_first is None else nulls_first


# ------------------------------------------------------------------------------------------------
# user-facing Column
# ------------------------------------------------------------------------------------------------

def _expr(x) -> Expr:
    if isinstance(x, Column):
        return x._expr
    if isinstance(x, Expr):
        return x
    return Lit(x)


class Column:
    def __init__(self, expr: Union[Expr, str]):
        self._expr = ColRef(expr) if isinstance(expr, str) else expr

    # arithmetic
    def __add__(self, o): return Column(BinOp("+", self._expr, _expr(o)))
    def __radd__(self, o): return Column(BinOp("+", _expr(o), self._expr))
    def __sub__(self, o): return Column(BinOp("-", self._expr, _expr(o)))
    def __rsub__(self, o): return Column(BinOp("-", _expr(o), self._expr))
    def __mul__(self, o): return Column(BinOp("*", self._expr, _expr(o)))
    def __rmul__(self, o): return Column(BinOp("*", _expr(o), self._expr))
    def __truediv__(self, o): return Column(BinOp("/", self._expr, _expr(o)))
    def __rtruediv__(self, o): return Column(BinOp("/", _expr(o), self._expr))
    def __mod__(self, o): return Column(BinOp("%", self._expr, _expr(o)))
    def __neg__(self): return Column(Unary("neg", self._expr))

    # comparison
    def __eq__(self, o): return Column(BinOp("==", self._expr, _expr(o)))  # type: ignore[override]
    def __ne__(self, o): return Column(BinOp("!=", self._expr, _expr(o)))  # type: ignore[override]
    def __lt__(self, o): return Column(BinOp("<", self._expr, _expr(o)))
    def __le__(self, o): return Column(BinOp("<=", self._expr, _expr(o)))
    def __gt__(self, o): return Column(BinOp(">", self._expr, _expr(o)))
    def __ge__(self, o): return Column(BinOp(">=", self._expr, _expr(o)))

    # boolean
    def __and__(self, o): return Column(BinOp("and", self._expr, _expr(o)))
    def __or__(self, o): return Column(BinOp("or", self._expr, _expr(o)))
    def __invert__(self): return Column(Unary("not", self._expr))
    __hash__ = None  # type: ignore[assignment]

    def __bool__(self):
        raise ValueError("Cannot convert column into bool: use '&' for 'and', '|' for 'or', '~' for 'not'")

    def isNull(self): return Column(Unary("isnull", self._expr))
    def isNotNull(self): return Column(Unary("isnotnull", self._expr))
    def isnan(self): return Column(Unary("isnan", self._expr))

    def between(self, lower, upper):
        return Column(BinOp("and", BinOp(">=", self._expr, _expr(lower)), BinOp("<=", self._expr, _expr(upper))))

    def isin(self, *values):
        if len(values) == 1 and isinstance(values[0], (list, tuple, set)):
            values = tuple(values[0])
        e: Optional[Expr] = None
        for v in values:
            t = BinOp("==", self._expr, _expr(v))
            e = t if e is None else BinOp("or", e, t)
        return Column(e if e is not None else Lit(False))

    def cast(self, to):
        return Column(Cast(self._expr, T.parse_type(to)))

    astype = cast

    def alias(self, *names):
        # several names: the columns of a multi-column generator (posexplode -> pos, col)
        return Column(Alias(self._expr, names[0] if len(names) == 1 else tuple(names)))

    name = alias

    def when(self, cond, value):
        if not isinstance(self._expr, When) or self._expr.other is not None:
            raise ValueError("when() can only be applied on a Column previously generated by when()")
        return Column(When(self._expr.branches + [(_expr(cond), _expr(value))]))

    def otherwise(self, value):
        if not isinstance(self._expr, When):
            raise ValueError("otherwise() can only be applied on a Column previously generated by when()")
        return Column(When(self._expr.branches, _expr(value)))

    def over(self, window):
        """Window function / aggregate evaluated over ``window`` (``sql.window.WindowSpec``)."""
        from .window import over
        return over(self, window)

    def asc(self): return SortOrder(self._expr, True)
    def desc(self): return SortOrder(self._expr, False)
    def asc_nulls_first(self): return SortOrder(self._expr, True, True)
    def asc_nulls_last(self): return SortOrder(self._expr, True, False)
    def desc_nulls_first(self): return SortOrder(self._expr, False, True)
    def desc_nulls_last(self): return SortOrder(self._expr, False, False)

    # ---- pyspark Column methods built on sql.functions (string predicates / regex / substr run
    # once per distinct value on dictionary-encoded columns, see functions._host_map)
    def __pow__(self, o):
        from .functions import pow as _pow
        return _pow(self, o)

    def __rpow__(self, o):
        from .functions import pow as _pow
        return _pow(Column(_expr(o)), self)

    def __rmod__(self, o): return Column(BinOp("%", _expr(o), self._expr))

    def contains(self, other):
        from .functions_tail import contains
        return contains(self, other)

    def startswith(self, other):
        from .functions_tail import startswith
        return startswith(self, other)

    def endswith(self, other):
        from .functions_tail import endswith
        return endswith(self, other)

    def like(self, pattern: str):
        from .functions_tail import like
        return like(self, pattern)

    def ilike(self, pattern: str):
        from .functions_tail import ilike
        return ilike(self, pattern)

    def rlike(self, pattern: str):
        from .functions_tail import regexp_like
        return regexp_like(self, pattern)

    def substr(self, startPos, length):
        from .functions import substring
        if isinstance(startPos, Column) or isinstance(length, Column):
            from .functions_tail import substr
            return substr(self, startPos, length)
        return substring(self, int(startPos), int(length))

    def getItem(self, key):
        from .sqlparse import Subscript
        return Column(Subscript(self._expr, _expr(key)))

    def getField(self, name: str):
        from .sqlparse import GetField
        return Column(GetField(self._expr, name))

    def __getitem__(self, k):
        if isinstance(k, slice):
            if k.step is not None:
                raise ValueError("slice with step is not supported")
            return self.substr(k.start, k.stop)
        from .functions_tail import _ItemOrField
        return Column(_ItemOrField(self._expr, k))

    def eqNullSafe(self, other):
        from .functions_tail import equal_null
        return equal_null(self, other if isinstance(other, Column) else Column(Lit(other)))

    def bitwiseAND(self, other):
        from .functions_tail import _bitwise
        return _bitwise("&", self, other)

    def bitwiseOR(self, other):
        from .functions_tail import _bitwise
        return _bitwise("|", self, other)

    def bitwiseXOR(self, other):
        from .functions_tail import _bitwise
        return _bitwise("^", self, other)

    def isNaN(self): return Column(Unary("isnan", self._expr))

    def try_cast(self, to):
        """Cast with null for values that do not convert (the engine's casts already do)."""
        return self.cast(to)

    def withField(self, fieldName: str, col):
        from .functions_tail import _with_field
        return _with_field(self, fieldName, col)

    def dropFields(self, *fieldNames: str):
        from .functions_tail import _drop_fields
        return _drop_fields(self, fieldNames)

    def __getattr__(self, item):
        if item.startswith("_"):
            raise AttributeError(item)
        raise AttributeError(f"Column has no attribute {item!r}")

    def __repr__(self):
        return f"Column<'{self._expr}'>"

    def __str__(self):
        return str(self._expr)
