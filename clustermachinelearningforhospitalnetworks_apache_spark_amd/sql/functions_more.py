"""More pyspark.sql.functions: statistical aggregates computed on the device, math / date / string
scalars, array and struct builders, and the explode family of generators.

Statistical aggregates (``skewness``, ``kurtosis``, ``corr``, ``covar_pop``/``covar_samp``, ``product``,
``count_if``, ``bool_and``/``bool_or``, ``max_by``/``min_by``) are custom aggregates of the frame's
aggregation operator (group.aggregate): each group's partial is a few device reductions over its
rows (central moments up to the 4th order, co-moments) and partials merge across ranks with the
pairwise update formulas (Chan et al. / Pébay), so results do not depend on the GPU count.
``median`` / ``percentile`` / ``mode`` / ``sum_distinct`` need the values themselves and gather them.
"""
from __future__ import annotations

import builtins
import datetime as _dt
import hashlib
import math
import zlib
from typing import List, Optional

import numpy as np
import torch

from . import types as T
from .column import AggExpr, Column, ColumnData, Expr, Func, _to_host
from .functions import ColumnOrName, UserDefinedFunction, _c, _host_map


# ------------------------------------------------------------------------------------------ aggregates

class _DevAgg(AggExpr):
    """Custom aggregate over one or more numeric columns: rows where every input is non-null and not
    NaN contribute. Subclasses implement ``_local(vals)`` (device tensors of the group's rows ->
    picklable partial), ``_merge(parts)`` and ``_type``."""
    custom = True
    _type: T.DataType = T.DoubleType()

    def __init__(self, fn: str, children: List[Expr], label: Optional[str] = None):
        super().__init__(fn, children[0] if children else None)
        self.children = children
        self.label = label

    def refs(self):
        return [r for c in self.children for r in c.refs()]

    def __str__(self):
        return self.label or f"{self.fn}({', '.join(str(c) for c in self.children)})"

    def prepare(self, df):
        out = []
        for c in self.children:
            cd = c.eval(df)
            if cd.is_host:
                raise TypeError(f"{self.fn}: column {c} is not numeric")
            v = cd.values
            v = v.to(torch.float64) if v.dtype != torch.bool else v.to(torch.float64)
            ok = cd.valid_mask().to(v.device) & ~torch.isnan(v)
            out.append((v, ok))
        return out

    def partial(self, vals, rows):
        if not vals:
            return self._local([])
        dev = vals[0][0].device
        idx = torch.as_tensor(rows, dtype=torch.int64, device=dev)
        ok = torch.ones(idx.numel(), dtype=torch.bool, device=dev)
        for _, m in vals:
            ok &= m[idx]
        sel = idx[ok]
        return self._local([v[sel] for v, _ in vals])

    def merge(self, parts):
        return self._merge(parts)

    def result_type(self):
        return self._type


def _moments4(x: torch.Tensor):
    n = int(x.numel())
    if n == 0:
        return (0, 0.0, 0.0, 0.0, 0.0)
    m = x.mean()
    d = x - m
    d2 = d * d
    return (n, float(m), float(d2.sum()), float((d2 * d).sum()), float((d2 * d2).sum()))


def _merge_moments4(parts):
    n, mean, m2, m3, m4 = 0, 0.0, 0.0, 0.0, 0.0
    for nb, mb, m2b, m3b, m4b in parts:
        if nb == 0:
            continue
        if n == 0:
            n, mean, m2, m3, m4 = nb, mb, m2b, m3b, m4b
            continue
        na = n
        nn = na + nb
        delta = mb - mean
        d_n = delta / nn
        m4 = (m4 + m4b + delta * d_n ** 3 * na * nb * (na * na - na * nb + nb * nb)
              + 6.0 * d_n * d_n * (na * na * m2b + nb * nb * m2) + 4.0 * d_n * (na * m3b - nb * m3))
        m3 = m3 + m3b + delta * d_n * d_n * na * nb * (na - nb) + 3.0 * d_n * (na * m2b - nb * m2)
        m2 = m2 + m2b + delta * d_n * na * nb
        mean = mean + d_n * nb
        n = nn
    return n, mean, m2, m3, m4


class _Skewness(_DevAgg):
    def _local(self, v):
        return _moments4(v[0]) if v else (0, 0.0, 0.0, 0.0, 0.0)

    def _merge(self, parts):
        n, _, m2, m3, _ = _merge_moments4(parts)
        if n == 0 or m2 == 0.0:
            return None
        return math.sqrt(n) * m3 / (m2 ** 1.5)


class _Kurtosis(_Skewness):
    def _merge(self, parts):
        n, _, m2, _, m4 = _merge_moments4(parts)
        if n == 0 or m2 == 0.0:
            return None
        return n * m4 / (m2 * m2) - 3.0


class _CoMoment(_DevAgg):
    """corr / covar_pop / covar_samp: partial (n, mean_x, mean_y, C_xy, M2_x, M2_y)."""

    def _local(self, v):
        x, y = v
        n = int(x.numel())
        if n == 0:
            return (0, 0.0, 0.0, 0.0, 0.0, 0.0)
        mx, my = x.mean(), y.mean()
        dx, dy = x - mx, y - my
        return (n, float(mx), float(my), float((dx * dy).sum()), float((dx * dx).sum()), float((dy * dy).sum()))

    def _merge(self, parts):
        n, mx, my, c, m2x, m2y = 0, 0.0, 0.0, 0.0, 0.0, 0.0
        for nb, mxb, myb, cb, m2xb, m2yb in parts:
            if nb == 0:
                continue
            nn = n + nb
            dx, dy = mxb - mx, myb - my
            c += cb + dx * dy * n * nb / nn
            m2x += m2xb + dx * dx * n * nb / nn
            m2y += m2yb + dy * dy * n * nb / nn
            mx += dx * nb / nn
            my += dy * nb / nn
            n = nn
        if self.fn == "covar_pop":
            return c / n if n else None
        if self.fn == "covar_samp":
            return c / (n - 1) if n > 1 else None
        if n < 2:
            return None
        den = math.sqrt(m2x * m2y)
        return c / den if den > 0 else float("nan")


class _Product(_DevAgg):
    def _local(self, v):
        x = v[0]
        return (int(x.numel()), float(torch.prod(x)) if x.numel() else 1.0)

    def _merge(self, parts):
        n = builtins.sum(p[0] for p in parts)
        out = 1.0
        for p in parts:
            out *= p[1]
        return out if n else None


class _CountIf(_DevAgg):
    _type = T.LongType()

    def _local(self, v):
        return int((v[0] != 0).sum()) if v else 0

    def _merge(self, parts):
        return int(builtins.sum(parts))


class _BoolAgg(_DevAgg):
    _type = T.BooleanType()

    def _local(self, v):
        x = v[0]
        if x.numel() == 0:
            return None
        return bool((x != 0).all()) if self.fn == "bool_and" else bool((x != 0).any())

    def _merge(self, parts):
        vals = [p for p in parts if p is not None]
        if not vals:
            return None
        return builtins.all(vals) if self.fn == "bool_and" else builtins.any(vals)


class _ByAgg(_DevAgg):
    """max_by(x, ord) / min_by(x, ord): the x of the row with the largest / smallest ord."""

    def prepare(self, df):
        xcd = self.children[0].eval(df)
        ocd = self.children[1].eval(df)
        o = ocd.values.to(torch.float64)
        ok = ocd.valid_mask().to(o.device) & ~torch.isnan(o)
        return [(xcd, None), (o, ok)]

    def partial(self, vals, rows):
        (xcd, _), (o, ok) = vals
        idx = torch.as_tensor(rows, dtype=torch.int64, device=o.device)
        idx = idx[ok[idx]]
        if idx.numel() == 0:
            return None
        j = int(idx[torch.argmax(o[idx]) if self.fn == "max_by" else torch.argmin(o[idx])])
        from .dataframe import column_to_python
        return (float(o[j]), column_to_python(xcd.take(torch.tensor([j], device=o.device)))[0])

    def _merge(self, parts):
        vals = [p for p in parts if p is not None]
        if not vals:
            return None
        best = (builtins.max if self.fn == "max_by" else builtins.min)(vals, key=lambda p: p[0])
        return best[1]

    def result_type(self):
        return self._xtype

    def bind_type(self, t):
        self._xtype = t
        return self


class _ValuesAgg(_DevAgg):
    """Aggregates that need the values: median / percentile (linear interpolation between order
    statistics, Spark's ``percentile``), mode (most frequent, ties -> smallest), sum_distinct."""

    def __init__(self, fn, children, arg=None, label=None):
        if label is None and arg is not None:  # distinct names for different percentages
            label = f"{fn}({', '.join(str(c) for c in children)}, {arg})"
        super().__init__(fn, children, label)
        self.arg = arg
        if fn == "percentile" and isinstance(arg, (list, tuple)):
            self._type = T.ArrayType(T.DoubleType())

    def _local(self, v):
        x = v[0]
        if self.fn in ("mode", "sum_distinct"):
            u, cnt = torch.unique(x, return_counts=True)
            return (u.cpu().numpy(), cnt.cpu().numpy())
        return x.cpu().numpy()

    def _merge(self, parts):
        if self.fn in ("mode", "sum_distinct"):
            tot = {}
            for u, cnt in parts:
                for a, b in zip(u.tolist(), cnt.tolist()):
                    tot[a] = tot.get(a, 0) + b
            if not tot:
                return None
            if self.fn == "sum_distinct":
                return float(builtins.sum(tot))
            best = builtins.max(tot.values())
            return builtins.min(a for a, b in tot.items() if b == best)
        allv = np.concatenate(parts) if parts else np.zeros(0)
        if allv.size == 0:
            return None
        srt = np.sort(allv)

        def one(p):
            if not 0.0 <= p <= 1.0:
                raise ValueError("percentile must be in [0, 1]")
            pos = p * (srt.size - 1)
            lo = int(math.floor(pos))
            hi = builtins.min(lo + 1, srt.size - 1)
            return float(srt[lo] + (pos - lo) * (srt[hi] - srt[lo]))
        p = 0.5 if self.fn == "median" else self.arg
        return [one(float(q)) for q in p] if isinstance(p, (list, tuple)) else one(float(p))


def skewness(c: ColumnOrName) -> Column:
    return Column(_Skewness("skewness", [_c(c)]))


def kurtosis(c: ColumnOrName) -> Column:
    return Column(_Kurtosis("kurtosis", [_c(c)]))


def corr(c1: ColumnOrName, c2: ColumnOrName) -> Column:
    return Column(_CoMoment("corr", [_c(c1), _c(c2)]))


def covar_pop(c1: ColumnOrName, c2: ColumnOrName) -> Column:
    return Column(_CoMoment("covar_pop", [_c(c1), _c(c2)]))


def covar_samp(c1: ColumnOrName, c2: ColumnOrName) -> Column:
    return Column(_CoMoment("covar_samp", [_c(c1), _c(c2)]))


def product(c: ColumnOrName) -> Column:
    return Column(_Product("product", [_c(c)]))


def count_if(c: ColumnOrName) -> Column:
    return Column(_CountIf("count_if", [_c(c)]))


def bool_and(c: ColumnOrName) -> Column:
    return Column(_BoolAgg("bool_and", [_c(c)]))


def bool_or(c: ColumnOrName) -> Column:
    return Column(_BoolAgg("bool_or", [_c(c)]))


every = bool_and
some = bool_or
any = bool_or  # noqa: A001 (pyspark name)


class _TypedBy(_ByAgg):
    """max_by / min_by with the x column's type resolved at prepare time."""

    def prepare(self, df):
        out = super().prepare(df)
        self._xtype = out[0][0].dtype
        return out


def max_by(c: ColumnOrName, ord: ColumnOrName) -> Column:  # noqa: A002
    return Column(_TypedBy("max_by", [_c(c), _c(ord)]))


def min_by(c: ColumnOrName, ord: ColumnOrName) -> Column:  # noqa: A002
    return Column(_TypedBy("min_by", [_c(c), _c(ord)]))


def median(c: ColumnOrName) -> Column:
    return Column(_ValuesAgg("median", [_c(c)]))


def percentile(c: ColumnOrName, percentage, frequency=1) -> Column:
    if frequency != 1:
        raise NotImplementedError("percentile: frequency != 1")
    return Column(_ValuesAgg("percentile", [_c(c)], percentage))


def mode(c: ColumnOrName) -> Column:
    return Column(_ValuesAgg("mode", [_c(c)]))


def sum_distinct(c: ColumnOrName) -> Column:
    return Column(_ValuesAgg("sum_distinct", [_c(c)]))


sumDistinct = sum_distinct


# ------------------------------------------------------------------------------------------ math

def _dev2(name, fn, a, b) -> Column:
    def impl(frame, args):
        x, y = args
        vx, vy = x.values.to(torch.float64), y.values.to(torch.float64)
        valid = None
        if x.valid is not None or y.valid is not None:
            valid = x.valid_mask() & y.valid_mask()
        return ColumnData(fn(vx, vy), valid, T.DoubleType())
    ea = _c(a) if isinstance(a, (str, Column)) else _c(Column(__import__(
        "clustermachinelearningforhospitalnetworks_apache_spark_amd.sql.column", fromlist=["Lit"]).Lit(a)))
    eb = _c(b) if isinstance(b, (str, Column)) else _c(Column(__import__(
        "clustermachinelearningforhospitalnetworks_apache_spark_amd.sql.column", fromlist=["Lit"]).Lit(b)))
    return Column(Func(name, [ea, eb], impl))


def pow(a, b) -> Column:  # noqa: A001
    return _dev2("POWER", torch.pow, a, b)


power = pow


def atan2(a, b) -> Column:
    return _dev2("ATAN2", torch.atan2, a, b)


def hypot(a, b) -> Column:
    return _dev2("HYPOT", torch.hypot, a, b)


def nanvl(a: ColumnOrName, b: ColumnOrName) -> Column:
    return _dev2("nanvl", lambda x, y: torch.where(torch.isnan(x), y, x), a, b)


def _dev1(name, fn):
    def f(c: ColumnOrName) -> Column:
        def impl(frame, args):
            a = args[0]
            out = fn(a.values.to(torch.float64))
            bad = ~torch.isfinite(out) & torch.isfinite(a.values.to(torch.float64))
            valid = a.valid
            if name in ("log1p", "acos", "asin", "cbrt") and bool(bad.any()):
                valid = ~bad if valid is None else valid & ~bad
            return ColumnData(out, valid, T.DoubleType())
        return Column(Func(f"{name}({c if isinstance(c, str) else _c(c)})", [_c(c)], impl))
    f.__name__ = name
    return f


tan = _dev1("tan", torch.tan)
asin = _dev1("asin", torch.asin)
acos = _dev1("acos", torch.acos)
atan = _dev1("atan", torch.atan)
sinh = _dev1("sinh", torch.sinh)
cosh = _dev1("cosh", torch.cosh)
cbrt = _dev1("cbrt", lambda v: torch.sign(v) * torch.abs(v).pow(1.0 / 3.0))
log1p = _dev1("log1p", torch.log1p)
expm1 = _dev1("expm1", torch.expm1)
rint = _dev1("rint", torch.round)
degrees = _dev1("degrees", torch.rad2deg)
radians = _dev1("radians", torch.deg2rad)


def bround(c: ColumnOrName, scale: int = 0) -> Column:
    """Round HALF_EVEN to ``scale`` decimals (torch.round is half-to-even)."""
    def impl(frame, args):
        a = args[0]
        f = 10.0 ** scale
        return ColumnData(torch.round(a.values.to(torch.float64) * f) / f, a.valid, T.DoubleType())
    return Column(Func(f"bround({scale})", [_c(c)], impl))


def isnotnull(c: ColumnOrName) -> Column:
    from .column import Unary
    return Column(Unary("isnotnull", _c(c)))


def asc(c: ColumnOrName):
    return Column(_c(c)).asc()


def desc(c: ColumnOrName):
    return Column(_c(c)).desc()


# ------------------------------------------------------------------------------------------ dates

def _to_date(v):
    if v is None:
        return None
    if isinstance(v, _dt.datetime):
        return v.date()
    return v


def dayofyear(c: ColumnOrName) -> Column:
    return _host_map("dayofyear", [c], lambda t: _to_date(t).timetuple().tm_yday, T.IntegerType())


def weekofyear(c: ColumnOrName) -> Column:
    return _host_map("weekofyear", [c], lambda t: _to_date(t).isocalendar()[1], T.IntegerType())


def quarter(c: ColumnOrName) -> Column:
    return _host_map("quarter", [c], lambda t: (_to_date(t).month - 1) // 3 + 1, T.IntegerType())


def _month_end(d: _dt.date) -> _dt.date:
    nxt = _dt.date(d.year + (d.month == 12), d.month % 12 + 1, 1)
    return nxt - _dt.timedelta(days=1)


def last_day(c: ColumnOrName) -> Column:
    return _host_map("last_day", [c], lambda t: _month_end(_to_date(t)), T.DateType())


def _add_months(d: _dt.date, m: int) -> _dt.date:
    y, mo = divmod(d.month - 1 + m, 12)
    first = _dt.date(d.year + y, mo + 1, 1)
    end = _month_end(first)
    # Spark 3 (LocalDate.plusMonths): keep the day of month, clamped to the target month's length; the
    # Spark 2 rule mapping a month's last day to the target's last day was dropped in 3.0
    day = builtins.min(d.day, end.day)
    return first.replace(day=day)


def add_months(c: ColumnOrName, months: int) -> Column:
    return _host_map("add_months", [c], lambda t: _add_months(_to_date(t), int(months)), T.DateType())


def months_between(end: ColumnOrName, start: ColumnOrName, roundOff: bool = True) -> Column:
    """Spark: whole months when both days are the same or both are month ends, else the fractional
    difference on a 31-day month (time of day included), rounded to 8 digits by default."""
    def f(a, b):
        ta = a if isinstance(a, _dt.datetime) else _dt.datetime.combine(a, _dt.time())
        tb = b if isinstance(b, _dt.datetime) else _dt.datetime.combine(b, _dt.time())
        months = (ta.year - tb.year) * 12 + (ta.month - tb.month)
        if ta.day == tb.day or (ta.date() == _month_end(ta.date()) and tb.date() == _month_end(tb.date())):
            return float(months)
        sa = (ta.day - 1) * 86400 + ta.hour * 3600 + ta.minute * 60 + ta.second
        sb = (tb.day - 1) * 86400 + tb.hour * 3600 + tb.minute * 60 + tb.second
        v = months + (sa - sb) / (31.0 * 86400)
        return builtins.round(v, 8) if roundOff else v
    return _host_map("months_between", [end, start], f, T.DoubleType())


_TRUNC = {"year": "year", "yyyy": "year", "yy": "year", "quarter": "quarter", "month": "month", "mon": "month",
          "mm": "month", "week": "week", "day": "day", "dd": "day", "hour": "hour", "minute": "minute",
          "second": "second"}


def _trunc_dt(t: _dt.datetime, unit: str) -> _dt.datetime:
    u = _TRUNC.get(unit.lower())
    if u is None:
        raise ValueError(f"unsupported truncation unit {unit!r}")
    if u == "year":
        return t.replace(month=1, day=1, hour=0, minute=0, second=0, microsecond=0)
    if u == "quarter":
        return t.replace(month=(t.month - 1) // 3 * 3 + 1, day=1, hour=0, minute=0, second=0, microsecond=0)
    if u == "month":
        return t.replace(day=1, hour=0, minute=0, second=0, microsecond=0)
    if u == "week":
        d = t - _dt.timedelta(days=t.weekday())
        return d.replace(hour=0, minute=0, second=0, microsecond=0)
    if u == "day":
        return t.replace(hour=0, minute=0, second=0, microsecond=0)
    if u == "hour":
        return t.replace(minute=0, second=0, microsecond=0)
    if u == "minute":
        return t.replace(second=0, microsecond=0)
    return t.replace(microsecond=0)


def date_trunc(fmt: str, c: ColumnOrName) -> Column:
    return _host_map("date_trunc", [c], lambda t: _trunc_dt(t if isinstance(t, _dt.datetime) else
                                                            _dt.datetime.combine(t, _dt.time()), fmt),
                     T.TimestampType())


def trunc(c: ColumnOrName, fmt: str) -> Column:
    return _host_map("trunc", [c], lambda t: _trunc_dt(t if isinstance(t, _dt.datetime) else
                                                       _dt.datetime.combine(t, _dt.time()), fmt).date(),
                     T.DateType())


# ------------------------------------------------------------------------------------------ strings

def initcap(c: ColumnOrName) -> Column:
    return _host_map("initcap", [c], lambda s: " ".join(w[:1].upper() + w[1:].lower() for w in str(s).split(" ")),
                     T.StringType())


def ltrim(c: ColumnOrName) -> Column:
    return _host_map("ltrim", [c], lambda s: str(s).lstrip(" "), T.StringType())


def rtrim(c: ColumnOrName) -> Column:
    return _host_map("rtrim", [c], lambda s: str(s).rstrip(" "), T.StringType())


def reverse(c: ColumnOrName) -> Column:
    return _host_map("reverse", [c], lambda s: s[::-1] if isinstance(s, list) else str(s)[::-1], T.StringType())


def instr(c: ColumnOrName, substr: str) -> Column:
    return _host_map("instr", [c], lambda s: str(s).find(substr) + 1, T.IntegerType())


def locate(substr: str, c: ColumnOrName, pos: int = 1) -> Column:
    return _host_map("locate", [c], lambda s: (str(s).find(substr, pos - 1) + 1) if pos >= 1 else 0,
                     T.IntegerType())


def translate(c: ColumnOrName, matching: str, replace: str) -> Column:
    table = {ord(a): (replace[i] if i < len(replace) else None) for i, a in enumerate(matching)}
    return _host_map("translate", [c], lambda s: str(s).translate(table), T.StringType())


def repeat(c: ColumnOrName, n: int) -> Column:
    return _host_map("repeat", [c], lambda s: str(s) * int(n), T.StringType())


def md5(c: ColumnOrName) -> Column:
    return _host_map("md5", [c], lambda s: hashlib.md5(_bytes(s)).hexdigest(), T.StringType())


def sha1(c: ColumnOrName) -> Column:
    return _host_map("sha1", [c], lambda s: hashlib.sha1(_bytes(s)).hexdigest(), T.StringType())


def sha2(c: ColumnOrName, numBits: int) -> Column:
    algo = {0: "sha256", 224: "sha224", 256: "sha256", 384: "sha384", 512: "sha512"}.get(int(numBits))
    if algo is None:
        raise ValueError("sha2: numBits must be 224, 256, 384, 512 or 0")
    return _host_map("sha2", [c], lambda s: hashlib.new(algo, _bytes(s)).hexdigest(), T.StringType())


def crc32(c: ColumnOrName) -> Column:
    return _host_map("crc32", [c], lambda s: zlib.crc32(_bytes(s)) & 0xFFFFFFFF, T.LongType())


def _bytes(s) -> bytes:
    return s if isinstance(s, (bytes, bytearray)) else str(s).encode("utf-8")


# ------------------------------------------------------------------------------------------ arrays / structs

def _elem_type(cd: ColumnData) -> T.DataType:
    return cd.dtype.elementType if isinstance(cd.dtype, T.ArrayType) else T.StringType()


def array(*cols) -> Column:
    if len(cols) == 1 and isinstance(cols[0], (list, tuple)):
        cols = tuple(cols[0])

    def impl(frame, args):
        from .dataframe import column_to_python
        pys = [column_to_python(a) for a in args]
        et = args[0].dtype if args else T.StringType()
        if builtins.all(T.is_numeric(a.dtype) for a in args) and args:
            et = T.DoubleType() if builtins.any(not T.is_integral(a.dtype) for a in args) else args[0].dtype
        out = np.empty(frame._nrows, dtype=object)
        for i in range(frame._nrows):
            out[i] = [p[i] for p in pys]
        return ColumnData(out, None, T.ArrayType(et))
    return Column(Func("array", [_c(c) for c in cols], impl))


def struct(*cols) -> Column:
    if len(cols) == 1 and isinstance(cols[0], (list, tuple)):
        cols = tuple(cols[0])
    exprs = [_c(c) for c in cols]

    def impl(frame, args):
        from .dataframe import column_to_python
        from .types import Row
        names = [e.name() for e in exprs]
        pys = [column_to_python(a) for a in args]
        out = np.empty(frame._nrows, dtype=object)
        for i in range(frame._nrows):
            out[i] = Row(**{n: p[i] for n, p in zip(names, pys)})
        st = T.StructType([T.StructField(n, a.dtype, True) for n, a in zip(names, args)])
        return ColumnData(out, None, st)
    return Column(Func("struct", exprs, impl))


def _arr_map(name, c, fn, rt_fn):
    def impl(frame, args):
        a = _to_host(args[0])
        vm = a.valid_mask() & np.array([v is not None for v in a.values], dtype=bool)
        vals = [fn(v) if ok else None for v, ok in zip(a.values, vm)]
        rt = rt_fn(args[0])
        from .builder import column_from_values
        return column_from_values(vals, rt, frame._device)
    return Column(Func(name, [_c(c)], impl))


def size(c: ColumnOrName) -> Column:
    """Array / map length; -1 for null (Spark's legacy sizeOfNull default)."""
    def impl(frame, args):
        a = _to_host(args[0])
        vm = a.valid_mask()
        out = np.array([len(v) if (ok and v is not None) else -1 for v, ok in zip(a.values, vm)], dtype=np.int32)
        return ColumnData(torch.as_tensor(out, device=frame._device), None, T.IntegerType())
    return Column(Func("size", [_c(c)], impl))


def array_contains(c: ColumnOrName, value) -> Column:
    return _arr_map("array_contains", c, lambda v: value in v, lambda cd: T.BooleanType())


def element_at(c: ColumnOrName, extraction) -> Column:
    def f(v):
        if isinstance(v, dict):
            return v.get(extraction)
        i = int(extraction)
        if i == 0:
            raise ValueError("element_at: SQL array indices start at 1")
        j = i - 1 if i > 0 else len(v) + i
        return v[j] if 0 <= j < len(v) else None
    return _arr_map("element_at", c, f, lambda cd: cd.dtype.valueType if isinstance(cd.dtype, T.MapType)
                    else _elem_type(cd))


def sort_array(c: ColumnOrName, asc: bool = True) -> Column:  # noqa: A002
    def f(v):
        nn = sorted(x for x in v if x is not None)
        nulls = [None] * (len(v) - len(nn))
        return nulls + nn if asc else nn[::-1] + nulls
    return _arr_map("sort_array", c, f, lambda cd: cd.dtype)


def array_distinct(c: ColumnOrName) -> Column:
    return _arr_map("array_distinct", c, lambda v: list(dict.fromkeys(v)), lambda cd: cd.dtype)


def array_max(c: ColumnOrName) -> Column:
    return _arr_map("array_max", c, lambda v: builtins.max((x for x in v if x is not None), default=None),
                    _elem_type)


def array_min(c: ColumnOrName) -> Column:
    return _arr_map("array_min", c, lambda v: builtins.min((x for x in v if x is not None), default=None),
                    _elem_type)


def array_join(c: ColumnOrName, delimiter: str, null_replacement: Optional[str] = None) -> Column:
    def f(v):
        return delimiter.join(str(x) if x is not None else null_replacement for x in v
                              if x is not None or null_replacement is not None)
    return _arr_map("array_join", c, f, lambda cd: T.StringType())


# ------------------------------------------------------------------------------------------ generators

class Generator(Expr):
    """explode / explode_outer / posexplode / posexplode_outer of an array or map column. Only valid
    as a top-level ``select`` / ``withColumn`` item (DataFrame._select_generator expands the rows)."""

    def __init__(self, fn: str, child: Expr):
        self.fn, self.child = fn, child
        self.names: Optional[List[str]] = None

    def refs(self):
        return self.child.refs()

    def __str__(self):
        return f"{self.fn}({self.child})"

    def name(self):
        return "col"

    def eval(self, frame):
        raise ValueError(f"{self.fn} is only allowed as a top-level select / withColumn expression")

    def output_names(self, is_map: bool) -> List[str]:
        base = ["key", "value"] if is_map else ["col"]
        return (["pos"] if self.fn.startswith("pos") else []) + base


def explode(c: ColumnOrName) -> Column:
    return Column(Generator("explode", _c(c)))


def explode_outer(c: ColumnOrName) -> Column:
    return Column(Generator("explode_outer", _c(c)))


def posexplode(c: ColumnOrName) -> Column:
    return Column(Generator("posexplode", _c(c)))


def posexplode_outer(c: ColumnOrName) -> Column:
    return Column(Generator("posexplode_outer", _c(c)))


def _generator_plan(ge: "Generator", cd: ColumnData):
    """(output names, output types, value -> list of output tuples) for one generator."""
    outer = ge.fn.endswith("_outer")
    if ge.fn == "json_tuple":
        import json as _json
        fields = list(getattr(ge, "fields", []))

        def expand_json(v):
            try:
                obj = _json.loads(v) if v is not None else None
            except (ValueError, TypeError):
                obj = None
            if not isinstance(obj, dict):
                return [tuple(None for _ in fields)]
            out = []
            for f in fields:
                x = obj.get(f)
                out.append(None if x is None else (x if isinstance(x, str) else _json.dumps(x, separators=(",", ":"))))
            return [tuple(out)]
        return [f"c{i}" for i in range(len(fields))], [T.StringType()] * len(fields), expand_json
    if ge.fn.startswith("inline"):
        st = cd.dtype.elementType if isinstance(cd.dtype, T.ArrayType) else None
        if not isinstance(st, T.StructType):
            raise TypeError("inline() needs an array of structs")
        width = len(st.fields)

        def expand_inline(v):
            items = [tuple(e) if e is not None else tuple([None] * width) for e in (v or [])]
            return items if items else ([tuple([None] * width)] if outer else [])
        return [f.name for f in st.fields], [f.dataType for f in st.fields], expand_inline
    is_map = isinstance(cd.dtype, T.MapType)
    pos = ge.fn.startswith("pos")
    names = ge.output_names(is_map)
    if is_map:
        types = ([T.IntegerType()] if pos else []) + [cd.dtype.keyType, cd.dtype.valueType]
    else:
        types = ([T.IntegerType()] if pos else []) + [cd.dtype.elementType if isinstance(cd.dtype, T.ArrayType)
                                                      else T.StringType()]

    def expand(v):
        items = list(v.items()) if (is_map and v is not None) else (list(v) if v is not None else [])
        if not items:
            if not outer:
                return []
            return [((None,) if pos else ()) + ((None, None) if is_map else (None,))]
        return [((p,) if pos else ()) + (tuple(e) if is_map else (e,)) for p, e in enumerate(items)]
    return names, types, expand


def select_with_generator(df, exprs: List[Expr]):
    """``df.select(...)`` where one item is a Generator: each input row is repeated once per element
    (``_outer``: at least once, with null elements for null / empty inputs); the other items are
    evaluated on the repeated rows. Row ids are renumbered globally (a fresh dense id space)."""
    from .builder import column_from_values
    from .column import Alias
    from .dataframe import column_to_python
    gi = [i for i, e in enumerate(exprs) if isinstance(e.child if isinstance(e, Alias) else e, Generator)]
    if len(gi) != 1:
        raise ValueError("only one generator (explode / posexplode) is allowed per select clause")
    gi = gi[0]
    ge = exprs[gi]
    alias = None
    if isinstance(ge, Alias):
        alias, ge = ge.alias, ge.child
    cd = ge.child.eval(df)
    vals = column_to_python(cd)
    gnames, gtypes, expand = _generator_plan(ge, cd)
    rep, rows = [], []
    for i, v in enumerate(vals):
        for r in expand(v):
            rep.append(i)
            rows.append(r)
    idx = torch.as_tensor(rep, dtype=torch.int64, device=df._device)
    base = df._take_rows(idx)
    names, datas = [], []
    if alias is not None:
        al = alias if isinstance(alias, (list, tuple)) else [alias]
        if len(al) != len(gnames):
            raise ValueError(f"{ge.fn} produces {len(gnames)} columns, got aliases {al}")
        gnames = list(al)
    for j, e in enumerate(exprs):
        if j != gi:
            names.append(e.name())
            datas.append(e.eval(base))
            continue
        for k, (gn, gt) in enumerate(zip(gnames, gtypes)):
            names.append(gn)
            datas.append(column_from_values([r[k] for r in rows], gt, df._device))
    out = base._from_columns(names, datas)
    counts = df._comm.allgather_object(len(rep))
    off = builtins.sum(counts[:df._comm.rank])
    out._row_ids = torch.arange(off, off + len(rep), dtype=torch.int64, device=df._device)
    return out


__all__ = ["skewness", "kurtosis", "corr", "covar_pop", "covar_samp", "product", "count_if", "bool_and", "bool_or",
           "every", "some", "max_by", "min_by", "median", "percentile", "mode", "sum_distinct", "sumDistinct", "pow",
           "power", "atan2", "hypot", "nanvl", "tan", "asin", "acos", "atan", "sinh", "cosh", "cbrt", "log1p", "expm1",
           "rint", "degrees", "radians", "bround", "isnotnull", "asc", "desc", "dayofyear", "weekofyear", "quarter",
           "last_day", "add_months", "months_between", "date_trunc", "trunc", "initcap", "ltrim", "rtrim", "reverse",
           "instr", "locate", "translate", "repeat", "md5", "sha1", "sha2", "crc32", "array", "struct", "size",
           "array_contains", "element_at", "sort_array", "array_distinct", "array_max", "array_min", "array_join",
           "explode", "explode_outer", "posexplode", "posexplode_outer"]
