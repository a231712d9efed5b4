"""Spark 3.4/3.5 additions to pyspark.sql.functions: regression aggregates (``regr_*``), string
aggregation, bitwise aggregates, discrete percentiles, the ``try_*`` family, regex / URL / string
helpers, null-safe comparisons and date aliases.

``regr_*`` aggregates reuse the co-moment partials of ``corr`` (n, means, C_xy, M2_x, M2_y merged
pairwise across groups and ranks), so they run as device reductions like the other statistical
aggregates; ``string_agg`` / ``listagg`` and the bitwise aggregates gather the group's values.
"""
from __future__ import annotations

import builtins
import datetime as _dt
import getpass
import math
import re
import urllib.parse
import uuid as _uuid
from typing import Any, List, Optional

import numpy as np
import torch

from . import types as T
from .column import AggExpr, Column, ColumnData, Func, Lit
from .functions import ColumnOrName, UserDefinedFunction, _c, _host_map
from .functions_more import _CoMoment, _ValuesAgg


def _e(c):
    from .functions_extra import _e as e
    return e(c)


# ------------------------------------------------------------------------------------------ aggregates

class _Regr(_CoMoment):
    """regr_*(y, x) over rows where both are non-null: partial (n, mean_y, mean_x, C, M2_y, M2_x)."""

    def result_type(self):
        return T.LongType() if self.fn == "regr_count" else T.DoubleType()

    def _merge(self, parts):
        n, my, mx, c, m2y, m2x = 0, 0.0, 0.0, 0.0, 0.0, 0.0
        for nb, myb, mxb, cb, m2yb, m2xb in parts:
            if nb == 0:
                continue
            nn = n + nb
            dy, dx = myb - my, mxb - mx
            c += cb + dx * dy * n * nb / nn
            m2x += m2xb + dx * dx * n * nb / nn
            m2y += m2yb + dy * dy * n * nb / nn
            mx += dx * nb / nn
            my += dy * nb / nn
            n = nn
        fn = self.fn
        if fn == "regr_count":
            return n
        if n == 0:
            return None
        if fn == "regr_avgx":
            return mx
        if fn == "regr_avgy":
            return my
        if fn == "regr_sxx":
            return m2x
        if fn == "regr_syy":
            return m2y
        if fn == "regr_sxy":
            return c
        if m2x == 0.0:
            return None
        slope = c / m2x
        if fn == "regr_slope":
            return slope
        if fn == "regr_intercept":
            return my - slope * mx
        if m2y == 0.0:  # regr_r2
            return 1.0
        return c * c / (m2x * m2y)


def _regr(fn):
    def f(y: ColumnOrName, x: ColumnOrName) -> Column:
        return Column(_Regr(fn, [_c(y), _c(x)]))
    f.__name__ = fn
    return f


regr_count = _regr("regr_count")
regr_avgx = _regr("regr_avgx")
regr_avgy = _regr("regr_avgy")
regr_sxx = _regr("regr_sxx")
regr_syy = _regr("regr_syy")
regr_sxy = _regr("regr_sxy")
regr_slope = _regr("regr_slope")
regr_intercept = _regr("regr_intercept")
regr_r2 = _regr("regr_r2")


class _PercentileDisc(_ValuesAgg):
    """percentile_disc: the smallest value whose cumulative fraction reaches p."""

    def _merge(self, parts):
        allv = np.concatenate(parts) if parts else np.zeros(0)
        if allv.size == 0:
            return None
        srt = np.sort(allv)
        p = float(self.arg)
        if not 0.0 <= p <= 1.0:
            raise ValueError("percentile must be in [0, 1]")
        k = builtins.max(int(math.ceil(p * srt.size)) - 1, 0)
        return float(srt[k])


def percentile_cont(c: ColumnOrName, percentage: float = 0.5) -> Column:
    return Column(_ValuesAgg("percentile", [_c(c)], float(percentage),
                             label=f"percentile_cont({c if isinstance(c, str) else _c(c)}, {percentage})"))


def percentile_disc(c: ColumnOrName, percentage: float = 0.5) -> Column:
    return Column(_PercentileDisc("percentile_disc", [_c(c)], float(percentage)))


def approx_percentile(c: ColumnOrName, percentage, accuracy: int = 10000) -> Column:
    from .functions import percentile_approx
    return percentile_approx(c, percentage, accuracy)


class _HostValuesAgg(AggExpr):
    """Aggregates over the group's raw values (strings, 64-bit integers): string_agg, bit_*."""
    custom = True

    def __init__(self, fn: str, child, arg=None, rtype: Optional[T.DataType] = None):
        super().__init__(fn, child)
        self.arg = arg
        self._rtype = rtype

    def __str__(self):
        return f"{self.fn}({self.child})"

    def prepare(self, df):
        from .dataframe import column_to_python
        cd = self.child.eval(df)
        if self._rtype is None:
            self._rtype = cd.dtype
        return column_to_python(cd)

    def partial(self, vals, rows):
        return [vals[i] for i in rows if vals[i] is not None]

    def merge(self, parts):
        vals = [v for p in parts for v in p]
        if not vals:
            return None
        if self.fn == "string_agg":
            return (self.arg or "").join(str(v) for v in vals)
        out = int(vals[0])
        for v in vals[1:]:
            out = out & int(v) if self.fn == "bit_and" else (out | int(v) if self.fn == "bit_or" else out ^ int(v))
        return out

    def result_type(self):
        return T.StringType() if self.fn == "string_agg" else (self._rtype or T.LongType())


def string_agg(c: ColumnOrName, delimiter: Optional[str] = None) -> Column:
    """Concatenation of the group's non-null values (row order of the shards) with ``delimiter``."""
    d = delimiter
    if isinstance(d, Column):
        d = d._expr.value if isinstance(d._expr, Lit) else str(d._expr)
    return Column(_HostValuesAgg("string_agg", _c(c), d))


listagg = string_agg


def bit_and(c: ColumnOrName) -> Column:
    return Column(_HostValuesAgg("bit_and", _c(c)))


def bit_or(c: ColumnOrName) -> Column:
    return Column(_HostValuesAgg("bit_or", _c(c)))


def bit_xor(c: ColumnOrName) -> Column:
    return Column(_HostValuesAgg("bit_xor", _c(c)))


def array_agg(c: ColumnOrName) -> Column:
    from .functions import collect_list
    return collect_list(c)


def any_value(c: ColumnOrName, ignoreNulls: bool = False) -> Column:
    from .functions import first
    return first(c, ignorenulls=bool(ignoreNulls))


def first_value(c: ColumnOrName, ignoreNulls: bool = False) -> Column:
    from .functions import first
    return first(c, ignorenulls=bool(ignoreNulls))


def last_value(c: ColumnOrName, ignoreNulls: bool = False) -> Column:
    from .functions import last
    return last(c, ignorenulls=bool(ignoreNulls))


def std(c: ColumnOrName) -> Column:
    from .functions import stddev
    return stddev(c)


def try_sum(c: ColumnOrName) -> Column:
    """Spark's try_sum: sum, but null (instead of a wrapped 64-bit value) when an integral total
    leaves the LongType range. Floating sums behave as sum (overflow to ±Infinity)."""
    from .column import AggExpr
    return Column(AggExpr("try_sum", _c(c)))


def try_avg(c: ColumnOrName) -> Column:
    """Spark's try_avg. Average accumulates integral and floating input in a double (Average's
    sumDataType), which cannot overflow to an error; only decimal/interval sums differ from avg, and
    decimals here are averaged in f64 too — so the value is avg's, named try_avg."""
    from .column import AggExpr
    return Column(AggExpr("try_avg", _c(c)))


# ------------------------------------------------------------------------------------------ try_* / null-safe

def _int_op(name, op, ovf):
    def f(left: ColumnOrName, right: ColumnOrName) -> Column:
        def impl(frame, args):
            a, b = args
            valid = a.valid_mask() & b.valid_mask()
            if T.is_integral(a.dtype) and T.is_integral(b.dtype):
                x, y = a.values.to(torch.int64), b.values.to(torch.int64)
                s = op(x, y)
                bad = ovf(x, y, s)
                long_out = isinstance(a.dtype, T.LongType) or isinstance(b.dtype, T.LongType)
                if not long_out:
                    bad = bad | (s > 2 ** 31 - 1) | (s < -2 ** 31)
                    s = s.to(torch.int32)
                return ColumnData(s, valid & ~bad, T.LongType() if long_out else T.IntegerType())
            return ColumnData(op(a.values.to(torch.float64), b.values.to(torch.float64)), valid, T.DoubleType())
        return Column(Func(name, [_e(left), _e(right)], impl))
    f.__name__ = name
    return f


try_subtract = _int_op("try_subtract", lambda x, y: x - y,
                       lambda x, y, s: ((x >= 0) != (y >= 0)) & ((s >= 0) != (x >= 0)))


def _mul_ovf(x, y, s):
    nz = x != 0
    back = torch.where(nz, torch.div(s, torch.where(nz, x, torch.ones_like(x)), rounding_mode="trunc"), y)
    return nz & (back != y)


try_multiply = _int_op("try_multiply", lambda x, y: x * y, _mul_ovf)


def try_element_at(c: ColumnOrName, extraction) -> Column:
    def f(v):
        if isinstance(v, dict):
            return v.get(extraction)
        i = int(extraction)
        j = i - 1 if i > 0 else len(v) + i
        return v[j] if i != 0 and 0 <= j < len(v) else None
    from .functions_extra import _arr_fn, _elem
    return _arr_fn("try_element_at", [c], f, lambda args: args[0].dtype.valueType
                   if isinstance(args[0].dtype, T.MapType) else _elem(args[0]))


def try_to_number(c: ColumnOrName, format: str) -> Column:  # noqa: A002
    from .functions_extra import to_number
    return to_number(c, format)


def try_to_timestamp(c: ColumnOrName, format: Optional[str] = None) -> Column:
    from .functions import to_timestamp
    return to_timestamp(c, format)


def to_binary(c: ColumnOrName, format: Optional[str] = None) -> Column:  # noqa: A002
    fmt = (format or "hex").lower() if not isinstance(format, Column) else "hex"

    def f(s):
        s = str(s)
        try:
            if fmt == "hex":
                return bytes.fromhex(s if len(s) % 2 == 0 else "0" + s)
            if fmt in ("utf-8", "utf8"):
                return s.encode("utf-8")
            if fmt == "base64":
                import base64
                return base64.b64decode(s)
        except ValueError:
            return None
        raise ValueError(f"to_binary: unsupported format {format!r}")
    return _host_map("to_binary", [c], f, T.BinaryType(), params=[fmt])


def try_to_binary(c: ColumnOrName, format: Optional[str] = None) -> Column:  # noqa: A002
    return to_binary(c, format)


def equal_null(col1: ColumnOrName, col2: ColumnOrName) -> Column:
    """Null-safe equality: true when both are null, false when one is."""
    def impl(frame, args):
        from .dataframe import column_to_python
        a, b = column_to_python(args[0]), column_to_python(args[1])
        out = [(x is None and y is None) or (x is not None and y is not None and x == y) for x, y in zip(a, b)]
        return ColumnData(torch.as_tensor(out, dtype=torch.bool, device=frame._device), None, T.BooleanType())
    return Column(Func("equal_null", [_e(col1), _e(col2)], impl))


def zeroifnull(c: ColumnOrName) -> Column:
    from .functions import coalesce, lit
    return coalesce(Column(_e(c)), lit(0))


def nullifzero(c: ColumnOrName) -> Column:
    from .functions_extra import nullif
    return nullif(c, Column(Lit(0)))


# ------------------------------------------------------------------------------------------ math

def pmod(dividend, divisor) -> Column:
    def impl(frame, args):
        a, b = args
        valid = a.valid_mask() & b.valid_mask() & (b.values != 0)
        if T.is_integral(a.dtype) and T.is_integral(b.dtype):
            x, y = a.values.to(torch.int64), b.values.to(torch.int64)
            ys = torch.where(y != 0, y, torch.ones_like(y))
            r = torch.remainder(x, ys.abs())
            return ColumnData(r.to(a.values.dtype if a.values.dtype == b.values.dtype else torch.int64), valid,
                              a.dtype if type(a.dtype) is type(b.dtype) else T.LongType())
        x, y = a.values.to(torch.float64), b.values.to(torch.float64)
        r = torch.fmod(x, y)
        r = torch.where(r < 0, torch.fmod(r + y.abs(), y.abs()), r)
        return ColumnData(r, valid, T.DoubleType())
    return Column(Func("pmod", [_e(dividend), _e(divisor)], impl))


def positive(c: ColumnOrName) -> Column:
    return Column(_e(c))


def negative(c: ColumnOrName) -> Column:
    return -Column(_e(c))


def e() -> Column:
    from .functions import lit
    return lit(math.e)


def pi() -> Column:
    from .functions import lit
    return lit(math.pi)


def log(arg1, arg2=None) -> Column:
    """log(x) natural logarithm, or log(base, x)."""
    def impl(frame, args):
        if len(args) == 1:
            a = args[0]
            v = a.values.to(torch.float64)
            return ColumnData(torch.log(v), a.valid_mask() & (v > 0), T.DoubleType())
        b, a = args
        vb, va = b.values.to(torch.float64), a.values.to(torch.float64)
        return ColumnData(torch.log(va) / torch.log(vb), a.valid_mask() & b.valid_mask() & (va > 0) & (vb > 0),
                          T.DoubleType())
    cols = [_e(arg1)] if arg2 is None else [_e(arg1), _e(arg2)]
    return Column(Func("LOG" if arg2 is not None else "ln", cols, impl))


def width_bucket(v: ColumnOrName, min: ColumnOrName, max: ColumnOrName, numBucket) -> Column:  # noqa: A002
    def f(x, lo, hi, nb):
        nb = int(nb)
        if nb <= 0 or lo == hi:
            return None
        if lo < hi:
            if x < lo:
                return 0
            if x >= hi:
                return nb + 1
            return int(math.floor((x - lo) / (hi - lo) * nb)) + 1
        if x > lo:
            return 0
        if x <= hi:
            return nb + 1
        return int(math.floor((lo - x) / (lo - hi) * nb)) + 1
    return _host_map("width_bucket", [v, min, max, numBucket if isinstance(numBucket, (str, Column))
                                      else Column(Lit(numBucket))], f, T.LongType())


def bit_count(c: ColumnOrName) -> Column:
    return _host_map("bit_count", [c], lambda v: builtins.bin(int(v) & ((1 << 64) - 1)).count("1") if not isinstance(
        v, bool) else int(v), T.IntegerType())


def bit_get(c: ColumnOrName, pos) -> Column:
    return _host_map("bit_get", [c, pos if isinstance(pos, (str, Column)) else Column(Lit(pos))],
                     lambda v, p: (int(v) >> int(p)) & 1, T.ByteType())


getbit = bit_get


def sign(c: ColumnOrName) -> Column:
    from .functions import signum
    return signum(c)


def ceiling(c: ColumnOrName) -> Column:
    from .functions import ceil
    return ceil(c)


def random(seed: int = 0) -> Column:
    from .functions import rand
    return rand(seed)


# ------------------------------------------------------------------------------------------ strings

def _rx(pattern):
    p = pattern._expr.value if isinstance(pattern, Column) and isinstance(pattern._expr, Lit) else pattern
    return re.compile(str(p))


def regexp_like(s: ColumnOrName, regexp) -> Column:
    rx = _rx(regexp)
    return _host_map("regexp_like", [s], lambda v: rx.search(str(v)) is not None, T.BooleanType())


rlike = regexp_like
regexp = regexp_like


def regexp_count(s: ColumnOrName, regexp) -> Column:
    rx = _rx(regexp)
    return _host_map("regexp_count", [s], lambda v: len(rx.findall(str(v))), T.IntegerType())


def regexp_substr(s: ColumnOrName, regexp) -> Column:
    rx = _rx(regexp)

    def f(v):
        m = rx.search(str(v))
        return m.group(0) if m else None
    return _host_map("regexp_substr", [s], f, T.StringType())


def regexp_instr(s: ColumnOrName, regexp, idx=None) -> Column:
    rx = _rx(regexp)

    def f(v):
        m = rx.search(str(v))
        return m.start() + 1 if m else 0
    return _host_map("regexp_instr", [s], f, T.IntegerType())


def split_part(src: ColumnOrName, delimiter, partNum) -> Column:
    def f(s, d, k):
        s, d, k = str(s), str(d), int(k)
        if k == 0:
            raise ValueError("split_part: the index 0 is invalid")
        parts = s.split(d) if d else [s]
        j = k - 1 if k > 0 else len(parts) + k
        return parts[j] if 0 <= j < len(parts) else ""
    lit_ = (lambda x: x if isinstance(x, (str, Column)) and not isinstance(x, str) else Column(Lit(x)))
    return _host_map("split_part", [src, lit_(delimiter), lit_(partNum)], f, T.StringType())


def _bool2(name, fn):
    def f(left: ColumnOrName, right) -> Column:
        r = right if isinstance(right, Column) else Column(Lit(right))
        return _host_map(name, [left, r], lambda a, b: fn(str(a), str(b)), T.BooleanType())
    f.__name__ = name
    return f


startswith = _bool2("startswith", lambda a, b: a.startswith(b))
endswith = _bool2("endswith", lambda a, b: a.endswith(b))
contains = _bool2("contains", lambda a, b: b in a)


def left(s: ColumnOrName, length) -> Column:
    n = length._expr.value if isinstance(length, Column) else int(length)
    return _host_map("left", [s], lambda v: str(v)[:builtins.max(int(n), 0)], T.StringType())


def right(s: ColumnOrName, length) -> Column:
    n = length._expr.value if isinstance(length, Column) else int(length)
    return _host_map("right", [s], lambda v: str(v)[-int(n):] if int(n) > 0 else "", T.StringType())


def btrim(s: ColumnOrName, trim: Optional[Any] = None) -> Column:
    chars = None if trim is None else (trim._expr.value if isinstance(trim, Column) else str(trim))
    return _host_map("btrim", [s], lambda v: str(v).strip(chars if chars is not None else " "), T.StringType())


def lcase(c: ColumnOrName) -> Column:
    from .functions import lower
    return lower(c)


def ucase(c: ColumnOrName) -> Column:
    from .functions import upper
    return upper(c)


def char(c: ColumnOrName) -> Column:
    return _host_map("char", [c], lambda v: builtins.chr(int(v) % 256) if int(v) >= 0 else "", T.StringType())


chr = char  # noqa: A001


def mask(c: ColumnOrName, upperChar="X", lowerChar="x", digitChar="n", otherChar=None) -> Column:
    def val(x):
        return x._expr.value if isinstance(x, Column) else x
    up, lo, dg, ot = val(upperChar), val(lowerChar), val(digitChar), val(otherChar)

    def f(s):
        out = []
        for ch in str(s):
            if ch.isupper() and up is not None:
                out.append(up)
            elif ch.islower() and lo is not None:
                out.append(lo)
            elif ch.isdigit() and dg is not None:
                out.append(dg)
            elif not ch.isalnum() and ot is not None:
                out.append(ot)
            else:
                out.append(ch)
        return "".join(out)
    return _host_map("mask", [c], f, T.StringType(), params=[up, lo, dg, ot])


def url_encode(c: ColumnOrName) -> Column:
    return _host_map("url_encode", [c], lambda s: urllib.parse.quote_plus(str(s)), T.StringType())


def url_decode(c: ColumnOrName) -> Column:
    return _host_map("url_decode", [c], lambda s: urllib.parse.unquote_plus(str(s)), T.StringType())


def parse_url(url: ColumnOrName, partToExtract, key=None) -> Column:
    part = (partToExtract._expr.value if isinstance(partToExtract, Column) else str(partToExtract)).upper()
    k = key._expr.value if isinstance(key, Column) else key

    def f(u):
        p = urllib.parse.urlsplit(str(u))
        if part == "HOST":
            return p.hostname
        if part == "PATH":
            return p.path
        if part == "QUERY":
            if k is None:
                return p.query or None
            vals = urllib.parse.parse_qs(p.query, keep_blank_values=True).get(k)
            return vals[0] if vals else None
        if part == "REF":
            return p.fragment or None
        if part == "PROTOCOL":
            return p.scheme or None
        if part == "FILE":
            return p.path + ("?" + p.query if p.query else "")
        if part == "AUTHORITY":
            return p.netloc or None
        if part == "USERINFO":
            return p.netloc.rsplit("@", 1)[0] if "@" in p.netloc else None
        return None
    return _host_map("parse_url", [url], f, T.StringType(), params=[part] + ([k] if k is not None else []))


def to_char(c: ColumnOrName, format) -> Column:  # noqa: A002
    """Numbers with a Spark number format ('9', '0', ',', '.', '$', 'S', 'MI'); dates and timestamps
    with a datetime pattern."""
    fmt = format._expr.value if isinstance(format, Column) else str(format)

    def f(v):
        if isinstance(v, (_dt.date, _dt.datetime)):
            from .datetimefmt import formatter
            return formatter(fmt)(v)
        dec = len(fmt.split(".", 1)[1].rstrip("MIS")) if "." in fmt else 0
        body = f"{builtins.abs(float(v)):,.{dec}f}" if "," in fmt else f"{builtins.abs(float(v)):.{dec}f}"
        sign_ = "-" if float(v) < 0 else ""
        if "$" in fmt:
            body = "$" + body
        if fmt.endswith("MI"):
            return body + ("-" if sign_ else " ")
        if fmt.startswith("S"):
            return ("-" if sign_ else "+") + body
        return sign_ + body
    return _host_map("to_char", [c], f, T.StringType(), params=[fmt])


to_varchar = to_char


# ------------------------------------------------------------------------------------------ dates / misc

def convert_timezone(sourceTz, targetTz, sourceTs: Optional[ColumnOrName] = None) -> Column:
    from .functions_extra import _zone
    if sourceTs is None:  # convert_timezone(targetTz, sourceTs): source is the session zone (UTC)
        sourceTz, targetTz, sourceTs = Column(Lit("UTC")), sourceTz, targetTz
    src = sourceTz._expr.value if isinstance(sourceTz, Column) else str(sourceTz)
    dst = targetTz._expr.value if isinstance(targetTz, Column) else str(targetTz)
    zs, zd = _zone(src), _zone(dst)

    def f(t):
        t = t if isinstance(t, _dt.datetime) else _dt.datetime.combine(t, _dt.time())
        return t.replace(tzinfo=zs).astimezone(zd).replace(tzinfo=None)
    return _host_map("convert_timezone", [sourceTs], f, T.TimestampType(), params=[src, dst])


def curdate() -> Column:
    from .functions import current_date
    return current_date()


def now() -> Column:
    from .functions import current_timestamp
    return current_timestamp()


localtimestamp = now


def date_diff(end: ColumnOrName, start: ColumnOrName) -> Column:
    from .functions import datediff
    return datediff(end, start)


def dateadd(start: ColumnOrName, days) -> Column:
    from .functions import date_add
    return date_add(start, days)


_UNITS_US = {"MICROSECOND": 1, "MILLISECOND": 1000, "SECOND": 10 ** 6, "MINUTE": 60 * 10 ** 6,
             "HOUR": 3600 * 10 ** 6, "DAY": 86400 * 10 ** 6, "WEEK": 7 * 86400 * 10 ** 6}


def timestampadd(unit: str, quantity, ts: ColumnOrName) -> Column:
    u = str(unit).upper().rstrip("S")
    from .functions_more import _add_months

    def f(q, t):
        t = t if isinstance(t, _dt.datetime) else _dt.datetime.combine(t, _dt.time())
        q = int(q)
        if u in _UNITS_US:
            return t + _dt.timedelta(microseconds=q * _UNITS_US[u])
        months = {"MONTH": 1, "QUARTER": 3, "YEAR": 12}.get(u)
        if months is None:
            raise ValueError(f"timestampadd: unsupported unit {unit!r}")
        d = _add_months(t.date(), q * months)
        return _dt.datetime.combine(d, t.time())
    qc = quantity if isinstance(quantity, (str, Column)) else Column(Lit(quantity))
    return _host_map("timestampadd", [qc, ts], f, T.TimestampType(), params=[u])


def timestampdiff(unit: str, start: ColumnOrName, end: ColumnOrName) -> Column:
    u = str(unit).upper().rstrip("S")

    def f(a, b):
        a = a if isinstance(a, _dt.datetime) else _dt.datetime.combine(a, _dt.time())
        b = b if isinstance(b, _dt.datetime) else _dt.datetime.combine(b, _dt.time())
        if u in _UNITS_US:
            us = (b - a) // _dt.timedelta(microseconds=1)
            return int(us / _UNITS_US[u]) if us >= 0 else -int(-us / _UNITS_US[u])
        months = (b.year - a.year) * 12 + (b.month - a.month)
        if months > 0 and (b.day, b.time()) < (a.day, a.time()):
            months -= 1
        elif months < 0 and (b.day, b.time()) > (a.day, a.time()):
            months += 1
        per = {"MONTH": 1, "QUARTER": 3, "YEAR": 12}.get(u)
        if per is None:
            raise ValueError(f"timestampdiff: unsupported unit {unit!r}")
        return int(months / per)
    return _host_map("timestampdiff", [start, end], f, T.LongType(), params=[u])


def dayname(c: ColumnOrName) -> Column:
    return _host_map("dayname", [c], lambda t: t.strftime("%a"), T.StringType())


def monthname(c: ColumnOrName) -> Column:
    return _host_map("monthname", [c], lambda t: t.strftime("%b"), T.StringType())


def weekday(c: ColumnOrName) -> Column:
    return _host_map("weekday", [c], lambda t: t.weekday(), T.IntegerType())


def day(c: ColumnOrName) -> Column:
    from .functions import dayofmonth
    return dayofmonth(c)


def uuid() -> Column:
    def impl(frame, args):
        out = np.empty(frame._nrows, dtype=object)
        for i in range(frame._nrows):
            out[i] = str(_uuid.uuid4())
        return ColumnData(out, None, T.StringType())
    return Column(Func("uuid", [], impl))


def current_user() -> Column:
    from .functions import lit
    try:
        name = getpass.getuser()
    except Exception:  # noqa: BLE001 — no passwd entry
        name = "unknown"
    return lit(name)


user = current_user
session_user = current_user


def version() -> Column:
    from .functions import lit
    from .. import __version__ as v
    return lit(f"{v} (MI355X-native)")


def input_file_block_start() -> Column:
    from .functions import lit
    return lit(-1).cast("bigint")


def input_file_block_length() -> Column:
    from .functions import lit
    return lit(-1).cast("bigint")


# ------------------------------------------------------------------ Column-method helpers, misc
def _like_rx(pattern: str, escape: str = "\\", flags=0):
    out, i = [], 0
    while i < len(pattern):
        ch = pattern[i]
        if ch == escape and i + 1 < len(pattern):
            out.append(re.escape(pattern[i + 1]))
            i += 2
            continue
        out.append(".*" if ch == "%" else "." if ch == "_" else re.escape(ch))
        i += 1
    return re.compile("".join(out), re.S | flags)


def like(s: ColumnOrName, pattern, escapeChar=None) -> Column:
    r"""SQL LIKE: ``%`` any run, ``_`` one character, ``escapeChar`` (default ``\``) escapes."""
    pat = pattern._expr.value if isinstance(pattern, Column) else str(pattern)
    rx = _like_rx(pat, escapeChar or "\\")
    return _host_map("like", [s], lambda v: rx.fullmatch(str(v)) is not None, T.BooleanType(), params=[pat])


def ilike(s: ColumnOrName, pattern, escapeChar=None) -> Column:
    pat = pattern._expr.value if isinstance(pattern, Column) else str(pattern)
    rx = _like_rx(pat, escapeChar or "\\", re.IGNORECASE)
    return _host_map("ilike", [s], lambda v: rx.fullmatch(str(v)) is not None, T.BooleanType(), params=[pat])


def substr(s: ColumnOrName, pos, len=None) -> Column:  # noqa: A002
    """``substr(str, pos[, len])`` with column or literal position / length (1-based, Spark)."""
    lit_ = (lambda x: x if isinstance(x, Column) else Column(Lit(x)))
    args = [s, lit_(pos)] + ([] if len is None else [lit_(len)])

    from .functions import spark_substr

    def f(v, p, n=None):
        v = str(v)
        return spark_substr(v, int(p), builtins.len(v) + 1 if n is None else int(n))
    return _host_map("substr", args, f, T.StringType())


class _ItemOrField(Func):
    """``col[key]``: a struct field for struct columns, ``getItem`` (array index / map key) otherwise."""

    def __init__(self, child, key):
        super().__init__("getitem", [child], None)
        self.key = key

    def __str__(self):
        return f"{self.args[0]}[{self.key}]"

    def name(self):
        return str(self)

    def eval(self, frame):
        from .sqlparse import GetField, Subscript
        cd = self.args[0].eval(frame)
        if isinstance(cd.dtype, T.StructType) and isinstance(self.key, str):
            return GetField(self.args[0], self.key).eval(frame)
        return Subscript(self.args[0], Lit(self.key)).eval(frame)


def _bitwise(op: str, a: Column, b) -> Column:
    fn = {"&": torch.bitwise_and, "|": torch.bitwise_or, "^": torch.bitwise_xor}[op]
    bb = b if isinstance(b, Column) else Column(Lit(b))

    def impl(frame, args):
        x, y = args
        if x.is_host or y.is_host:
            raise TypeError("bitwise operators need integral columns")
        dt = x.dtype if T.is_integral(x.dtype) else T.LongType()
        v = fn(x.values.to(torch.int64), y.values.to(torch.int64).to(x.values.device))
        ok = None if x.valid is None and y.valid is None else x.valid_mask() & y.valid_mask().to(x.values.device)
        return ColumnData(v.to(dt.torch_dtype), ok, dt)
    f = Func(op, [a._expr, bb._expr], impl)
    f.label = f"({a._expr} {op} {bb._expr})"
    return Column(f)


def _struct_rows(cd):
    from .dataframe import column_to_python
    return column_to_python(cd)


def _with_field(c: Column, name: str, value: Column) -> Column:
    from .builder import column_from_values
    from .dataframe import column_to_python
    from .types import Row
    v = value if isinstance(value, Column) else Column(Lit(value))

    def impl(frame, args):
        st, val = args
        if not isinstance(st.dtype, T.StructType):
            raise TypeError("withField needs a struct column")
        fields = [f for f in st.dtype.fields if f.name != name]
        pos = next((i for i, f in enumerate(st.dtype.fields) if f.name == name), len(fields))
        fields.insert(pos, T.StructField(name, val.dtype, True))
        dt = T.StructType(fields)
        out = []
        for r, x in zip(column_to_python(st), column_to_python(val)):
            if r is None:
                out.append(None)
                continue
            d = r.asDict() if isinstance(r, Row) else dict(r)
            d[name] = x
            out.append(Row(**{f.name: d.get(f.name) for f in fields}))
        return column_from_values(out, dt, frame._device)
    f = Func("update_fields", [c._expr, v._expr], impl)
    f.label = f"update_fields({c._expr}, WithField({name}, {v._expr}))"
    return Column(f)


def _drop_fields(c: Column, names) -> Column:
    from .builder import column_from_values
    from .dataframe import column_to_python
    from .types import Row

    def impl(frame, args):
        st = args[0]
        if not isinstance(st.dtype, T.StructType):
            raise TypeError("dropFields needs a struct column")
        fields = [f for f in st.dtype.fields if f.name not in names]
        dt = T.StructType(fields)
        out = [None if r is None else Row(**{f.name: (r.asDict() if isinstance(r, Row) else r).get(f.name)
                                                for f in fields}) for r in column_to_python(st)]
        return column_from_values(out, dt, frame._device)
    f = Func("drop_fields", [c._expr], impl)
    f.label = f"update_fields({c._expr}, {', '.join(f'dropfield({n})' for n in names)})"
    return Column(f)


def find_in_set(s: ColumnOrName, strArray: ColumnOrName) -> Column:
    """1-based index of ``s`` in the comma-separated list (0 when absent or ``s`` contains a comma)."""
    return _host_map("find_in_set", [s, strArray], lambda a, b: 0 if "," in str(a) else (
        str(b).split(",").index(str(a)) + 1 if str(a) in str(b).split(",") else 0), T.IntegerType())


def elt(*inputs: ColumnOrName) -> Column:
    """``elt(n, s1, s2, ...)``: the n-th string (1-based), null when out of range."""
    def f(n, *vals):
        if n is None:
            return None
        n = int(n)
        return vals[n - 1] if 1 <= n <= len(vals) else None
    return UserDefinedFunction(f, T.StringType(), name="elt")(*inputs)


def get(col: ColumnOrName, index) -> Column:
    """Array element at a 0-based index, null when out of range."""
    from .sqlparse import Subscript
    ix = index if isinstance(index, Column) else Column(Lit(index))
    return Column(Subscript(_c(col), ix._expr))


def negate(c: ColumnOrName) -> Column:
    return -Column(_c(c))


def position(substr: ColumnOrName, str: ColumnOrName, start=None) -> Column:  # noqa: A002
    """1-based position of ``substr`` in ``str`` at or after ``start`` (0 when absent)."""
    args = [substr, str] + ([] if start is None else [start if isinstance(start, Column) else Column(Lit(start))])

    def f(sub, s, st=1):
        st = int(st)
        if st < 1:
            return 0
        return builtins.str(s).find(builtins.str(sub), st - 1) + 1
    return _host_map("position", args, f, T.IntegerType())


def raise_error(errMsg) -> Column:
    msg = errMsg._expr.value if isinstance(errMsg, Column) and isinstance(errMsg._expr, Lit) else errMsg

    def impl(frame, args):
        if frame._nrows:
            raise RuntimeError(str(msg))
        return ColumnData(np.empty(0, dtype=object), None, T.NullType())
    return Column(Func("raise_error", [], impl))


def assert_true(col: ColumnOrName, errMsg=None) -> Column:
    def impl(frame, args):
        from .dataframe import column_to_python
        vals = column_to_python(args[0])
        if any(not v for v in vals):
            raise RuntimeError(str(errMsg) if errMsg is not None else f"'{args[0]}' is not true!")
        return ColumnData(np.full(frame._nrows, None, dtype=object), np.zeros(frame._nrows, dtype=bool),
                          T.NullType())
    return Column(Func("assert_true", [_c(col)], impl))


def str_to_map(text: ColumnOrName, pairDelim=None, keyValueDelim=None) -> Column:
    pd_ = pairDelim._expr.value if isinstance(pairDelim, Column) else (pairDelim or ",")
    kd = keyValueDelim._expr.value if isinstance(keyValueDelim, Column) else (keyValueDelim or ":")

    def f(s):
        out = {}
        for part in re.split(pd_, str(s)):
            kv = re.split(kd, part, maxsplit=1)
            out[kv[0]] = kv[1] if len(kv) > 1 else None
        return out
    return _host_map("str_to_map", [text], f, T.MapType(T.StringType(), T.StringType()))


def sha(col: ColumnOrName) -> Column:
    from .functions_more import sha1
    return sha1(col)


def replace(src: ColumnOrName, search, replace=None) -> Column:  # noqa: A002
    s_ = search._expr.value if isinstance(search, Column) else search
    r_ = "" if replace is None else (replace._expr.value if isinstance(replace, Column) else replace)
    return _host_map("replace", [src], lambda v: str(v).replace(s_, r_) if s_ else str(v), T.StringType())


def regexp_extract_all(s: ColumnOrName, regexp, idx=1) -> Column:
    rx = _rx(regexp)
    i = idx._expr.value if isinstance(idx, Column) else int(idx)

    def f(v):
        return [(m.group(i) or "") for m in rx.finditer(str(v))]
    return _host_map("regexp_extract_all", [s], f, T.ArrayType(T.StringType()))


def call_function(funcName: str, *cols) -> Column:
    """Call a built-in or registered function by name."""
    from . import functions as F
    from .functions import REGISTERED_UDFS
    if funcName in REGISTERED_UDFS:
        return REGISTERED_UDFS[funcName](*cols)
    fn = getattr(F, funcName, None) or getattr(F, funcName.lower(), None)
    if fn is None or not callable(fn):
        raise ValueError(f"unknown function {funcName}")
    return fn(*cols)


def call_udf(udfName: str, *cols) -> Column:
    from .functions import REGISTERED_UDFS
    if udfName not in REGISTERED_UDFS:
        raise ValueError(f"no registered UDF {udfName}")
    return REGISTERED_UDFS[udfName](*cols)


def _const_str(name, getter):
    def impl(frame, args):
        v = getter(frame)
        out = np.empty(frame._nrows, dtype=object)
        out[:] = v
        return ColumnData(out, None, T.StringType())
    return Column(Func(name, [], impl))


def current_catalog() -> Column:
    return _const_str("current_catalog", lambda f: "spark_catalog")


def current_database() -> Column:
    return _const_str("current_database", lambda f: f._session.catalog.currentDatabase())


current_schema = current_database


def _csv_line(vals, sep=","):
    import csv
    import io
    buf = io.StringIO()
    csv.writer(buf, delimiter=sep, lineterminator="").writerow(["" if v is None else v for v in vals])
    return buf.getvalue()


def to_csv(col: ColumnOrName, options=None) -> Column:
    from .types import Row
    sep = (options or {}).get("sep", ",")

    def f(v):
        vals = list(v.asDict().values()) if isinstance(v, Row) else list(v.values()) if isinstance(v, dict) \
            else list(v)
        return _csv_line(vals, sep)
    return _host_map("to_csv", [col], f, T.StringType())


def from_csv(col: ColumnOrName, schema, options=None) -> Column:
    import csv
    from .functions_extra import _typed
    from .types import Row
    dt = T.parse_ddl_schema(schema) if isinstance(schema, str) else schema
    if isinstance(schema, Column):
        dt = T.parse_ddl_schema(schema._expr.value)
    sep = (options or {}).get("sep", ",")

    def f(s):
        fields = next(csv.reader([str(s)], delimiter=sep), [])
        vals = {}
        for i, fl in enumerate(dt.fields):
            raw = fields[i] if i < len(fields) else None
            vals[fl.name] = None if raw in (None, "") else _typed(_parse_scalar(raw, fl.dataType), fl.dataType)
        return Row(**vals)
    return _host_map("from_csv", [col], f, dt)


def _parse_scalar(raw: str, dt):
    try:
        if T.is_integral(dt):
            return int(raw)
        if isinstance(dt, (T.DoubleType, T.FloatType)):
            return float(raw)
        if isinstance(dt, T.BooleanType):
            return raw.strip().lower() == "true"
    except ValueError:
        return None
    return raw


def schema_of_csv(csv_str, options=None) -> Column:
    text = csv_str._expr.value if isinstance(csv_str, Column) else str(csv_str)
    import csv
    sep = (options or {}).get("sep", ",")
    fields = next(csv.reader([text], delimiter=sep), [])

    def kind(x):
        for cast, name in ((int, "INT"), (float, "DOUBLE")):
            try:
                cast(x)
                return name
            except ValueError:
                pass
        return "BOOLEAN" if x.lower() in ("true", "false") else "STRING"
    ddl = "STRUCT<" + ", ".join(f"_c{i}: {kind(x)}" for i, x in enumerate(fields)) + ">"
    return _const_str("schema_of_csv", lambda f: ddl)


class _PartitionTransform(Func):
    """``years`` / ``months`` / ``days`` / ``hours`` / ``bucket`` partition transforms
    (``writeTo(...).partitionedBy``); evaluated they give the partition value."""

    def __init__(self, kind, child, n=None):
        super().__init__(kind, [child], None)
        self.kind, self.n = kind, n

    def eval(self, frame):
        cd = self.args[0].eval(frame)
        if self.kind == "bucket":
            from .hashing import device_hash
            h = device_hash([cd], 42) if not cd.is_host else None
            if h is None:
                from .functions_extra import hash as _hash
                h = _hash(Column(self.args[0]))._expr.eval(frame).values
            return ColumnData(torch.remainder(h.to(torch.int64), self.n).to(torch.int32), cd.valid, T.IntegerType())
        us = cd.values.to(torch.int64) * (86_400_000_000 if isinstance(cd.dtype, T.DateType) else 1)
        if self.kind == "hours":
            return ColumnData(torch.div(us, 3_600_000_000, rounding_mode="floor").to(torch.int32), cd.valid,
                              T.IntegerType())
        days = torch.div(us, 86_400_000_000, rounding_mode="floor")
        if self.kind == "days":
            return ColumnData(days.to(torch.int32), cd.valid, T.DateType())
        d = np.asarray(days.cpu().numpy(), dtype="datetime64[D]")
        y = d.astype("datetime64[Y]").astype(np.int64)
        if self.kind == "years":
            return ColumnData(torch.as_tensor(y.astype(np.int32), device=cd.values.device), cd.valid,
                              T.IntegerType())
        m = d.astype("datetime64[M]").astype(np.int64)
        return ColumnData(torch.as_tensor(m.astype(np.int32), device=cd.values.device), cd.valid, T.IntegerType())


def years(col: ColumnOrName) -> Column:
    return Column(_PartitionTransform("years", _c(col)))


def months(col: ColumnOrName) -> Column:
    return Column(_PartitionTransform("months", _c(col)))


def days(col: ColumnOrName) -> Column:
    return Column(_PartitionTransform("days", _c(col)))


def hours(col: ColumnOrName) -> Column:
    return Column(_PartitionTransform("hours", _c(col)))


def bucket(numBuckets, col: ColumnOrName) -> Column:
    n = numBuckets._expr.value if isinstance(numBuckets, Column) else int(numBuckets)
    return Column(_PartitionTransform("bucket", _c(col), n))


def to_timestamp_ltz(timestamp: ColumnOrName, format=None) -> Column:  # noqa: A002
    from .functions import to_timestamp
    return to_timestamp(timestamp, format._expr.value if isinstance(format, Column) else format)


to_timestamp_ntz = to_timestamp_ltz


def make_timestamp_ltz(years, months, days, hours, mins, secs, timezone=None) -> Column:
    from .functions_extra import make_timestamp
    return make_timestamp(years, months, days, hours, mins, secs, timezone)


def make_timestamp_ntz(years, months, days, hours, mins, secs) -> Column:
    from .functions_extra import make_timestamp
    return make_timestamp(years, months, days, hours, mins, secs)


def to_unix_timestamp(timestamp: ColumnOrName, format=None) -> Column:  # noqa: A002
    from .functions import unix_timestamp
    return unix_timestamp(timestamp, format._expr.value if isinstance(format, Column) else format)


class _HistogramNumeric(_HostValuesAgg):
    """``histogram_numeric(col, nBins)``: Spark's streaming histogram (Ben-Haim & Tom-Tov): merge the
    two closest centroids until ``nBins`` remain; result array<struct<x, y>>."""

    def result_type(self):
        return T.ArrayType(T.StructType([T.StructField("x", T.DoubleType()), T.StructField("y", T.DoubleType())]))

    def merge(self, parts):
        from .types import Row
        vals = [v for p in parts for v in p]
        if not vals:
            return None
        nb = int(self.arg)
        pts = {}
        for v in vals:
            pts[float(v)] = pts.get(float(v), 0.0) + 1.0
        cs = sorted(pts.items())
        while len(cs) > nb:
            i = builtins.min(range(len(cs) - 1), key=lambda j: cs[j + 1][0] - cs[j][0])
            (x1, y1), (x2, y2) = cs[i], cs[i + 1]
            cs[i:i + 2] = [((x1 * y1 + x2 * y2) / (y1 + y2), y1 + y2)]
        return [Row(x=x, y=y) for x, y in cs]


def histogram_numeric(col: ColumnOrName, nBins) -> Column:
    n = nBins._expr.value if isinstance(nBins, Column) else int(nBins)
    a = _HistogramNumeric("histogram_numeric", _c(col))
    a.arg = n
    return Column(a)


def nth_value(col: ColumnOrName, offset: int, ignoreNulls: bool = False) -> Column:
    """Window function: the ``offset``-th value (1-based) of the window frame, null if it has fewer rows."""
    from .window import WindowFunc
    return Column(WindowFunc("nth_value", _c(col), int(offset), bool(ignoreNulls)))


__all__ = [n for n in dir() if not n.startswith("_") and n not in (
    "annotations", "builtins", "getpass", "math", "np", "re", "torch", "T", "Any", "List", "Optional", "urllib",
    "AggExpr", "Column", "ColumnData", "Func", "Lit", "UserDefinedFunction", "ColumnOrName")]
