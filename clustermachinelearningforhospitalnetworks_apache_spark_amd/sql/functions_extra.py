"""The rest of pyspark.sql.functions: null helpers, bit / base conversion math, string utilities,
hashes (bit-exact Murmur3 / XXH64, sql/hashing.py), time zones, collection functions, higher-order
functions over arrays and maps, map builders and JSON.

Higher-order functions (``transform``, ``filter``, ``exists``, ``forall``, ``aggregate``,
``zip_with``, ``map_filter``, ``transform_keys``, ``transform_values``) take a Python lambda over
Columns, as in pyspark. The lambda's expression is evaluated ONCE, vectorised, on a frame of the
flattened elements (each element row carries its parent row's columns, so the lambda may
reference outer columns): numeric lambdas therefore run as device kernels over every element of
every array at once, and the results are regrouped into per-row arrays. ``aggregate`` folds
position by position, each step one vectorised evaluation over the rows still holding elements.
"""
from __future__ import annotations

import base64 as _b64
import builtins
import datetime as _dt
import inspect
import json
import math
import random as _random
import re
from typing import Any, Callable, Dict, List, Optional

import numpy as np
import torch

from . import types as T
from .column import ColRef, Column, ColumnData, Expr, Func, Lit, _to_host
from .functions import ColumnOrName, UserDefinedFunction, _c, _host_map


def _e(c) -> Expr:
    """Column / name / literal -> Expr."""
    if isinstance(c, (str, Column)):
        return _c(c)
    if isinstance(c, Expr):
        return c
    return Lit(c)


def _py(cd: ColumnData) -> List[Any]:
    from .dataframe import column_to_python
    return column_to_python(cd)


def _from_values(vals, dt, frame) -> ColumnData:
    from .builder import column_from_values
    return column_from_values(vals, dt, frame._device)


# ------------------------------------------------------------------------------------------ null helpers

def ifnull(col1: ColumnOrName, col2: ColumnOrName) -> Column:
    from .functions import coalesce
    return coalesce(col1, col2)


nvl = ifnull


def nvl2(col1: ColumnOrName, col2: ColumnOrName, col3: ColumnOrName) -> Column:
    from .functions import when
    return when(Column(_e(col1)).isNotNull(), Column(_e(col2))).otherwise(Column(_e(col3)))


def nullif(col1: ColumnOrName, col2: ColumnOrName) -> Column:
    from .functions import lit, when
    return when(Column(_e(col1)) == Column(_e(col2)), lit(None)).otherwise(Column(_e(col1)))


def try_divide(left: ColumnOrName, right: ColumnOrName) -> Column:
    """left / right as double, null when right is 0 (or either side is null)."""
    def impl(frame, args):
        a, b = args
        x, y = a.values.to(torch.float64), b.values.to(torch.float64)
        valid = a.valid_mask() & b.valid_mask() & (y != 0)
        return ColumnData(torch.where(y != 0, x / torch.where(y != 0, y, torch.ones_like(y)), torch.zeros_like(x)),
                          valid, T.DoubleType())
    return Column(Func("try_divide", [_e(left), _e(right)], impl))


def try_add(left: ColumnOrName, right: ColumnOrName) -> Column:
    """left + right; for integral inputs null where the 64-bit sum overflows."""
    def impl(frame, args):
        a, b = args
        valid = a.valid_mask() & b.valid_mask()
        if T.is_integral(a.dtype) and T.is_integral(b.dtype):
            x, y = a.values.to(torch.int64), b.values.to(torch.int64)
            s = x + y
            ovf = ((x >= 0) == (y >= 0)) & ((s >= 0) != (x >= 0))
            rt = T.LongType() if isinstance(a.dtype, T.LongType) or isinstance(b.dtype, T.LongType) else T.IntegerType()
            if isinstance(rt, T.IntegerType):
                ovf = ovf | (s > 2 ** 31 - 1) | (s < -2 ** 31)
                s = s.to(torch.int32)
            return ColumnData(s, valid & ~ovf, rt)
        return ColumnData(a.values.to(torch.float64) + b.values.to(torch.float64), valid, T.DoubleType())
    return Column(Func("try_add", [_e(left), _e(right)], impl))


# ------------------------------------------------------------------------------------------ math / bits

def _dev1(name, fn, rt=T.DoubleType()):
    def f(c: ColumnOrName) -> Column:
        def impl(frame, args):
            a = args[0]
            return ColumnData(fn(a.values), a.valid, rt)
        return Column(Func(f"{name}({c if isinstance(c, str) else _e(c)})", [_e(c)], impl))
    f.__name__ = name
    return f


acosh = _dev1("acosh", lambda v: torch.acosh(v.to(torch.float64)))
asinh = _dev1("asinh", lambda v: torch.asinh(v.to(torch.float64)))
atanh = _dev1("atanh", lambda v: torch.atanh(v.to(torch.float64)))
cot = _dev1("cot", lambda v: 1.0 / torch.tan(v.to(torch.float64)))
sec = _dev1("sec", lambda v: 1.0 / torch.cos(v.to(torch.float64)))
csc = _dev1("csc", lambda v: 1.0 / torch.sin(v.to(torch.float64)))
ln = _dev1("ln", lambda v: torch.log(v.to(torch.float64)))


def factorial(c: ColumnOrName) -> Column:
    """n! for 0 <= n <= 20 (null otherwise, like Spark)."""
    def impl(frame, args):
        a = args[0]
        n = a.values.to(torch.int64)
        table = torch.as_tensor([math.factorial(i) for i in range(21)], dtype=torch.int64, device=n.device)
        ok = (n >= 0) & (n <= 20)
        out = table[n.clamp(0, 20)]
        return ColumnData(out, a.valid_mask() & ok, T.LongType())
    return Column(Func("factorial", [_e(c)], impl))


def bitwise_not(c: ColumnOrName) -> Column:
    def impl(frame, args):
        a = args[0]
        return ColumnData(torch.bitwise_not(a.values), a.valid, a.dtype)
    return Column(Func("~", [_e(c)], impl))


bitwiseNOT = bitwise_not


def _shift(name, op):
    def f(c: ColumnOrName, numBits: int) -> Column:
        def impl(frame, args):
            a = args[0]
            v = a.values
            if isinstance(a.dtype, T.LongType):
                bits = int(numBits) & 63
                x = v.to(torch.int64)
                if op == "l":
                    out = x << bits
                elif op == "r":
                    out = x >> bits
                else:
                    out = (x >> bits) & ((1 << (64 - bits)) - 1) if bits else x
                return ColumnData(out, a.valid, T.LongType())
            bits = int(numBits) & 31
            x = v.to(torch.int64) & 0xFFFFFFFF
            if op == "l":
                out = (x << bits) & 0xFFFFFFFF
            elif op == "r":
                out = (v.to(torch.int64) >> bits) & 0xFFFFFFFF
            else:
                out = x >> bits
            out = torch.where(out >= 2 ** 31, out - 2 ** 32, out).to(torch.int32)
            return ColumnData(out, a.valid, T.IntegerType())
        return Column(Func(f"{name}({numBits})", [_e(c)], impl))
    f.__name__ = name
    return f


shiftleft = shiftLeft = _shift("shiftleft", "l")
shiftright = shiftRight = _shift("shiftright", "r")
shiftrightunsigned = shiftRightUnsigned = _shift("shiftrightunsigned", "u")


def _to_base(n: int, base: int) -> str:
    digits = "0123456789ABCDEFGHIJKLMNOPQRSTUVWXYZ"
    if n == 0:
        return "0"
    out = []
    while n:
        n, r = divmod(n, base)
        out.append(digits[r])
    return "".join(reversed(out))


def bin(c: ColumnOrName) -> Column:  # noqa: A001
    return _host_map("bin", [c], lambda v: _to_base(int(v) & ((1 << 64) - 1), 2), T.StringType())


def hex(c: ColumnOrName) -> Column:  # noqa: A001
    def f(v):
        if isinstance(v, (bytes, bytearray)):
            return v.hex().upper()
        if isinstance(v, str):
            return v.encode("utf-8").hex().upper()
        return _to_base(int(v) & ((1 << 64) - 1), 16)
    return _host_map("hex", [c], f, T.StringType())


def unhex(c: ColumnOrName) -> Column:
    def f(s):
        s = str(s)
        if len(s) % 2:
            s = "0" + s
        try:
            return bytes.fromhex(s)
        except ValueError:
            return None
    return _host_map("unhex", [c], f, T.BinaryType())


def conv(c: ColumnOrName, fromBase: int, toBase: int) -> Column:
    """Base conversion of a number string (Spark: unsigned 64-bit unless toBase is negative)."""
    def f(s):
        s = str(s).strip()
        neg = s.startswith("-")
        digits = s[1:] if neg else s
        try:
            v = int(digits, abs(int(fromBase))) if digits else 0
        except ValueError:
            m = re.match(r"[0-9A-Za-z]*", digits)
            try:
                v = int(m.group(0), abs(int(fromBase))) if m and m.group(0) else 0
            except ValueError:
                return None
        if neg:
            v = -v
        if toBase < 0:
            v = v - (1 << 64) if v >= (1 << 63) else v
            return ("-" if v < 0 else "") + _to_base(builtins.abs(v), -toBase)
        return _to_base(v & ((1 << 64) - 1), toBase)
    return _host_map("conv", [c], f, T.StringType())


def randn(seed: int = 0) -> Column:
    """Standard normal per row from two counter-based uniforms of the row id (Box–Muller)."""
    from ..utils import rng

    def impl(frame, args):
        u1 = rng.uniform(frame._row_ids, seed, stream=11).clamp(min=1e-300)
        u2 = rng.uniform(frame._row_ids, seed, stream=12)
        return ColumnData(torch.sqrt(-2.0 * torch.log(u1)) * torch.cos(2.0 * math.pi * u2), None, T.DoubleType())
    return Column(Func(f"randn({seed})", [], impl))


def hash(*cols: ColumnOrName) -> Column:  # noqa: A001
    """Spark's Murmur3 row hash (seed 42), as int."""
    return _row_hash("hash", "murmur3", cols)


def xxhash64(*cols: ColumnOrName) -> Column:
    """Spark's XXH64 row hash (seed 42), as bigint."""
    return _row_hash("xxhash64", "xx", cols)


def _row_hash(name: str, algo: str, cols) -> Column:
    from .hashing import device_hash, hash_value

    def impl(frame, args):
        n, dev = frame._nrows, frame._device
        h = torch.full((n,), 42, dtype=torch.int64, device=dev)
        for a in args:
            if isinstance(a.dtype, T.NullType):
                continue
            wide_dec = isinstance(a.dtype, T.DecimalType) and a.dtype.precision > 18
            if not a.is_host and a.values.dim() == 1 and not wide_dec and (T.is_numeric(a.dtype) or isinstance(
                    a.dtype, (T.BooleanType, T.DateType, T.TimestampType))):
                nh = device_hash(a.values, a.dtype, h, algo)
                h = nh if a.valid is None else torch.where(a.valid.to(dev), nh, h)
                continue
            hv = h.cpu().tolist()
            vals = _py(a)
            mask = (1 << 32) - 1 if algo == "murmur3" else (1 << 64) - 1
            out = []
            for v, s in zip(vals, hv):
                r = hash_value(v, a.dtype, s & mask, algo)
                out.append(r - (1 << 64) if r >= (1 << 63) else r)
            h = torch.as_tensor(out, dtype=torch.int64, device=dev)
        if algo == "murmur3":
            h = h & 0xFFFFFFFF
            return ColumnData(torch.where(h >= 2 ** 31, h - 2 ** 32, h).to(torch.int32), None, T.IntegerType())
        return ColumnData(h, None, T.LongType())
    return Column(Func(name, [_e(c) for c in cols], impl))


# ------------------------------------------------------------------------------------------ strings

def ascii(c: ColumnOrName) -> Column:  # noqa: A001
    return _host_map("ascii", [c], lambda s: ord(str(s)[0]) if str(s) else 0, T.IntegerType())


def base64(c: ColumnOrName) -> Column:
    return _host_map("base64", [c], lambda s: _b64.b64encode(s if isinstance(s, (bytes, bytearray))
                                                              else str(s).encode("utf-8")).decode("ascii"),
                     T.StringType())


def unbase64(c: ColumnOrName) -> Column:
    def f(s):
        try:
            return _b64.b64decode(str(s))
        except (ValueError, TypeError):
            return None
    return _host_map("unbase64", [c], f, T.BinaryType())


def encode(c: ColumnOrName, charset: str) -> Column:
    return _host_map("encode", [c], lambda s: str(s).encode(charset), T.BinaryType())


def decode(c: ColumnOrName, charset: str) -> Column:
    return _host_map("decode", [c], lambda b: bytes(b).decode(charset, errors="replace")
                     if isinstance(b, (bytes, bytearray)) else str(b), T.StringType())


def bit_length(c: ColumnOrName) -> Column:
    return _host_map("bit_length", [c], lambda s: 8 * len(s if isinstance(s, (bytes, bytearray))
                                                         else str(s).encode("utf-8")), T.IntegerType())


def octet_length(c: ColumnOrName) -> Column:
    return _host_map("octet_length", [c], lambda s: len(s if isinstance(s, (bytes, bytearray))
                                                       else str(s).encode("utf-8")), T.IntegerType())


def char_length(c: ColumnOrName) -> Column:
    return _host_map("char_length", [c], lambda s: len(str(s)), T.IntegerType())


character_length = char_length


def format_number(c: ColumnOrName, d: int) -> Column:
    """'#,###,###.##' with d decimals, HALF_EVEN like Java's DecimalFormat."""
    from decimal import ROUND_HALF_EVEN, Decimal

    def f(v):
        if d < 0:
            return None
        q = Decimal(repr(float(v))).quantize(Decimal(1).scaleb(-d), rounding=ROUND_HALF_EVEN)
        return f"{q:,.{d}f}"
    return _host_map("format_number", [c], f, T.StringType())


def format_string(format: str, *cols: ColumnOrName) -> Column:  # noqa: A002
    """printf-style formatting (Java Formatter subset: %s %d %f %e %x %o %c %b %%)."""
    py = re.sub(r"%(\d+)\$", "%", format)

    def f(*vals):
        conv = []
        for v in vals:
            conv.append("null" if v is None else v)
        try:
            return py % tuple(conv)
        except (TypeError, ValueError):
            return None
    return UserDefinedFunction(f, T.StringType(), name="format_string")(*cols)


printf = format_string


def levenshtein(left: ColumnOrName, right: ColumnOrName, threshold: Optional[int] = None) -> Column:
    def lev(a, b):
        a, b = str(a), str(b)
        prev = list(range(len(b) + 1))
        for i, ca in enumerate(a, 1):
            cur = [i]
            for j, cb in enumerate(b, 1):
                cur.append(builtins.min(prev[j] + 1, cur[j - 1] + 1, prev[j - 1] + (ca != cb)))
            prev = cur
        d = prev[-1]
        return -1 if threshold is not None and d > threshold else d
    return _host_map("levenshtein", [left, right], lev, T.IntegerType())


_SOUNDEX = {c: d for d, letters in (("1", "BFPV"), ("2", "CGJKQSXZ"), ("3", "DT"), ("4", "L"), ("5", "MN"),
                                    ("6", "R")) for c in letters}


def soundex(c: ColumnOrName) -> Column:
    def f(s):
        s = str(s)
        if not s or not s[0].isalpha():
            return s
        up = s.upper()
        out = up[0]
        last = _SOUNDEX.get(up[0], "")
        for ch in up[1:]:
            code = _SOUNDEX.get(ch, "")
            if ch in "HW":
                continue
            if code and code != last:
                out += code
                if len(out) == 4:
                    break
            last = code
        return out.ljust(4, "0")
    return _host_map("soundex", [c], f, T.StringType())


def overlay(src: ColumnOrName, replace: ColumnOrName, pos, len=-1) -> Column:  # noqa: A002
    def f(s, r):
        s, r = str(s), str(r)
        p = int(pos)
        n = builtins.len(r) if int(len) < 0 else int(len)
        return s[:p - 1] + r + s[p - 1 + n:]
    return _host_map("overlay", [src, replace], f, T.StringType())


def substring_index(c: ColumnOrName, delim: str, count: int) -> Column:
    def f(s):
        s = str(s)
        if count == 0 or not delim:
            return ""
        parts = s.split(delim)
        return delim.join(parts[:count]) if count > 0 else delim.join(parts[count:])
    return _host_map("substring_index", [c], f, T.StringType())


def sentences(string: ColumnOrName, language=None, country=None) -> Column:
    """Split text into sentences of words (array<array<string>>), punctuation dropped."""
    def f(s):
        out = []
        for sent in re.split(r"(?<=[.!?])\s+", str(s).strip()):
            words = re.findall(r"[\w']+", sent)
            if words:
                out.append(words)
        return out
    return _host_map("sentences", [string], f, T.ArrayType(T.ArrayType(T.StringType())))


def to_number(c: ColumnOrName, format: str) -> Column:  # noqa: A002
    """Parse a number string written with a Spark number format ('9', '0', ',', '.', '$', 'S', 'MI')."""
    def f(s):
        s = str(s).strip().replace(",", "").replace("$", "")
        neg = s.endswith("-") or s.startswith("-")
        s = s.strip("+-")
        try:
            v = float(s)
        except ValueError:
            return None
        return -v if neg else v
    return _host_map("to_number", [c], f, T.DoubleType())


def typeof(c: ColumnOrName) -> Column:
    def impl(frame, args):
        out = np.empty(frame._nrows, dtype=object)
        out[:] = args[0].dtype.simpleString()
        return ColumnData(out, None, T.StringType())
    return Column(Func("typeof", [_e(c)], impl))


# ------------------------------------------------------------------------------------------ dates / time zones

def _zone(tz: str):
    from zoneinfo import ZoneInfo
    if re.fullmatch(r"[+-]\d{2}:\d{2}", tz):
        sign = -1 if tz[0] == "-" else 1
        return _dt.timezone(sign * _dt.timedelta(hours=int(tz[1:3]), minutes=int(tz[4:6])))
    return ZoneInfo(tz)


def from_utc_timestamp(timestamp: ColumnOrName, tz: str) -> Column:
    """Render a UTC instant as wall-clock time in ``tz`` (returned as a timestamp)."""
    z = _zone(tz)

    def f(t):
        t = t if isinstance(t, _dt.datetime) else _dt.datetime.combine(t, _dt.time())
        return t.replace(tzinfo=_dt.timezone.utc).astimezone(z).replace(tzinfo=None)
    return _host_map("from_utc_timestamp", [timestamp], f, T.TimestampType())


def to_utc_timestamp(timestamp: ColumnOrName, tz: str) -> Column:
    """Interpret a wall-clock time in ``tz`` and return the UTC instant."""
    z = _zone(tz)

    def f(t):
        t = t if isinstance(t, _dt.datetime) else _dt.datetime.combine(t, _dt.time())
        return t.replace(tzinfo=z).astimezone(_dt.timezone.utc).replace(tzinfo=None)
    return _host_map("to_utc_timestamp", [timestamp], f, T.TimestampType())


def make_date(year: ColumnOrName, month: ColumnOrName, day: ColumnOrName) -> Column:
    def f(y, m, d):
        try:
            return _dt.date(int(y), int(m), int(d))
        except ValueError:
            return None
    return _host_map("make_date", [year, month, day], f, T.DateType())


def make_timestamp(years, months, days, hours, mins, secs, timezone=None) -> Column:
    def f(y, mo, d, h, mi, s):
        try:
            whole = int(math.floor(float(s)))
            us = int(round((float(s) - whole) * 1e6))
            return _dt.datetime(int(y), int(mo), int(d), int(h), int(mi), whole, us)
        except ValueError:
            return None
    return _host_map("make_timestamp", [years, months, days, hours, mins, secs], f, T.TimestampType())


_DOW = {"MO": 0, "TU": 1, "WE": 2, "TH": 3, "FR": 4, "SA": 5, "SU": 6}


def next_day(date: ColumnOrName, dayOfWeek: str) -> Column:
    target = _DOW.get(dayOfWeek.strip().upper()[:2])

    def f(d):
        if target is None:
            return None
        d = d.date() if isinstance(d, _dt.datetime) else d
        delta = (target - d.weekday()) % 7 or 7
        return d + _dt.timedelta(days=delta)
    return _host_map("next_day", [date], f, T.DateType())


def timestamp_seconds(c: ColumnOrName) -> Column:
    def impl(frame, args):
        a = args[0]
        v = a.values
        us = (v.to(torch.float64) * 1e6).round().to(torch.int64) if v.is_floating_point() else v.to(torch.int64) * 1_000_000
        return ColumnData(us, a.valid, T.TimestampType())
    return Column(Func("timestamp_seconds", [_e(c)], impl))


def timestamp_millis(c: ColumnOrName) -> Column:
    def impl(frame, args):
        a = args[0]
        return ColumnData(a.values.to(torch.int64) * 1000, a.valid, T.TimestampType())
    return Column(Func("timestamp_millis", [_e(c)], impl))


def timestamp_micros(c: ColumnOrName) -> Column:
    def impl(frame, args):
        a = args[0]
        return ColumnData(a.values.to(torch.int64), a.valid, T.TimestampType())
    return Column(Func("timestamp_micros", [_e(c)], impl))


def unix_seconds(c: ColumnOrName) -> Column:
    def impl(frame, args):
        a = args[0]
        return ColumnData(torch.div(a.values.to(torch.int64), 1_000_000, rounding_mode="floor"), a.valid, T.LongType())
    return Column(Func("unix_seconds", [_e(c)], impl))


def unix_millis(c: ColumnOrName) -> Column:
    def impl(frame, args):
        a = args[0]
        return ColumnData(torch.div(a.values.to(torch.int64), 1000, rounding_mode="floor"), a.valid, T.LongType())
    return Column(Func("unix_millis", [_e(c)], impl))


def unix_micros(c: ColumnOrName) -> Column:
    def impl(frame, args):
        a = args[0]
        return ColumnData(a.values.to(torch.int64), a.valid, T.LongType())
    return Column(Func("unix_micros", [_e(c)], impl))


def unix_date(c: ColumnOrName) -> Column:
    def impl(frame, args):
        a = args[0]
        return ColumnData(a.values.to(torch.int32), a.valid, T.IntegerType())
    return Column(Func("unix_date", [_e(c)], impl))


def date_from_unix_date(c: ColumnOrName) -> Column:
    def impl(frame, args):
        a = args[0]
        return ColumnData(a.values.to(torch.int32), a.valid, T.DateType())
    return Column(Func("date_from_unix_date", [_e(c)], impl))


_PARTS = {"YEAR": "year", "Y": "year", "YEARS": "year", "YR": "year", "YRS": "year", "MONTH": "month",
          "MON": "month", "MONS": "month", "MONTHS": "month", "DAY": "day", "D": "day", "DAYS": "day",
          "HOUR": "hour", "H": "hour", "HOURS": "hour", "HR": "hour", "HRS": "hour", "MINUTE": "minute",
          "M": "minute", "MIN": "minute", "MINS": "minute", "MINUTES": "minute", "SECOND": "second",
          "S": "second", "SEC": "second", "SECONDS": "second", "SECS": "second", "QUARTER": "quarter",
          "QTR": "quarter", "WEEK": "week", "W": "week", "WEEKS": "week", "DAYOFWEEK": "dow", "DOW": "dow",
          "DAYOFWEEK_ISO": "dow_iso", "DOY": "doy"}


def date_part(field, source: ColumnOrName) -> Column:
    """EXTRACT(field FROM source): year / quarter / month / week / day / dayofweek / doy / hour /
    minute / second (with fraction, as double)."""
    fname = field if isinstance(field, str) else getattr(getattr(field, "_expr", None), "value", str(field))
    part = _PARTS.get(str(fname).strip().upper())
    if part is None:
        raise ValueError(f"unsupported date_part field {fname!r}")

    def f(t):
        d = t.date() if isinstance(t, _dt.datetime) else t
        if part == "year":
            return d.year
        if part == "month":
            return d.month
        if part == "day":
            return d.day
        if part == "quarter":
            return (d.month - 1) // 3 + 1
        if part == "week":
            return d.isocalendar()[1]
        if part == "dow":
            return (d.weekday() + 1) % 7 + 1
        if part == "dow_iso":
            return d.weekday() + 1
        if part == "doy":
            return d.timetuple().tm_yday
        tt = t if isinstance(t, _dt.datetime) else _dt.datetime.combine(t, _dt.time())
        if part == "hour":
            return tt.hour
        if part == "minute":
            return tt.minute
        return tt.second + tt.microsecond / 1e6
    rt = T.DoubleType() if part == "second" else T.IntegerType()
    return _host_map("date_part", [source], f, rt)


def extract(field, source: ColumnOrName) -> Column:
    return date_part(field, source)


datepart = date_part


def current_timezone() -> Column:
    from .functions import lit
    return lit("UTC")


def session_window(timeColumn: ColumnOrName, gapDuration) -> Column:
    """Session windows for groupBy: events of one key closer than ``gapDuration`` share a session."""
    from .window import SessionWindow, parse_duration_us
    return Column(SessionWindow(_e(timeColumn), parse_duration_us(gapDuration)))


def window_time(windowColumn: ColumnOrName) -> Column:
    """The event time of a window struct: its end minus 1 microsecond."""
    def f(w):
        end = w["end"] if isinstance(w, dict) else w.end
        return end - _dt.timedelta(microseconds=1)
    return _host_map("window_time", [windowColumn], f, T.TimestampType())


# ------------------------------------------------------------------------------------------ collections

def _elem(cd: ColumnData) -> T.DataType:
    return cd.dtype.elementType if isinstance(cd.dtype, T.ArrayType) else T.StringType()


def _arr_fn(name: str, cols, fn: Callable, rt_fn: Callable) -> Column:
    """Row-wise function over array (or other) columns; null in -> null out."""
    def impl(frame, args):
        pys = [_py(a) for a in args]
        out = [None if builtins.any(p[i] is None for p in pys) else fn(*[p[i] for p in pys])
               for i in range(frame._nrows)]
        return _from_values(out, rt_fn(args), frame)
    return Column(Func(name, [_e(c) for c in cols], impl))


def _same(args):
    return args[0].dtype


def array_except(col1: ColumnOrName, col2: ColumnOrName) -> Column:
    return _arr_fn("array_except", [col1, col2], lambda a, b: list(dict.fromkeys(x for x in a if x not in b)), _same)


def array_intersect(col1: ColumnOrName, col2: ColumnOrName) -> Column:
    return _arr_fn("array_intersect", [col1, col2], lambda a, b: list(dict.fromkeys(x for x in a if x in b)), _same)


def array_union(col1: ColumnOrName, col2: ColumnOrName) -> Column:
    return _arr_fn("array_union", [col1, col2], lambda a, b: list(dict.fromkeys(list(a) + list(b))), _same)


def arrays_overlap(a1: ColumnOrName, a2: ColumnOrName) -> Column:
    def f(a, b):
        if set(x for x in a if x is not None) & set(x for x in b if x is not None):
            return True
        if (None in a and len(b)) or (None in b and len(a)):
            return None
        return False
    return _arr_fn("arrays_overlap", [a1, a2], f, lambda args: T.BooleanType())


def array_position(c: ColumnOrName, value) -> Column:
    return _arr_fn("array_position", [c], lambda a: next((i + 1 for i, x in enumerate(a) if x == value), 0),
                   lambda args: T.LongType())


def array_remove(c: ColumnOrName, element) -> Column:
    return _arr_fn("array_remove", [c], lambda a: [x for x in a if x != element], _same)


def array_repeat(c: ColumnOrName, count) -> Column:
    def impl(frame, args):
        v = _py(args[0])
        n = _py(args[1])
        out = [None if k is None else [x] * builtins.max(int(k), 0) for x, k in zip(v, n)]
        return _from_values(out, T.ArrayType(args[0].dtype), frame)
    return Column(Func("array_repeat", [_e(c), _e(count)], impl))


def array_sort(c: ColumnOrName, comparator: Optional[Callable] = None) -> Column:
    """Ascending with nulls last (Spark's array_sort); a comparator lambda is evaluated pairwise."""
    if comparator is None:
        def f(a):
            nn = sorted(x for x in a if x is not None)
            return nn + [None] * (len(a) - len(nn))
        return _arr_fn("array_sort", [c], f, _same)
    return _sort_with(c, comparator)


def _sort_with(c, comparator):
    """array_sort with a comparator lambda: all element pairs of all rows are compared in one
    vectorised evaluation, then each array is sorted with the cached outcomes."""
    import functools

    def impl(frame, args):
        vals = _py(args[0])
        et = _elem(args[0])
        rep, ls, rs, keys = [], [], [], []
        for i, a in enumerate(vals):
            if a is None:
                continue
            for x_i, x in enumerate(a):
                for y_i, y in enumerate(a):
                    rep.append(i)
                    ls.append(x)
                    rs.append(y)
                    keys.append((i, x_i, y_i))
        tmp = _lambda_frame(frame, rep, {"__hof_l": _from_values(ls, et, frame),
                                         "__hof_r": _from_values(rs, et, frame)})
        res = _py(_e(comparator(Column(ColRef("__hof_l")), Column(ColRef("__hof_r")))).eval(tmp)) if rep else []
        cmp = {k: (r or 0) for k, r in zip(keys, res)}
        out = []
        for i, a in enumerate(vals):
            if a is None:
                out.append(None)
                continue
            order = sorted(range(len(a)), key=functools.cmp_to_key(lambda p, q: cmp[(i, p, q)]))
            out.append([a[j] for j in order])
        return _from_values(out, args[0].dtype, frame)
    return _hof(Column(Func("array_sort", [_e(c)], impl)), (comparator, ["left", "right"]))


def arrays_zip(*cols: ColumnOrName) -> Column:
    exprs = [_e(c) for c in cols]

    def impl(frame, args):
        from .types import Row
        names = [e.name() if isinstance(e, ColRef) or hasattr(e, "alias") else str(i) for i, e in enumerate(exprs)]
        names = [n if n else str(i) for i, n in enumerate(names)]
        pys = [_py(a) for a in args]
        out = []
        for i in range(frame._nrows):
            arrs = [p[i] for p in pys]
            if builtins.any(a is None for a in arrs):
                out.append(None)
                continue
            m = builtins.max((len(a) for a in arrs), default=0)
            out.append([Row(**{n: (a[j] if j < len(a) else None) for n, a in zip(names, arrs)}) for j in range(m)])
        st = T.StructType([T.StructField(n, _elem(a), True) for n, a in zip(names, args)])
        return _from_values(out, T.ArrayType(st), frame)
    return Column(Func("arrays_zip", exprs, impl))


def flatten(c: ColumnOrName) -> Column:
    def f(a):
        if builtins.any(x is None for x in a):
            return None
        return [y for x in a for y in x]
    return _arr_fn("flatten", [c], f, lambda args: _elem(args[0]))


def sequence(start: ColumnOrName, stop: ColumnOrName, step: Optional[ColumnOrName] = None) -> Column:
    cols = [start, stop] + ([step] if step is not None else [])

    def f(a, b, s=None):
        if isinstance(a, (_dt.date, _dt.datetime)):
            st = _dt.timedelta(days=1) if s is None else s
            out, x = [], a
            while (x <= b) if st > _dt.timedelta(0) else (x >= b):
                out.append(x)
                x = x + st
            return out
        s = (1 if b >= a else -1) if s is None else s
        if s == 0:
            return None
        return list(range(int(a), int(b) + (1 if s > 0 else -1), int(s)))
    return _arr_fn("sequence", cols, f, lambda args: T.ArrayType(args[0].dtype))


def shuffle(c: ColumnOrName, seed: Optional[int] = None) -> Column:
    def impl(frame, args):
        vals = _py(args[0])
        ids = frame._row_ids.cpu().tolist()
        out = []
        for v, rid in zip(vals, ids):
            if v is None:
                out.append(None)
                continue
            r = _random.Random((seed or 0) * 1_000_003 + rid)
            w = list(v)
            r.shuffle(w)
            out.append(w)
        return _from_values(out, args[0].dtype, frame)
    return Column(Func("shuffle", [_e(c)], impl))


def slice(x: ColumnOrName, start, length) -> Column:  # noqa: A001
    def impl(frame, args):
        vals, ss, ls = _py(args[0]), _py(args[1]), _py(args[2])
        out = []
        for v, s, n in zip(vals, ss, ls):
            if v is None or s is None or n is None:
                out.append(None)
                continue
            s, n = int(s), int(n)
            if s == 0:
                raise ValueError("slice: SQL array indices start at 1")
            a = s - 1 if s > 0 else len(v) + s
            out.append(list(v[builtins.max(a, 0):builtins.max(a, 0) + n]) if a >= 0 or a + n > 0 else [])
        return _from_values(out, args[0].dtype, frame)
    return Column(Func("slice", [_e(x), _e(start), _e(length)], impl))


def array_append(c: ColumnOrName, value) -> Column:
    return _arr_fn("array_append", [c], lambda a: list(a) + [value], _same) if not isinstance(value, (str, Column)) \
        else _arr_fn("array_append", [c, value], lambda a, v: list(a) + [v], _same)


def array_prepend(c: ColumnOrName, value) -> Column:
    return _arr_fn("array_prepend", [c], lambda a: [value] + list(a), _same) if not isinstance(value, (str, Column)) \
        else _arr_fn("array_prepend", [c, value], lambda a, v: [v] + list(a), _same)


def array_compact(c: ColumnOrName) -> Column:
    return _arr_fn("array_compact", [c], lambda a: [x for x in a if x is not None], _same)


def array_size(c: ColumnOrName) -> Column:
    return _arr_fn("array_size", [c], lambda a: len(a), lambda args: T.IntegerType())


def cardinality(c: ColumnOrName) -> Column:
    from .functions_more import size
    return size(c)


def array_insert(arr: ColumnOrName, pos, value) -> Column:
    def f(a):
        p = int(pos)
        w = list(a)
        i = p - 1 if p > 0 else len(w) + p + 1
        if i > len(w):
            w += [None] * (i - len(w))
        w.insert(builtins.max(i, 0), value)
        return w
    return _arr_fn("array_insert", [arr], f, _same)


# ------------------------------------------------------------------------------------------ maps / structs

def create_map(*cols) -> Column:
    if len(cols) == 1 and isinstance(cols[0], (list, tuple)):
        cols = tuple(cols[0])
    if len(cols) % 2:
        raise ValueError("create_map needs an even number of columns (key, value, ...)")

    def impl(frame, args):
        pys = [_py(a) for a in args]
        out = []
        for i in range(frame._nrows):
            m = {}
            for j in range(0, len(pys), 2):
                k = pys[j][i]
                if k is None:
                    raise ValueError("create_map: map keys cannot be null")
                m[k] = pys[j + 1][i]
            out.append(m)
        kt = args[0].dtype if args else T.StringType()
        vt = args[1].dtype if len(args) > 1 else T.StringType()
        return _from_values(out, T.MapType(kt, vt), frame)
    return Column(Func("map", [_e(c) for c in cols], impl))


def map_from_arrays(col1: ColumnOrName, col2: ColumnOrName) -> Column:
    def f(k, v):
        if len(k) != len(v):
            raise ValueError("map_from_arrays: key and value arrays differ in length")
        return dict(zip(k, v))
    return _arr_fn("map_from_arrays", [col1, col2], f, lambda args: T.MapType(_elem(args[0]), _elem(args[1])))


def map_from_entries(c: ColumnOrName) -> Column:
    def f(a):
        return {(e[0] if not hasattr(e, "asDict") else e[0]): e[1] for e in a}
    return _arr_fn("map_from_entries", [c], f, lambda args: T.MapType(
        _elem(args[0]).fields[0].dataType, _elem(args[0]).fields[1].dataType)
        if isinstance(_elem(args[0]), T.StructType) else T.MapType(T.StringType(), T.StringType()))


def map_keys(c: ColumnOrName) -> Column:
    return _arr_fn("map_keys", [c], lambda m: list(m.keys()), lambda args: T.ArrayType(args[0].dtype.keyType))


def map_values(c: ColumnOrName) -> Column:
    return _arr_fn("map_values", [c], lambda m: list(m.values()), lambda args: T.ArrayType(args[0].dtype.valueType))


def map_entries(c: ColumnOrName) -> Column:
    from .types import Row

    def rt(args):
        mt = args[0].dtype
        return T.ArrayType(T.StructType([T.StructField("key", mt.keyType, False),
                                         T.StructField("value", mt.valueType, True)]))
    return _arr_fn("map_entries", [c], lambda m: [Row(key=k, value=v) for k, v in m.items()], rt)


def map_concat(*cols) -> Column:
    if len(cols) == 1 and isinstance(cols[0], (list, tuple)):
        cols = tuple(cols[0])

    def f(*ms):
        out = {}
        for m in ms:
            for k, v in m.items():
                if k in out:
                    raise ValueError(f"map_concat: duplicate map key {k!r}")
                out[k] = v
        return out
    return _arr_fn("map_concat", list(cols), f, _same)


def map_contains_key(c: ColumnOrName, value) -> Column:
    return _arr_fn("map_contains_key", [c], lambda m: value in m, lambda args: T.BooleanType())


def named_struct(*cols) -> Column:
    """named_struct(lit('a'), col1, lit('b'), col2, ...)."""
    if len(cols) % 2:
        raise ValueError("named_struct needs name / value pairs")
    from .functions_more import struct
    names = []
    for n in cols[0::2]:
        e = _e(n)
        names.append(e.value if isinstance(e, Lit) else str(n))
    return struct(*[Column(_e(v)).alias(nm) for nm, v in zip(names, cols[1::2])])


# ------------------------------------------------------------------------------------------ higher-order functions

def _nargs(f: Callable) -> int:
    try:
        return len([p for p in inspect.signature(f).parameters.values()
                    if p.default is inspect.Parameter.empty and p.kind in (p.POSITIONAL_ONLY, p.POSITIONAL_OR_KEYWORD)])
    except (TypeError, ValueError):
        return 1


def _lambda_frame(frame, rep: List[int], extra: Dict[str, ColumnData]):
    idx = torch.as_tensor(rep, dtype=torch.int64, device=frame._device)
    base = frame._take_rows(idx)
    names = list(base.columns) + list(extra)
    datas = [base._cols[c] for c in base.columns] + list(extra.values())
    return base._from_columns(names, datas)


def _flatten(vals, is_map=False):
    rep, elems, pos = [], [], []
    for i, v in enumerate(vals):
        if v is None:
            continue
        items = list(v.items()) if is_map else list(v)
        for j, e in enumerate(items):
            rep.append(i)
            elems.append(e)
            pos.append(j)
    return rep, elems, pos


def _regroup(n, vals, rep, results):
    out = [None if v is None else [] for v in vals]
    for r, x in zip(rep, results):
        out[r].append(x)
    return out


def _lambda_str(fn: Callable, names: List[str]) -> str:
    """Spark-style ``lambdafunction(body, x, y)`` text of a lambda, for the output column name."""
    k = builtins.max(1, builtins.min(_nargs(fn), len(names)))
    try:
        body = _e(fn(*[Column(ColRef(n)) for n in names[:k]]))
    except Exception:  # noqa: BLE001 — naming only
        return "lambdafunction"
    return f"lambdafunction({body}, {', '.join(names[:k])})"


def _hof(col: Column, *lams) -> Column:
    col._expr.params = [_lambda_str(f, names) for f, names in lams if f is not None]
    return col


def _apply_elements(frame, arr: ColumnData, fn: Callable):
    """(parent row of each element, element values, lambda results column) for an array column."""
    vals = _py(arr)
    rep, elems, pos = _flatten(vals)
    et = _elem(arr)
    extra = {"__hof_x": _from_values(elems, et, frame), "__hof_i": _from_values(pos, T.IntegerType(), frame)}
    tmp = _lambda_frame(frame, rep, extra)
    args = [Column(ColRef("__hof_x")), Column(ColRef("__hof_i"))][:builtins.max(1, _nargs(fn))]
    res = _e(fn(*args)).eval(tmp)
    return vals, rep, elems, res


def transform(col: ColumnOrName, f: Callable) -> Column:
    """Apply ``f(x)`` or ``f(x, i)`` to every element (one vectorised evaluation)."""
    def impl(frame, args):
        vals, rep, _, res = _apply_elements(frame, args[0], f)
        return _from_values(_regroup(frame._nrows, vals, rep, _py(res)), T.ArrayType(res.dtype), frame)
    return _hof(Column(Func("transform", [_e(col)], impl)), (f, ["x", "i"]))


def filter(col: ColumnOrName, f: Callable) -> Column:  # noqa: A001
    def impl(frame, args):
        vals, rep, elems, res = _apply_elements(frame, args[0], f)
        keep = _py(res)
        out = [None if v is None else [] for v in vals]
        for r, e, k in zip(rep, elems, keep):
            if k:
                out[r].append(e)
        return _from_values(out, args[0].dtype, frame)
    return _hof(Column(Func("filter", [_e(col)], impl)), (f, ["x", "i"]))


def exists(col: ColumnOrName, f: Callable) -> Column:
    def impl(frame, args):
        vals, rep, _, res = _apply_elements(frame, args[0], f)
        out = [None if v is None else False for v in vals]
        unknown = [False] * len(vals)
        for r, k in zip(rep, _py(res)):
            if k:
                out[r] = True
            elif k is None:
                unknown[r] = True
        out = [None if (o is False and u) else o for o, u in zip(out, unknown)]
        return _from_values(out, T.BooleanType(), frame)
    return _hof(Column(Func("exists", [_e(col)], impl)), (f, ["x"]))


def forall(col: ColumnOrName, f: Callable) -> Column:
    def impl(frame, args):
        vals, rep, _, res = _apply_elements(frame, args[0], f)
        out = [None if v is None else True for v in vals]
        unknown = [False] * len(vals)
        for r, k in zip(rep, _py(res)):
            if k is False:
                out[r] = False
            elif k is None:
                unknown[r] = True
        out = [None if (o is True and u) else o for o, u in zip(out, unknown)]
        return _from_values(out, T.BooleanType(), frame)
    return _hof(Column(Func("forall", [_e(col)], impl)), (f, ["x"]))


def aggregate(col: ColumnOrName, initialValue, merge: Callable, finish: Optional[Callable] = None) -> Column:
    """Fold ``merge(acc, x)`` over each array from ``initialValue``, then ``finish(acc)``."""
    def impl(frame, args):
        arr, init = args
        vals = _py(arr)
        acc = _py(init)
        acc_t = init.dtype
        et = _elem(arr)
        longest = builtins.max((len(v) for v in vals if v is not None), default=0)
        for j in range(longest):
            rows = [i for i, v in enumerate(vals) if v is not None and len(v) > j]
            tmp = _lambda_frame(frame, rows, {"__hof_acc": _from_values([acc[i] for i in rows], acc_t, frame),
                                              "__hof_x": _from_values([vals[i][j] for i in rows], et, frame)})
            res = _e(merge(Column(ColRef("__hof_acc")), Column(ColRef("__hof_x")))).eval(tmp)
            acc_t = res.dtype if not isinstance(res.dtype, T.NullType) else acc_t
            for i, r in zip(rows, _py(res)):
                acc[i] = r
        acc = [None if v is None else a for v, a in zip(vals, acc)]
        if finish is None:
            return _from_values(acc, acc_t, frame)
        tmp = _lambda_frame(frame, list(range(frame._nrows)), {"__hof_acc": _from_values(acc, acc_t, frame)})
        res = _e(finish(Column(ColRef("__hof_acc")))).eval(tmp)
        out = [None if v is None else r for v, r in zip(vals, _py(res))]
        return _from_values(out, res.dtype, frame)
    return _hof(Column(Func("aggregate", [_e(col), _e(initialValue)], impl)), (merge, ["acc", "x"]),
                (finish, ["acc"]))


reduce = aggregate


def zip_with(left: ColumnOrName, right: ColumnOrName, f: Callable) -> Column:
    def impl(frame, args):
        a, b = _py(args[0]), _py(args[1])
        rep, xs, ys = [], [], []
        for i, (u, v) in enumerate(zip(a, b)):
            if u is None or v is None:
                continue
            for j in range(builtins.max(len(u), len(v))):
                rep.append(i)
                xs.append(u[j] if j < len(u) else None)
                ys.append(v[j] if j < len(v) else None)
        tmp = _lambda_frame(frame, rep, {"__hof_x": _from_values(xs, _elem(args[0]), frame),
                                         "__hof_y": _from_values(ys, _elem(args[1]), frame)})
        res = _e(f(Column(ColRef("__hof_x")), Column(ColRef("__hof_y")))).eval(tmp)
        vals = [None if (u is None or v is None) else [] for u, v in zip(a, b)]
        return _from_values(_regroup(frame._nrows, vals, rep, _py(res)), T.ArrayType(res.dtype), frame)
    return _hof(Column(Func("zip_with", [_e(left), _e(right)], impl)), (f, ["x", "y"]))


def _apply_entries(frame, m: ColumnData, fn: Callable):
    vals = _py(m)
    rep, items, _ = _flatten(vals, is_map=True)
    mt = m.dtype
    tmp = _lambda_frame(frame, rep, {"__hof_k": _from_values([k for k, _ in items], mt.keyType, frame),
                                     "__hof_v": _from_values([v for _, v in items], mt.valueType, frame)})
    res = _e(fn(Column(ColRef("__hof_k")), Column(ColRef("__hof_v")))).eval(tmp)
    return vals, rep, items, res


def map_filter(col: ColumnOrName, f: Callable) -> Column:
    def impl(frame, args):
        vals, rep, items, res = _apply_entries(frame, args[0], f)
        out = [None if v is None else {} for v in vals]
        for r, (k, v), keep in zip(rep, items, _py(res)):
            if keep:
                out[r][k] = v
        return _from_values(out, args[0].dtype, frame)
    return _hof(Column(Func("map_filter", [_e(col)], impl)), (f, ["k", "v"]))


def transform_values(col: ColumnOrName, f: Callable) -> Column:
    def impl(frame, args):
        vals, rep, items, res = _apply_entries(frame, args[0], f)
        out = [None if v is None else {} for v in vals]
        for r, (k, _), nv in zip(rep, items, _py(res)):
            out[r][k] = nv
        return _from_values(out, T.MapType(args[0].dtype.keyType, res.dtype), frame)
    return _hof(Column(Func("transform_values", [_e(col)], impl)), (f, ["k", "v"]))


def transform_keys(col: ColumnOrName, f: Callable) -> Column:
    def impl(frame, args):
        vals, rep, items, res = _apply_entries(frame, args[0], f)
        out = [None if v is None else {} for v in vals]
        for r, (_, v), nk in zip(rep, items, _py(res)):
            if nk is None:
                raise ValueError("transform_keys: map keys cannot be null")
            if nk in out[r]:
                raise ValueError(f"transform_keys: duplicate map key {nk!r}")
            out[r][nk] = v
        return _from_values(out, T.MapType(res.dtype, args[0].dtype.valueType), frame)
    return _hof(Column(Func("transform_keys", [_e(col)], impl)), (f, ["k", "v"]))


def map_zip_with(col1: ColumnOrName, col2: ColumnOrName, f: Callable) -> Column:
    def impl(frame, args):
        a, b = _py(args[0]), _py(args[1])
        rep, ks, xs, ys = [], [], [], []
        for i, (u, v) in enumerate(zip(a, b)):
            if u is None or v is None:
                continue
            for k in list(dict.fromkeys(list(u) + list(v))):
                rep.append(i)
                ks.append(k)
                xs.append(u.get(k))
                ys.append(v.get(k))
        mt1, mt2 = args[0].dtype, args[1].dtype
        tmp = _lambda_frame(frame, rep, {"__hof_k": _from_values(ks, mt1.keyType, frame),
                                         "__hof_x": _from_values(xs, mt1.valueType, frame),
                                         "__hof_y": _from_values(ys, mt2.valueType, frame)})
        res = _e(f(Column(ColRef("__hof_k")), Column(ColRef("__hof_x")), Column(ColRef("__hof_y")))).eval(tmp)
        out = [None if (u is None or v is None) else {} for u, v in zip(a, b)]
        for r, k, nv in zip(rep, ks, _py(res)):
            out[r][k] = nv
        return _from_values(out, T.MapType(mt1.keyType, res.dtype), frame)
    return _hof(Column(Func("map_zip_with", [_e(col1), _e(col2)], impl)), (f, ["k", "v1", "v2"]))


# ------------------------------------------------------------------------------------------ JSON

def _schema_of(schema) -> T.DataType:
    if isinstance(schema, T.DataType):
        return schema
    if isinstance(schema, Column):
        e = schema._expr
        schema = e.value if isinstance(e, Lit) else str(e)
    s = str(schema).strip()
    if s.lower().startswith(("array<", "map<", "struct<")):
        return T.parse_type(s)
    return T.parse_ddl_schema(s)


def _typed(v, dt: T.DataType):
    """JSON value -> Python value of Spark type ``dt`` (None when it does not fit)."""
    from .column import micros_to_datetime, ts_to_micros
    from .types import Row
    if v is None:
        return None
    try:
        if isinstance(dt, T.StructType):
            if not isinstance(v, dict):
                return None
            return Row(**{f.name: _typed(v.get(f.name), f.dataType) for f in dt.fields})
        if isinstance(dt, T.ArrayType):
            return [_typed(x, dt.elementType) for x in v] if isinstance(v, list) else None
        if isinstance(dt, T.MapType):
            return {str(k): _typed(x, dt.valueType) for k, x in v.items()} if isinstance(v, dict) else None
        if isinstance(dt, T.BooleanType):
            return v if isinstance(v, bool) else None
        if T.is_integral(dt):
            return int(v) if isinstance(v, int) and not isinstance(v, bool) else None
        if isinstance(dt, (T.FloatType, T.DoubleType, T.DecimalType)):
            return float(v) if isinstance(v, (int, float)) and not isinstance(v, bool) else None
        if isinstance(dt, T.TimestampType):
            return micros_to_datetime(ts_to_micros(str(v)))
        if isinstance(dt, T.DateType):
            return micros_to_datetime(ts_to_micros(str(v))).date()
        if isinstance(dt, T.StringType):
            return v if isinstance(v, str) else json.dumps(v, separators=(",", ":"))
    except (ValueError, TypeError):
        return None
    return v


def from_json(col: ColumnOrName, schema, options: Optional[Dict[str, str]] = None) -> Column:
    dt = _schema_of(schema)

    def f(s):
        try:
            v = json.loads(s)
        except (ValueError, TypeError):
            return None
        return _typed(v, dt)
    return _host_map("from_json", [col], f, dt)


def _jsonable(v):
    from .types import Row
    if isinstance(v, Row):
        return {k: _jsonable(x) for k, x in v.asDict().items() if x is not None}
    if isinstance(v, dict):
        return {str(k): _jsonable(x) for k, x in v.items()}
    if isinstance(v, (list, tuple)):
        return [_jsonable(x) for x in v]
    if isinstance(v, _dt.datetime):
        return v.strftime("%Y-%m-%dT%H:%M:%S.") + f"{v.microsecond // 1000:03d}Z"
    if isinstance(v, _dt.date):
        return v.isoformat()
    if hasattr(v, "toArray"):
        return {"type": 1, "values": [float(x) for x in v.toArray()]}
    if isinstance(v, float) and (math.isnan(v) or math.isinf(v)):
        return str(v).replace("inf", "Infinity").replace("nan", "NaN")
    return v


def to_json(col: ColumnOrName, options: Optional[Dict[str, str]] = None) -> Column:
    return _host_map("to_json", [col], lambda v: json.dumps(_jsonable(v), separators=(",", ":"),
                                                            ensure_ascii=False), T.StringType())


def _json_path(obj, path: str):
    if not path.startswith("$"):
        return None
    toks = re.findall(r"\.([^.\[\]]+)|\[(\d+|\*)\]|\['([^']+)'\]", path[1:])
    cur = [obj]
    wildcard = False
    for name, idx, qname in toks:
        nxt = []
        for o in cur:
            if name or qname:
                key = name or qname
                if key == "*" and isinstance(o, dict):
                    nxt.extend(o.values())
                    wildcard = True
                elif isinstance(o, dict) and key in o:
                    nxt.append(o[key])
            elif idx == "*":
                if isinstance(o, list):
                    nxt.extend(o)
                    wildcard = True
            elif isinstance(o, list) and int(idx) < len(o):
                nxt.append(o[int(idx)])
        cur = nxt
    if not cur:
        return None
    return cur if wildcard else cur[0]


def get_json_object(col: ColumnOrName, path: str) -> Column:
    def f(s):
        try:
            v = _json_path(json.loads(s), path)
        except (ValueError, TypeError):
            return None
        if v is None:
            return None
        return v if isinstance(v, str) else json.dumps(v, separators=(",", ":"))
    return _host_map("get_json_object", [col], f, T.StringType())


def schema_of_json(json_str, options: Optional[Dict[str, str]] = None) -> Column:
    from .functions import lit
    e = _e(json_str)
    text = e.value if isinstance(e, Lit) else str(json_str)

    def infer(v) -> str:
        if isinstance(v, bool):
            return "BOOLEAN"
        if isinstance(v, int):
            return "BIGINT"
        if isinstance(v, float):
            return "DOUBLE"
        if isinstance(v, list):
            return f"ARRAY<{infer(v[0]) if v else 'STRING'}>"
        if isinstance(v, dict):
            return "STRUCT<" + ", ".join(f"{k}: {infer(x)}" for k, x in sorted(v.items())) + ">"
        return "STRING"
    return lit(infer(json.loads(text)))


def json_object_keys(col: ColumnOrName) -> Column:
    def f(s):
        try:
            v = json.loads(s)
        except (ValueError, TypeError):
            return None
        return list(v.keys()) if isinstance(v, dict) else None
    return _host_map("json_object_keys", [col], f, T.ArrayType(T.StringType()))


def json_array_length(col: ColumnOrName) -> Column:
    def f(s):
        try:
            v = json.loads(s)
        except (ValueError, TypeError):
            return None
        return len(v) if isinstance(v, list) else None
    return _host_map("json_array_length", [col], f, T.IntegerType())


# ------------------------------------------------------------------------------------------ grouping sets

class GroupingMarker(Expr):
    """``grouping(col)`` / ``grouping_id(cols...)`` inside ``rollup`` / ``cube`` aggregations: resolved
    per grouping set by MultiGroupedData (1 where the column is rolled up)."""

    def __init__(self, kind: str, cols: List[str]):
        self.kind, self.cols = kind, cols

    def refs(self):
        return list(self.cols)

    def name(self):
        return f"{self.kind}({', '.join(self.cols)})"

    __str__ = name

    def is_aggregate(self):
        return True

    def eval(self, frame):
        raise ValueError(f"{self.kind}() can only be used with GroupingSets/Cube/Rollup")

    def value(self, keys: List[str], in_set: List[str]):
        if self.kind == "grouping":
            return (0 if self.cols[0] in in_set else 1), T.ByteType()
        cols = self.cols or keys
        v = 0
        for c in cols:
            v = (v << 1) | (0 if c in in_set else 1)
        return v, T.LongType()


def grouping(col: ColumnOrName) -> Column:
    return Column(GroupingMarker("grouping", [col if isinstance(col, str) else _e(col).name()]))


def grouping_id(*cols: ColumnOrName) -> Column:
    return Column(GroupingMarker("grouping_id", [c if isinstance(c, str) else _e(c).name() for c in cols]))


# ------------------------------------------------------------------------------------------ misc

def broadcast(df):
    """Broadcast-join hint: joins here already replicate the smaller side, so this is the frame."""
    return df


def input_file_name() -> Column:
    """The source file of each row: recorded by the file readers as hidden metadata when present,
    else the empty string (Spark's value for non-file sources)."""
    def impl(frame, args):
        out = np.empty(frame._nrows, dtype=object)
        src = getattr(frame, "_input_files", None)
        out[:] = ""
        if src is not None:
            out[:] = src(frame)
        return ColumnData(out, None, T.StringType())
    return Column(Func("input_file_name", [], impl))


def spark_partition_id() -> Column:
    """The rank holding the row (a rank is this framework's partition)."""
    def impl(frame, args):
        return ColumnData(torch.full((frame._nrows,), frame._comm.rank, dtype=torch.int32, device=frame._device),
                          None, T.IntegerType())
    return Column(Func("SPARK_PARTITION_ID()", [], impl))


def asc_nulls_first(c: ColumnOrName):
    return Column(_e(c)).asc_nulls_first()


def asc_nulls_last(c: ColumnOrName):
    return Column(_e(c)).asc_nulls_last()


def desc_nulls_first(c: ColumnOrName):
    return Column(_e(c)).desc_nulls_first()


def desc_nulls_last(c: ColumnOrName):
    return Column(_e(c)).desc_nulls_last()


def inline(c: ColumnOrName) -> Column:
    """Explode an array of structs into one row per element and one column per struct field."""
    from .functions_more import Generator
    return Column(Generator("inline", _e(c)))


def inline_outer(c: ColumnOrName) -> Column:
    from .functions_more import Generator
    return Column(Generator("inline_outer", _e(c)))


def json_tuple(col: ColumnOrName, *fields: str) -> Column:
    """One row per input row with columns c0, c1, ... holding the top-level ``fields`` of a JSON
    object (as strings)."""
    from .functions_more import Generator
    g = Generator("json_tuple", _e(col))
    g.fields = list(fields)
    return Column(g)


__all__ = [n for n in dir() if not n.startswith("_") and n not in (
    "annotations", "builtins", "inspect", "json", "math", "np", "re", "torch", "T", "Any", "Callable", "Dict",
    "List", "Optional", "ColRef", "Column", "ColumnData", "Expr", "Func", "Lit", "UserDefinedFunction",
    "ColumnOrName")]
