"""pyspark.sql.functions-compatible builders.

The reference imports ``current_timestamp`` and ``when`` (ref.py:28) and uses
them at ref.py:82 and ref.py:176-177; the rest are the commonly used siblings.
"""
from __future__ import annotations

import builtins
import time
from typing import Iterable, Union

import numpy as np
import torch

from . import types as T
from .column import (AggExpr, Alias, BinOp, Cast, ColRef, Column, ColumnData, Expr, Func, Lit, Unary, When,
                     _expr, ts_to_micros)

ColumnOrName = Union[Column, str]


def _c(x: ColumnOrName) -> Expr:
    return ColRef(x) if isinstance(x, str) else _expr(x)


def col(name: str) -> Column:
    return Column(ColRef(name))


column = col


def lit(value) -> Column:
    return value if isinstance(value, Column) else Column(Lit(value))


def when(condition: Column, value) -> Column:
    return Column(When([(_expr(condition), _expr(value))]))


def expr(sql: str) -> Column:
    from .sqlparse import parse_expression
    return Column(parse_expression(sql))


def current_timestamp() -> Column:
    """One timestamp per evaluation (Spark: one value per micro-batch / query, ref.py:82)."""
    def impl(frame, args):
        now = getattr(frame, "_batch_time_us", None)
        if now is None:
            now = int(time.time() * 1e6)
        return ColumnData(torch.full((frame._nrows,), now, dtype=torch.int64, device=frame._device), None,
                          T.TimestampType())
    return Column(Alias(Func("current_timestamp", [], impl), "current_timestamp()"))


def current_date() -> Column:
    def impl(frame, args):
        days = int(time.time() // 86400)
        return ColumnData(torch.full((frame._nrows,), days, dtype=torch.int32, device=frame._device), None,
                          T.DateType())
    return Column(Func("current_date", [], impl))


def to_timestamp(c: ColumnOrName, fmt: str = None) -> Column:
    """Cast to timestamp; with ``fmt`` parse strings with that Spark datetime pattern (null when a
    value does not match)."""
    if fmt is None:
        return Column(Cast(_c(c), T.TimestampType()))
    from .datetimefmt import parser
    p = parser(fmt)
    return _host_map("to_timestamp", [c], lambda s: p(s) if isinstance(s, str) else _as_datetime(s),
                     T.TimestampType(), params=[fmt])


def monotonically_increasing_id() -> Column:
    """Unique 64-bit ids: the frame's global row ids (stable across GPU counts)."""
    def impl(frame, args):
        return ColumnData(frame._row_ids.clone(), None, T.LongType())
    return Column(Func("monotonically_increasing_id", [], impl))


def rand(seed: int = 0) -> Column:
    from ..utils import rng

    def impl(frame, args):
        return ColumnData(rng.uniform(frame._row_ids, seed, stream=7), None, T.DoubleType())
    return Column(Func(f"rand({seed})", [], impl))


def _unary(op):
    def f(c: ColumnOrName) -> Column:
        return Column(Unary(op, _c(c)))
    f.__name__ = op
    return f


abs = _unary("abs")  # noqa: A001
sqrt = _unary("sqrt")
exp = _unary("exp")
log = _unary("log")
log10 = _unary("log10")
log2 = _unary("log2")
floor = _unary("floor")
ceil = _unary("ceil")
sin = _unary("sin")
cos = _unary("cos")
tanh = _unary("tanh")
signum = _unary("signum")
upper = _unary("upper")
lower = _unary("lower")
trim = _unary("trim")
length = _unary("length")
year = _unary("year")
month = _unary("month")
dayofmonth = _unary("dayofmonth")
dayofweek = _unary("dayofweek")
hour = _unary("hour")
minute = _unary("minute")
second = _unary("second")


def isnull(c: ColumnOrName) -> Column:
    return Column(Unary("isnull", _c(c)))


def isnan(c: ColumnOrName) -> Column:
    return Column(Unary("isnan", _c(c)))


def round(c: ColumnOrName, scale: int = 0) -> Column:  # noqa: A001
    def impl(frame, args):
        a = args[0]
        v = a.values.to(torch.float64)
        f = 10.0 ** scale
        # Spark rounds HALF_UP
        out = torch.sign(v) * torch.floor(torch.abs(v) * f + 0.5) / f
        return ColumnData(out, a.valid, T.DoubleType())
    return Column(Func(f"round({scale})", [_c(c)], impl))


def coalesce(*cols: ColumnOrName) -> Column:
    def impl(frame, args):
        if any(a.is_host for a in args):
            from .column import _to_host
            hs = [_to_host(a) for a in args]
            out = np.empty(frame._nrows, dtype=object)
            vm = np.zeros(frame._nrows, dtype=bool)
            for h in hs:
                take = ~vm & h.valid_mask() & np.array([v is not None for v in h.values])
                out[take] = h.values[take]
                vm |= take
            return ColumnData(out, vm, hs[0].dtype)
        out = args[-1].values.clone()
        vm = args[-1].valid_mask().clone()
        for a in reversed(args[:-1]):
            m = a.valid_mask()
            out = torch.where(m, a.values.to(out.dtype), out)
            vm = vm | m
        return ColumnData(out, vm, args[0].dtype)
    return Column(Func("coalesce", [_c(c) for c in cols], impl))


def greatest(*cols: ColumnOrName) -> Column:
    def impl(frame, args):
        out = args[0].values.to(torch.float64)
        for a in args[1:]:
            out = torch.maximum(out, a.values.to(torch.float64))
        vm = args[0].valid_mask()
        for a in args[1:]:
            vm = vm & a.valid_mask()
        return ColumnData(out, vm, T.DoubleType())
    return Column(Func("greatest", [_c(c) for c in cols], impl))


def least(*cols: ColumnOrName) -> Column:
    def impl(frame, args):
        out = args[0].values.to(torch.float64)
        for a in args[1:]:
            out = torch.minimum(out, a.values.to(torch.float64))
        vm = args[0].valid_mask()
        for a in args[1:]:
            vm = vm & a.valid_mask()
        return ColumnData(out, vm, T.DoubleType())
    return Column(Func("least", [_c(c) for c in cols], impl))


def concat(*cols: ColumnOrName) -> Column:
    def impl(frame, args):
        from .column import _to_host
        hs = [_to_host(a) for a in args]
        out = np.empty(frame._nrows, dtype=object)
        vm = np.ones(frame._nrows, dtype=bool)
        for h in hs:
            vm &= h.valid_mask()
        for i in range(frame._nrows):
            out[i] = "".join(str(h.values[i]) for h in hs) if vm[i] else None
        return ColumnData(out, vm, T.StringType())
    return Column(Func("concat", [_c(c) for c in cols], impl))


# ------------------------------------------------------------------------------------------------ aggregates

def count(c: ColumnOrName = None) -> Column:
    if c is None or (isinstance(c, str) and c == "*"):
        return Column(AggExpr("count", None))
    return Column(AggExpr("count", _c(c)))


def countDistinct(c: ColumnOrName, *more) -> Column:
    return Column(AggExpr("count", _c(c), distinct=True))


count_distinct = countDistinct


def sum(c: ColumnOrName) -> Column:  # noqa: A001
    return Column(AggExpr("sum", _c(c)))


def avg(c: ColumnOrName) -> Column:
    return Column(AggExpr("avg", _c(c)))


mean = avg


def min(c: ColumnOrName) -> Column:  # noqa: A001
    return Column(AggExpr("min", _c(c)))


def max(c: ColumnOrName) -> Column:  # noqa: A001
    return Column(AggExpr("max", _c(c)))


def stddev(c: ColumnOrName) -> Column:
    return Column(AggExpr("stddev", _c(c)))


stddev_samp = stddev


def stddev_pop(c: ColumnOrName) -> Column:
    return Column(AggExpr("stddev_pop", _c(c)))


def variance(c: ColumnOrName) -> Column:
    return Column(AggExpr("variance", _c(c)))


var_samp = variance


def var_pop(c: ColumnOrName) -> Column:
    return Column(AggExpr("var_pop", _c(c)))


def first(c: ColumnOrName, ignorenulls: bool = False) -> Column:
    """Spark's first(col, ignorenulls=False): the value of the group's first row in row order (null
    included); with ignorenulls the first non-null value."""
    return Column(AggExpr("first", _c(c), ignore_nulls=ignorenulls))


def last(c: ColumnOrName, ignorenulls: bool = False) -> Column:
    """Spark's last(col, ignorenulls=False): the group's last row's value (null included); with
    ignorenulls the last non-null value."""
    return Column(AggExpr("last", _c(c), ignore_nulls=ignorenulls))


def collect_list(c: ColumnOrName) -> Column:
    return Column(AggExpr("collect_list", _c(c)))


def collect_set(c: ColumnOrName) -> Column:
    return Column(AggExpr("collect_set", _c(c)))


def approx_count_distinct(c: ColumnOrName, rsd: float = 0.05) -> Column:
    """Exact distinct count (a valid answer for any rsd; Spark uses HyperLogLog++)."""
    return Column(AggExpr("count", _c(c), distinct=True))


def percentile_approx(c: ColumnOrName, percentage, accuracy: int = 10000) -> Column:
    """Spark's percentile_approx on the exact sorted values: the smallest value whose rank reaches
    ceil(p * n) (what the approximate algorithm converges to). ``percentage`` may be a list."""
    e = AggExpr("percentile", _c(c))
    e.arg = percentage
    return Column(e)


# ------------------------------------------------------------------------------------------------ window functions

def window(timeColumn: ColumnOrName, windowDuration: str, slideDuration: str = None, startTime: str = None) -> Column:
    """Event-time buckets (tumbling, or sliding with ``slideDuration``) as struct<start, end>."""
    from .window import TimeWindow, parse_duration_us
    dur = parse_duration_us(windowDuration)
    slide = parse_duration_us(slideDuration) if slideDuration else dur
    start = parse_duration_us(startTime) if startTime else 0
    return Column(TimeWindow(_c(timeColumn), dur, slide, start))

def _wf(fn, child=None, arg=None, default=None) -> Column:
    from .window import WindowFunc
    return Column(WindowFunc(fn, child, arg, default))


def row_number() -> Column:
    return _wf("row_number")


def rank() -> Column:
    return _wf("rank")


def dense_rank() -> Column:
    return _wf("dense_rank")


def percent_rank() -> Column:
    return _wf("percent_rank")


def cume_dist() -> Column:
    return _wf("cume_dist")


def ntile(n: int) -> Column:
    if int(n) < 1:
        raise ValueError("ntile needs n >= 1")
    return _wf("ntile", None, int(n))


def lag(c: ColumnOrName, offset: int = 1, default=None) -> Column:
    return _wf("lag", _c(c), int(offset), default)


def lead(c: ColumnOrName, offset: int = 1, default=None) -> Column:
    return _wf("lead", _c(c), int(offset), default)


# ------------------------------------------------------------------------------------------------ UDFs

def _return_type(rt) -> T.DataType:
    if rt is None:
        return T.StringType()
    if isinstance(rt, T.DataType):
        return rt
    return T.parse_type(str(rt))


class UserDefinedFunction:
    """pyspark ``udf``: a Python function applied row by row on the host (rank-local shard).

    Nulls are passed as ``None``; the result is converted to ``returnType`` and moved back to
    the frame's device when that type is device-resident. Use ``pandas_udf`` for vectorised
    functions — both are host fallbacks, the GPU never runs Python.
    """

    def __init__(self, func, returnType=None, vectorized: bool = False, name: str = None):
        self.func = func
        self.returnType = _return_type(returnType)
        self.vectorized = vectorized
        self.__name__ = name or getattr(func, "__name__", "udf")
        self.evalType = 200 if vectorized else 100

    def __call__(self, *cols) -> Column:
        from .builder import column_from_values
        from .dataframe import column_to_python
        fn, rt, vec = self.func, self.returnType, self.vectorized

        def impl(frame, args):
            pys = [column_to_python(a) for a in args]
            if vec:
                import pandas as pd
                res = fn(*[pd.Series(p) for p in pys])
                vals = list(res.tolist() if hasattr(res, "tolist") else res)
                vals = [None if (v is not None and isinstance(v, float) and v != v and not isinstance(
                    rt, (T.DoubleType, T.FloatType))) else v for v in vals]
            else:
                vals = [fn(*row) for row in zip(*pys)] if pys else [fn() for _ in range(frame._nrows)]
            if len(vals) != frame._nrows:
                raise ValueError(f"UDF {self.__name__} returned {len(vals)} values for {frame._nrows} rows")
            return column_from_values(vals, rt, frame._device)
        return Column(Func(self.__name__, [_c(c) for c in cols], impl))

    def asNondeterministic(self):
        return self


REGISTERED_UDFS: dict = {}  # name -> UserDefinedFunction, callable from SQL (spark.udf.register)


class UDFRegistration:
    """``spark.udf``: register Python functions under a SQL name."""

    def register(self, name: str, f, returnType=None):
        u = f if isinstance(f, UserDefinedFunction) else UserDefinedFunction(f, returnType, name=name)
        if returnType is not None and isinstance(f, UserDefinedFunction):
            u = UserDefinedFunction(f.func, returnType, f.vectorized, name=name)
        REGISTERED_UDFS[name.lower()] = u
        return u

    def registerJavaFunction(self, name, javaClassName, returnType=None):
        raise NotImplementedError("JVM functions are not available in this framework")


def udf(f=None, returnType=None):
    """``udf(f, returnType)`` or ``@udf(returnType=...)`` / ``@udf``."""
    if f is None or isinstance(f, (str, T.DataType)):
        rt = f if returnType is None else returnType
        return lambda fn: UserDefinedFunction(fn, rt)
    return UserDefinedFunction(f, returnType)


def pandas_udf(f=None, returnType=None, functionType=None):
    """Vectorised UDF: the function receives one pandas Series per argument (the rank's shard)."""
    if f is None or isinstance(f, (str, T.DataType)):
        rt = f if returnType is None else returnType
        return lambda fn: UserDefinedFunction(fn, rt, vectorized=True)
    return UserDefinedFunction(f, returnType, vectorized=True)


# ------------------------------------------------------------------------------------------------ strings / dates

def _closure_params(fn) -> list:
    """Scalar parameters a row function closes over (used to make output column names unique, e.g.
    ``substring_index(s, ., 2)`` vs ``substring_index(s, ., -3)``)."""
    out = []
    for cell in (getattr(fn, "__closure__", None) or ()):
        try:
            v = cell.cell_contents
        except ValueError:
            continue
        if isinstance(v, (str, int, float, bool)):
            out.append(v)
        elif isinstance(getattr(v, "pattern", None), str):
            out.append(v.pattern)
    return out


def _host_map(name, cols, fn, rt, params=None):
    """Row-wise host function over one or more columns (null in -> null out unless fn handles it).
    ``params`` (default: the scalars ``fn`` closes over) are shown in the column name."""
    def wrapped(*vals):
        return None if any(v is None for v in vals) else fn(*vals)
    col = UserDefinedFunction(wrapped, rt, name=name)(*cols)
    ps = _closure_params(fn) if params is None else list(params)
    if ps:
        col._expr.params = ps
    col._expr.impl = _per_distinct(col._expr.impl, wrapped, rt, [isinstance(a, Lit) for a in col._expr.args])
    return col


_DISTINCT_MIN_ROWS = 1024


def _per_distinct(impl, fn, rt, lits):
    """Evaluate a deterministic row function once per distinct value when its only column argument
    is dictionary-encoded (ingest / createDataFrame ``DictColumnData``): ``fn`` runs over the
    dictionary, the rows gather the results by code. String results stay dictionary-encoded."""
    col_args = [i for i, lit_ in enumerate(lits) if not lit_]

    def run(frame, args):
        from .builder import column_from_values
        from .column import DictColumnData
        from .dataframe import column_to_python
        if len(col_args) != 1 or not isinstance(args[col_args[0]], DictColumnData) or \
                len(args[col_args[0]]) < _DISTINCT_MIN_ROWS:
            return impl(frame, args)
        j = col_args[0]
        cd = args[j]
        consts = [None if i == j else (column_to_python(a)[0] if len(a) else None) for i, a in enumerate(args)]
        outs = []
        for v in cd.dictionary[:-1]:
            call = list(consts)
            call[j] = v
            outs.append(fn(*call))
        codes = cd.codes.astype(np.int64)
        if cd.valid is not None:
            codes = np.where(np.asarray(cd.valid, dtype=bool), codes, -1)
        null_out = fn(*[None if i == j else c for i, c in enumerate(consts)])
        if isinstance(rt, T.StringType):
            import pandas as pd
            from .relational_fast import _dict_column
            vals = np.empty(len(outs) + 1, dtype=object)
            vals[:-1] = outs
            vals[-1] = null_out
            rc, uniq = pd.factorize(vals, use_na_sentinel=True)
            return _dict_column(rc[codes], np.asarray(uniq, dtype=object), rt)
        table = column_from_values(outs + [null_out], rt, frame._device)
        idx = np.where(codes >= 0, codes, len(outs))
        return table.take(torch.as_tensor(idx, device=table.values.device) if not table.is_host else idx)
    return run


def substring(c: ColumnOrName, pos: int, length: int) -> Column:
    """1-based position like Spark; 0 acts as 1, a negative position counts from the end."""
    return _host_map("substring", [c], lambda s: spark_substr(str(s), pos, length), T.StringType(),
                     params=[pos, length])


def spark_substr(s: str, pos: int, length: int) -> str:
    """UTF8String.substringSQL: the window [start, start + length) is taken BEFORE clamping start at 0, so
    a negative position reaching before the string start shortens the result (substring('0', -2, 1) = '')."""
    start = pos - 1 if pos > 0 else (len(s) + pos if pos < 0 else 0)
    end = start + length
    start = builtins.max(start, 0)
    return "" if start >= end else s[start:end]


def concat_ws(sep: str, *cols: ColumnOrName) -> Column:
    def f(*vals):
        return sep.join(str(v) for v in vals if v is not None)
    return UserDefinedFunction(f, T.StringType(), name="concat_ws")(*cols)


def regexp_replace(c: ColumnOrName, pattern: str, replacement: str) -> Column:
    import re
    rx = re.compile(pattern)
    repl = re.sub(r"\$(\d+)", r"\\\1", replacement)  # Java $1 -> Python \1
    return _host_map("regexp_replace", [c], lambda s: rx.sub(repl, str(s)), T.StringType())


def regexp_extract(c: ColumnOrName, pattern: str, idx: int) -> Column:
    import re
    rx = re.compile(pattern)

    def f(s):
        m = rx.search(str(s))
        return (m.group(idx) or "") if m else ""
    return _host_map("regexp_extract", [c], f, T.StringType())


def split(c: ColumnOrName, pattern: str) -> Column:
    import re
    rx = re.compile(pattern)
    return _host_map("split", [c], lambda s: rx.split(str(s)), T.ArrayType(T.StringType()))


def lpad(c: ColumnOrName, width: int, pad: str) -> Column:
    return _host_map("lpad", [c], lambda s: (pad * width + str(s))[-width:] if len(str(s)) < width
                     else str(s)[:width], T.StringType())


def rpad(c: ColumnOrName, width: int, pad: str) -> Column:
    return _host_map("rpad", [c], lambda s: (str(s) + pad * width)[:width], T.StringType())


def _as_datetime(t):
    import datetime as _dt
    from .column import micros_to_datetime, ts_to_micros
    if isinstance(t, str):
        try:
            return micros_to_datetime(ts_to_micros(t))
        except (ValueError, TypeError):
            return None
    return t if isinstance(t, (_dt.datetime, _dt.date)) else None


def date_format(c: ColumnOrName, fmt: str) -> Column:
    """Format a date / timestamp (or a timestamp string) with a Spark datetime pattern."""
    from .datetimefmt import formatter
    f = formatter(fmt)

    def g(t):
        t = _as_datetime(t)
        return None if t is None else f(t)
    return _host_map("date_format", [c], g, T.StringType(), params=[fmt])


def _days(cd: ColumnData) -> torch.Tensor:
    if isinstance(cd.dtype, T.DateType):
        return cd.values.to(torch.int64)
    if isinstance(cd.dtype, T.TimestampType):
        return torch.div(cd.values, 86_400_000_000, rounding_mode="floor")
    raise TypeError("date function needs a date or timestamp column")


def to_date(c: ColumnOrName, fmt: str = None) -> Column:
    if fmt is not None:
        from .datetimefmt import parser
        p = parser(fmt)

        def g(s):
            t = p(s) if isinstance(s, str) else _as_datetime(s)
            return None if t is None else (t.date() if hasattr(t, "date") else t)
        return _host_map("to_date", [c], g, T.DateType(), params=[fmt])

    def impl(frame, args):
        a = args[0]
        if a.is_host or isinstance(a.dtype, T.StringType):
            return _cast_host_date(frame, a)
        return ColumnData(_days(a).to(torch.int32), a.valid, T.DateType())
    return Column(Func("to_date", [_c(c)], impl))


def _cast_host_date(frame, a):
    from .column import Cast as _Cast
    tmp = ColumnData(a.values, a.valid, a.dtype)

    class _Const(Expr):
        def eval(self, fr):
            return tmp

        def refs(self):
            return []
    return _Cast(_Const(), T.DateType()).eval(frame)


def datediff(end: ColumnOrName, start: ColumnOrName) -> Column:
    def impl(frame, args):
        e, s = args
        valid = None
        if e.valid is not None or s.valid is not None:
            valid = e.valid_mask() & s.valid_mask()
        return ColumnData((_days(e) - _days(s)).to(torch.int32), valid, T.IntegerType())
    return Column(Func("datediff", [_c(end), _c(start)], impl))


def date_add(c: ColumnOrName, days: int) -> Column:
    def impl(frame, args):
        a = args[0]
        return ColumnData((_days(a) + int(days)).to(torch.int32), a.valid, T.DateType())
    return Column(Func(f"date_add({days})", [_c(c)], impl))


def date_sub(c: ColumnOrName, days: int) -> Column:
    return date_add(c, -int(days))


def unix_timestamp(c: ColumnOrName = None, fmt: str = None) -> Column:
    if c is None:
        return Column(Func("unix_timestamp", [], lambda frame, args: ColumnData(
            torch.full((frame._nrows,), int(time.time()), dtype=torch.int64, device=frame._device), None,
            T.LongType())))

    if fmt is not None:
        from .column import ts_to_micros
        from .datetimefmt import parser
        p = parser(fmt)

        def g(s):
            t = p(s) if isinstance(s, str) else _as_datetime(s)
            return None if t is None else ts_to_micros(t) // 1_000_000
        return _host_map("unix_timestamp", [c], g, T.LongType(), params=[fmt])

    def impl(frame, args):
        a = args[0]
        if isinstance(a.dtype, T.DateType):
            return ColumnData(a.values.to(torch.int64) * 86400, a.valid, T.LongType())
        if isinstance(a.dtype, T.TimestampType):
            return ColumnData(torch.div(a.values, 1_000_000, rounding_mode="floor"), a.valid, T.LongType())
        ts = _cast_host_ts(frame, a)
        return ColumnData(torch.div(ts.values, 1_000_000, rounding_mode="floor"), ts.valid, T.LongType())
    return Column(Func("unix_timestamp", [_c(c)], impl))


def _cast_host_ts(frame, a):
    from .column import Cast as _Cast

    class _Const(Expr):
        def eval(self, fr):
            return a

        def refs(self):
            return []
    return _Cast(_Const(), T.TimestampType()).eval(frame)


def from_unixtime(c: ColumnOrName, fmt: str = "yyyy-MM-dd HH:mm:ss") -> Column:
    import datetime as _dt
    from .datetimefmt import formatter
    f = formatter(fmt)
    return _host_map("from_unixtime", [c], lambda s: f(_dt.datetime(1970, 1, 1) + _dt.timedelta(seconds=int(s))),
                     T.StringType(), params=[fmt])


from .functions_more import *  # noqa: E402,F401,F403  (statistical aggregates, math/date/string, arrays, explode)
from .functions_extra import *  # noqa: E402,F401,F403  (null helpers, hashes, time zones, collections, lambdas, JSON)
from .functions_tail import *  # noqa: E402,F401,F403  (regr_* / string_agg / bit aggregates, try_*, regex, url, date aliases)
