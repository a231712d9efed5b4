"""pyspark.sql.functions-compatible builders.

The reference imports ``current_timestamp`` and ``when`` (ref.py:28) and uses
them at ref.py:82 and ref.py:176-177; the rest are the commonly used siblings.
"""
from __future__ import annotations

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
    return Column(Cast(_c(c), T.TimestampType()))


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


def first(c: ColumnOrName) -> Column:
    return Column(AggExpr("first", _c(c)))
