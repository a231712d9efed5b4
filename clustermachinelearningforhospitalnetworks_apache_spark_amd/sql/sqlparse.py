"""Mini SQL front end (N6): tokenizer + recursive-descent parser producing Column
expressions and a tiny logical plan executed on the sharded frame.

Covers the reference's query ``SELECT * FROM t WHERE event_time BETWEEN 'a' AND 'b'``
(ref.py:123-128) and the usual siblings: projections with aliases and arithmetic,
aggregates with GROUP BY / HAVING, ORDER BY, LIMIT, DISTINCT, IN, IS [NOT] NULL,
CASE WHEN, CAST, LIKE, and function calls mapped onto ``sql.functions``.
"""
from __future__ import annotations

import re
from dataclasses import dataclass, field
from typing import List, Optional, Tuple

from . import types as T
from .column import AggExpr, Alias, BinOp, Cast, ColRef, Column, ColumnData, Expr, Lit, SortOrder, Unary, When

_TOKEN = re.compile(r"""
    \s*(?:
      (?P<num>\d+\.\d*(?:[eE][-+]?\d+)?|\.\d+(?:[eE][-+]?\d+)?|\d+(?:[eE][-+]?\d+)?)
    | (?P<str>'(?:[^']|'')*')
    | (?P<dstr>"(?:[^"]|"")*")
    | (?P<ident>`[^`]+`|[A-Za-z_][A-Za-z_0-9]*(?:\.[A-Za-z_][A-Za-z_0-9]*)*)
    | (?P<op><=>|<=|>=|<>|!=|==|->|\|\||[-+*/%(),=<>.\[\]])
    )""", re.VERBOSE)

_KEYWORDS = {"SELECT", "FROM", "WHERE", "GROUP", "BY", "ORDER", "LIMIT", "AND", "OR", "NOT", "BETWEEN", "IN",
             "IS", "NULL", "AS", "ASC", "DESC", "DISTINCT", "HAVING", "CASE", "WHEN", "THEN", "ELSE", "END",
             "CAST", "TRUE", "FALSE", "LIKE", "TIMESTAMP", "DATE", "NULLS", "FIRST", "LAST", "INTERVAL"}


@dataclass
class Tok:
    kind: str
    val: str


def tokenize(s: str) -> List[Tok]:
    out, pos = [], 0
    s = s.strip().rstrip(";")
    while pos < len(s):
        m = _TOKEN.match(s, pos)
        if not m or m.end() == pos:
            if s[pos:].strip() == "":
                break
            raise SyntaxError(f"cannot tokenize SQL near {s[pos:pos + 20]!r}")
        pos = m.end()
        if m.group("num") is not None:
            out.append(Tok("num", m.group("num")))
        elif m.group("str") is not None:
            out.append(Tok("str", m.group("str")[1:-1].replace("''", "'")))
        elif m.group("dstr") is not None:
            out.append(Tok("str", m.group("dstr")[1:-1].replace('""', '"')))
        elif m.group("ident") is not None:
            v = m.group("ident")
            if v.startswith("`"):
                out.append(Tok("ident", v[1:-1]))
            elif v.upper() in _KEYWORDS:
                out.append(Tok("kw", v.upper()))
            else:
                out.append(Tok("ident", v))
        else:
            out.append(Tok("op", m.group("op")))
    return out


class Parser:
    def __init__(self, toks: List[Tok]):
        self.t = toks
        self.i = 0

    def peek(self, k=0) -> Optional[Tok]:
        j = self.i + k
        return self.t[j] if j < len(self.t) else None

    def at_kw(self, *kws) -> bool:
        p = self.peek()
        return p is not None and p.kind == "kw" and p.val in kws

    def at_op(self, *ops) -> bool:
        p = self.peek()
        return p is not None and p.kind == "op" and p.val in ops

    def take(self) -> Tok:
        tok = self.peek()
        if tok is None:
            raise SyntaxError("unexpected end of SQL")
        self.i += 1
        return tok

    def at_word(self, *words) -> bool:
        """A keyword or identifier spelled like one of ``words`` (window-clause words are not reserved)."""
        p = self.peek()
        return p is not None and p.kind in ("kw", "ident") and p.val.upper() in words

    def expect_word(self, word):
        if not self.at_word(word):
            tok = self.peek()
            raise SyntaxError(f"expected {word}, got {tok.val if tok else 'end of SQL'!r}")
        self.take()

    def expect_kw(self, kw):
        tok = self.take()
        if tok.kind != "kw" or tok.val != kw:
            raise SyntaxError(f"expected {kw}, got {tok.val!r}")

    def expect_op(self, op):
        tok = self.take()
        if tok.kind != "op" or tok.val != op:
            raise SyntaxError(f"expected {op!r}, got {tok.val!r}")

    # expressions -------------------------------------------------------------------------------
    def expr(self) -> Expr:
        return self.or_expr()

    def or_expr(self):
        e = self.and_expr()
        while self.at_kw("OR"):
            self.take()
            e = BinOp("or", e, self.and_expr())
        return e

    def and_expr(self):
        e = self.not_expr()
        while self.at_kw("AND"):
            self.take()
            e = BinOp("and", e, self.not_expr())
        return e

    def not_expr(self):
        if self.at_kw("NOT"):
            self.take()
            return Unary("not", self.not_expr())
        return self.predicate()

    def predicate(self):
        e = self.additive()
        while True:
            neg = False
            if self.at_kw("NOT") and self.peek(1) is not None and self.peek(1).val in ("BETWEEN", "IN", "LIKE"):
                self.take()
                neg = True
            if self.at_kw("BETWEEN"):
                self.take()
                lo = self.additive()
                self.expect_kw("AND")
                hi = self.additive()
                e2 = BinOp("and", BinOp(">=", e, lo), BinOp("<=", e, hi))
                e = Unary("not", e2) if neg else e2
            elif self.at_kw("IN"):
                self.take()
                self.expect_op("(")
                if self.at_kw("SELECT"):
                    q = _query(self)
                    self.expect_op(")")
                    e2 = InSubquery(e, q)
                    e = Unary("not", e2) if neg else e2
                    continue
                items = [self.expr()]
                while self.at_op(","):
                    self.take()
                    items.append(self.expr())
                self.expect_op(")")
                acc = None
                for it in items:
                    t = BinOp("==", e, it)
                    acc = t if acc is None else BinOp("or", acc, t)
                e = Unary("not", acc) if neg else acc
            elif self.at_kw("LIKE"):
                self.take()
                pat = self.take().val
                e2 = _like(e, pat)
                e = Unary("not", e2) if neg else e2
            elif self.at_kw("IS"):
                self.take()
                isnot = False
                if self.at_kw("NOT"):
                    self.take()
                    isnot = True
                self.expect_kw("NULL")
                e = Unary("isnotnull" if isnot else "isnull", e)
            elif self.at_op("<=>"):  # null-safe equality
                self.take()
                from .functions_tail import equal_null
                e = equal_null(Column(e), Column(self.additive()))._expr
            elif self.at_op("=", "==", "!=", "<>", "<", "<=", ">", ">=", "<=>"):
                op = self.take().val
                op = {"=": "==", "<>": "!="}.get(op, op)
                e = BinOp(op, e, self.additive())
            else:
                return e

    def additive(self):
        e = self.mult()
        while self.at_op("+", "-", "||"):
            op = self.take().val
            rhs = self.mult()
            if op == "||":
                from .functions import concat
                e = concat(Column(e), Column(rhs))._expr
            elif isinstance(rhs, IntervalLit):
                e = rhs.add_to(e, -1 if op == "-" else 1)
            else:
                e = BinOp(op, e, rhs)
        return e

    def interval(self) -> "IntervalLit":
        """INTERVAL n unit [n unit ...] / INTERVAL 'n' unit (units: year, month, week, day, hour, minute,
        second, millisecond, microsecond; plural forms accepted)."""
        months, micros = 0, 0
        while self.peek() is not None and self.peek().kind in ("num", "str") or self.at_op("-"):
            neg = False
            if self.at_op("-"):
                self.take()
                neg = True
            v = float(self.take().val)
            unit = self.take().val.upper().rstrip("S")
            v = -v if neg else v
            if unit in ("YEAR", "MONTH"):
                months += int(v) * (12 if unit == "YEAR" else 1)
            else:
                scale = {"WEEK": 7 * 86400e6, "DAY": 86400e6, "HOUR": 3600e6, "MINUTE": 60e6, "SECOND": 1e6,
                         "MILLISECOND": 1e3, "MICROSECOND": 1.0}.get(unit)
                if scale is None:
                    raise SyntaxError(f"unsupported interval unit {unit}")
                micros += int(round(v * scale))
        return IntervalLit(months, micros)

    def mult(self):
        e = self.unary()
        while self.at_op("*", "/", "%"):
            op = self.take().val
            e = BinOp(op, e, self.unary())
        return e

    def unary(self):
        if self.at_op("-"):
            self.take()
            return Unary("neg", self.unary())
        if self.at_op("+"):
            self.take()
            return self.unary()
        return self._postfix(self.primary())

    def _postfix(self, e: Expr) -> Expr:
        """``e[i]`` (0-based array index / map key) and ``e.field`` (struct field)."""
        while True:
            if self.at_op("["):
                self.take()
                idx = self.expr()
                self.expect_op("]")
                e = Subscript(e, idx)
            elif self.at_op(".") and self.peek(1) is not None and self.peek(1).kind == "ident":
                self.take()
                e = GetField(e, self.take().val)
            else:
                return e

    def _try_lambda(self) -> Optional[Expr]:
        """``x -> body`` or ``(x, y) -> body`` as a higher-order function argument."""
        t0, t1 = self.peek(), self.peek(1)
        if t0 is not None and t0.kind == "ident" and t1 is not None and t1.kind == "op" and t1.val == "->":
            self.take(), self.take()
            return SqlLambda([t0.val], self.expr())
        if t0 is not None and t0.kind == "op" and t0.val == "(":
            k, names = 1, []
            while True:
                t = self.peek(k)
                if t is None or t.kind != "ident":
                    return None
                names.append(t.val)
                t = self.peek(k + 1)
                if t is not None and t.kind == "op" and t.val == ",":
                    k += 2
                    continue
                if t is not None and t.kind == "op" and t.val == ")":
                    arrow = self.peek(k + 2)
                    if arrow is not None and arrow.kind == "op" and arrow.val == "->":
                        for _ in range(k + 3):
                            self.take()
                        return SqlLambda(names, self.expr())
                return None
        return None

    def primary(self) -> Expr:
        tok = self.take()
        if tok.kind == "num":
            v = tok.val
            return Lit(float(v) if any(c in v for c in ".eE") else int(v))
        if tok.kind == "str":
            return Lit(tok.val)
        if tok.kind == "op" and tok.val == "(":
            e = self.expr()
            self.expect_op(")")
            return e
        if tok.kind == "op" and tok.val == "*":
            return ColRef("*")
        if tok.kind == "kw":
            if tok.val == "NULL":
                return Lit(None)
            if tok.val in ("TRUE", "FALSE"):
                return Lit(tok.val == "TRUE")
            if tok.val in ("TIMESTAMP", "DATE") and self.peek() is not None and self.peek().kind == "str":
                return Cast(Lit(self.take().val), T.TimestampType() if tok.val == "TIMESTAMP" else T.DateType())
            if tok.val == "CASE":
                return self.case()
            if tok.val == "INTERVAL":
                return self.interval()
            if tok.val == "CAST":
                self.expect_op("(")
                e = self.expr()
                self.expect_kw("AS")
                typ = self.take().val
                if self.at_op("("):  # decimal(10,2) etc.
                    while not self.at_op(")"):
                        self.take()
                    self.take()
                    typ = "double"
                self.expect_op(")")
                return Cast(e, T.parse_type(typ))
            raise SyntaxError(f"unexpected keyword {tok.val}")
        if tok.kind == "ident":
            if self.at_op("("):
                return self.call(tok.val)
            if "." in tok.val:
                q, c = tok.val.rsplit(".", 1)
                return QualRef(q, c)
            return ColRef(tok.val)
        raise SyntaxError(f"unexpected token {tok.val!r}")

    def case(self) -> Expr:
        base = None
        if not self.at_kw("WHEN"):
            base = self.expr()
        branches = []
        other = None
        while self.at_kw("WHEN"):
            self.take()
            c = self.expr()
            if base is not None:
                c = BinOp("==", base, c)
            self.expect_kw("THEN")
            branches.append((c, self.expr()))
        if self.at_kw("ELSE"):
            self.take()
            other = self.expr()
        self.expect_kw("END")
        return When(branches, other)

    def call(self, name: str) -> Expr:
        from . import functions as F
        self.expect_op("(")
        lname = name.lower()
        special = self._special_call(lname)
        if special is not None:
            return special
        distinct = False
        if self.at_kw("DISTINCT"):
            self.take()
            distinct = True
        args: List[Expr] = []
        if self.at_op("*"):
            self.take()
            args = []
        elif not self.at_op(")"):
            args.append(self._try_lambda() or self.expr())
            while self.at_op(","):
                self.take()
                args.append(self._try_lambda() or self.expr())
        self.expect_op(")")
        e = self._call_expr(name, lname, args, distinct)
        if self.at_word("OVER"):
            self.take()
            from .window import WindowExpr
            e = WindowExpr(e, self.window_spec())
        return e

    def _special_call(self, lname: str) -> Optional[Expr]:
        """SQL-standard argument syntax: EXTRACT(f FROM e), POSITION(a IN b), TRIM([BOTH|LEADING|TRAILING]
        [chars] FROM s), SUBSTRING(s FROM p [FOR n]). Returns None (nothing consumed) otherwise."""
        from . import functions as F
        if lname in ("extract", "date_part") and self.peek(1) is not None and self.peek(1).kind == "kw" \
                and self.peek(1).val == "FROM":
            field_ = self.take().val
            self.expect_kw("FROM")
            src = self.expr()
            self.expect_op(")")
            return F.date_part(field_, Column(src))._expr
        if lname == "position":
            sub = self.additive()
            if not self.at_kw("IN"):
                args = [sub]
                while self.at_op(","):
                    self.take()
                    args.append(self.expr())
                self.expect_op(")")
                start = int(args[2].value) if len(args) > 2 else 1
                return F.locate(args[0].value, Column(args[1]), start)._expr
            self.take()
            src = self.expr()
            self.expect_op(")")
            return F.locate(sub.value if isinstance(sub, Lit) else str(sub), Column(src))._expr
        if lname == "trim" and (self.at_word("BOTH", "LEADING", "TRAILING") or self._trim_from_ahead()):
            mode = self.take().val.upper() if self.at_word("BOTH", "LEADING", "TRAILING") else "BOTH"
            chars = None
            if not self.at_kw("FROM"):
                chars = self.additive()
            self.expect_kw("FROM")
            src = self.expr()
            self.expect_op(")")
            cs = " " if chars is None else (chars.value if isinstance(chars, Lit) else str(chars))
            fn = {"BOTH": str.strip, "LEADING": str.lstrip, "TRAILING": str.rstrip}[mode]
            return F._host_map(f"trim_{mode.lower()}", [Column(src)], lambda v: fn(str(v), cs), T.StringType(),
                               params=[cs])._expr
        if lname in ("substring", "substr"):
            save = self.i
            first = self.expr()
            if self.at_kw("FROM"):
                self.take()
                pos = self.expr()
                ln = None
                if self.at_word("FOR"):
                    self.take()
                    ln = self.expr()
                self.expect_op(")")
                return F.substring(Column(first), int(pos.value), int(ln.value) if ln is not None else 2 ** 31 - 1)._expr
            self.i = save
        return None

    def _trim_from_ahead(self) -> bool:
        """TRIM('x' FROM s) / TRIM(FROM s): a FROM keyword inside the parentheses."""
        depth, k = 0, 0
        while True:
            t = self.peek(k)
            if t is None:
                return False
            if t.kind == "op" and t.val == "(":
                depth += 1
            elif t.kind == "op" and t.val == ")":
                if depth == 0:
                    return False
                depth -= 1
            elif t.kind == "kw" and t.val == "FROM" and depth == 0:
                return True
            k += 1

    def window_spec(self):
        """OVER ( [PARTITION BY e, ...] [ORDER BY e [ASC|DESC] [NULLS FIRST|LAST], ...]
                  [ROWS|RANGE BETWEEN bound AND bound] )"""
        from .window import Window, WindowSpec
        self.expect_op("(")
        part, orders, frame = [], [], None
        if self.at_word("PARTITION"):
            self.take()
            self.expect_kw("BY")
            part.append(self.expr())
            while self.at_op(","):
                self.take()
                part.append(self.expr())
        if self.at_kw("ORDER"):
            self.take()
            self.expect_kw("BY")
            while True:
                e = self.expr()
                asc = True
                if self.at_kw("ASC", "DESC"):
                    asc = self.take().val == "ASC"
                nulls_first = None
                if self.at_kw("NULLS"):
                    self.take()
                    nulls_first = self.take().val == "FIRST"
                orders.append(SortOrder(e, asc, nulls_first))
                if not self.at_op(","):
                    break
                self.take()
        if self.at_word("ROWS", "RANGE"):
            kind = self.take().val.lower()
            self.expect_kw("BETWEEN")
            lo = self._frame_bound()
            self.expect_kw("AND")
            hi = self._frame_bound()
            frame = (kind, lo, hi)
        self.expect_op(")")
        spec = WindowSpec(part, orders)
        if frame is not None:
            spec = spec.rowsBetween(frame[1], frame[2]) if frame[0] == "rows" else spec.rangeBetween(frame[1],
                                                                                                     frame[2])
        return spec

    def _frame_bound(self) -> int:
        from .window import Window
        if self.at_word("UNBOUNDED"):
            self.take()
            if self.at_word("PRECEDING"):
                self.take()
                return Window.unboundedPreceding
            self.expect_word("FOLLOWING")
            return Window.unboundedFollowing
        if self.at_word("CURRENT"):
            self.take()
            self.expect_word("ROW")
            return Window.currentRow
        tok = self.take()
        if tok.kind != "num":
            raise SyntaxError(f"expected a frame bound, got {tok.val!r}")
        v = float(tok.val)
        v = int(v) if v.is_integer() else v
        if self.at_word("PRECEDING"):
            self.take()
            return -v
        self.expect_word("FOLLOWING")
        return v

    def _call_expr(self, name: str, lname: str, args: List[Expr], distinct: bool) -> Expr:
        from . import functions as F
        if lname == "count":
            return AggExpr("count", args[0] if args else None, distinct)
        aggs = {"sum": "sum", "avg": "avg", "mean": "avg", "min": "min", "max": "max", "stddev": "stddev",
                "stddev_samp": "stddev", "stddev_pop": "stddev_pop", "variance": "variance",
                "var_samp": "variance", "var_pop": "var_pop", "first": "first", "last": "last",
                "collect_list": "collect_list", "collect_set": "collect_set"}
        if lname in aggs:
            return AggExpr(aggs[lname], args[0], distinct)
        if lname in ("lag", "lead"):
            off = int(args[1].value) if len(args) > 1 else 1
            default = args[2].value if len(args) > 2 else None
            return getattr(F, lname)(Column(args[0]), off, default)._expr
        if lname == "ntile":
            return F.ntile(int(args[0].value))._expr
        fn = F.REGISTERED_UDFS.get(lname) or getattr(F, lname, None)
        if fn is None:
            raise SyntaxError(f"unknown function {name}")
        lit_pos = _LIT_ARGS.get(lname, ())
        cols = [a.callable() if isinstance(a, SqlLambda) else
                a.value if (i in lit_pos and isinstance(a, Lit)) else Column(a) for i, a in enumerate(args)]
        if lname == "round" and len(args) == 2:
            return F.round(cols[0], int(args[1].value))._expr
        if lname in ("current_timestamp", "current_date", "now"):
            return fn()._expr
        return fn(*cols)._expr


# argument positions that the Python builders take as plain values (SQL passes literals there)
_LIT_ARGS = {
    "percentile": (1,), "percentile_approx": (1, 2), "sha2": (1,), "repeat": (1,), "instr": (1,), "locate": (0, 2),
    "translate": (1, 2), "add_months": (1,), "date_trunc": (0,), "trunc": (1,), "bround": (1,), "element_at": (1,),
    "array_contains": (1,), "array_join": (1, 2), "sort_array": (1,), "date_add": (1,), "date_sub": (1,),
    "substring": (1, 2), "substr": (1, 2), "lpad": (1, 2), "rpad": (1, 2), "regexp_replace": (1, 2),
    "regexp_extract": (1, 2), "split": (1,), "date_format": (1,), "concat_ws": (0,), "from_unixtime": (1,),
    "to_date": (1,), "to_timestamp": (1,), "unix_timestamp": (1,), "months_between": (2,),
    "approx_count_distinct": (1,),
}


def _like(e: Expr, pattern: str) -> Expr:
    from .column import ColumnData, Func
    import numpy as np
    import torch
    rx = re.compile("^" + "".join(".*" if ch == "%" else "." if ch == "_" else re.escape(ch) for ch in pattern)
                    + "$", re.S)

    def impl(frame, args):
        from .column import _to_host
        h = _to_host(args[0])
        vm = h.valid_mask() & np.array([v is not None for v in h.values], dtype=bool)
        out = np.array([bool(rx.match(str(v))) if ok else False for v, ok in zip(h.values, vm)], dtype=bool)
        return ColumnData(torch.as_tensor(out, device=frame._device), torch.as_tensor(vm, device=frame._device),
                          T.BooleanType())
    return Func(f"like({pattern})", [e], impl)


class QualRef(ColRef):
    """``alias.column``: resolves to the join output column ``alias.column`` when the join had to
    qualify it (the name exists on both sides), else to ``column``."""

    def __init__(self, qual: str, col: str):
        super().__init__(col)
        self.qual = qual

    def eval(self, frame):
        full = f"{self.qual}.{self.col}"
        if full in frame._cols or self.col in frame._cols:
            return frame._column_data(full if full in frame._cols else self.col)
        head = self.qual.split(".")[0]
        if head in frame._cols:  # struct column: s.a / s.a.b
            e: Expr = ColRef(head)
            for part in self.qual.split(".")[1:] + [self.col]:
                e = GetField(e, part)
            return e.eval(frame)
        return frame._column_data(self.col)

    def __str__(self):
        return f"{self.qual}.{self.col}"


class IntervalLit(Expr):
    """An INTERVAL literal: months + microseconds, added to dates / timestamps by ``+`` / ``-``."""

    def __init__(self, months: int, micros: int):
        self.months, self.micros = months, micros

    def refs(self):
        return []

    def __str__(self):
        return f"INTERVAL {self.months} MONTHS {self.micros} MICROSECONDS"

    def eval(self, frame):
        raise ValueError("an INTERVAL is only valid added to or subtracted from a date / timestamp")

    def add_to(self, e: Expr, sign: int) -> Expr:
        months, micros = sign * self.months, sign * self.micros
        from .column import Func

        def impl(frame, args):
            import torch
            a = args[0]
            if months:
                from .functions_more import _add_months
                from .column import micros_to_datetime, ts_to_micros
                from .dataframe import column_to_python
                from .builder import column_from_values
                import datetime as _dt
                vals = []
                for v in column_to_python(a):
                    if v is None:
                        vals.append(None)
                        continue
                    t = v if isinstance(v, _dt.datetime) else _dt.datetime.combine(v, _dt.time())
                    d = _add_months(t.date(), months)
                    vals.append(_dt.datetime.combine(d, t.time()) + _dt.timedelta(microseconds=micros))
                out = column_from_values(vals, T.TimestampType(), frame._device)
                if isinstance(a.dtype, T.DateType) and micros % 86_400_000_000 == 0:
                    out = ColumnData(torch.div(out.values, 86_400_000_000, rounding_mode="floor").to(torch.int32),
                                     out.valid, T.DateType())
                return out
            if isinstance(a.dtype, T.DateType):
                if micros % 86_400_000_000 == 0:
                    return ColumnData(a.values + micros // 86_400_000_000, a.valid, T.DateType())
                return ColumnData(a.values.to(torch.int64) * 86_400_000_000 + micros, a.valid, T.TimestampType())
            if isinstance(a.dtype, T.TimestampType):
                return ColumnData(a.values + micros, a.valid, T.TimestampType())
            raise TypeError(f"cannot add an INTERVAL to {a.dtype.simpleString()}")
        return Func(f"({e} {'+' if sign > 0 else '-'} INTERVAL)", [e], impl)


class GetField(Expr):
    """``struct_expr.field``."""

    def __init__(self, child: Expr, field: str):
        self.child, self.field = child, field

    def refs(self):
        return self.child.refs()

    def name(self):
        return self.field

    def __str__(self):
        return f"{self.child}.{self.field}"

    def eval(self, frame):
        from .builder import column_from_values
        from .dataframe import column_to_python
        cd = self.child.eval(frame)
        st = cd.dtype
        if not isinstance(st, T.StructType):
            raise TypeError(f"cannot extract field {self.field!r} from {st.simpleString()}")
        ft = next((f.dataType for f in st.fields if f.name == self.field), None)
        if ft is None:
            raise ValueError(f"no field {self.field!r} in {st.simpleString()}")
        vals = [None if v is None else (v[self.field] if isinstance(v, dict) else getattr(v, self.field))
                for v in column_to_python(cd)]
        return column_from_values(vals, ft, frame._device)


class Subscript(Expr):
    """``array[i]`` (0-based, null when out of range) / ``map[key]``."""

    def __init__(self, child: Expr, index: Expr):
        self.child, self.index = child, index

    def refs(self):
        return self.child.refs() + self.index.refs()

    def __str__(self):
        return f"{self.child}[{self.index}]"

    def eval(self, frame):
        from .builder import column_from_values
        from .dataframe import column_to_python
        cd = self.child.eval(frame)
        keys = column_to_python(self.index.eval(frame))
        vals = column_to_python(cd)
        out = []
        for v, k in zip(vals, keys):
            if v is None or k is None:
                out.append(None)
            elif isinstance(v, dict):
                out.append(v.get(k))
            else:
                i = int(k)
                out.append(v[i] if 0 <= i < len(v) else None)
        dt = cd.dtype.valueType if isinstance(cd.dtype, T.MapType) else (
            cd.dtype.elementType if isinstance(cd.dtype, T.ArrayType) else T.StringType())
        return column_from_values(out, dt, frame._device)


class SqlLambda(Expr):
    """``(x, y) -> body`` argument of a SQL higher-order function; becomes a Python callable over
    Columns whose parameters replace the body's references to x, y."""

    def __init__(self, params: List[str], body: Expr):
        self.params, self.body = params, body

    def refs(self):
        return []

    def __str__(self):
        return f"lambdafunction({self.body}, {', '.join(self.params)})"

    def eval(self, frame):
        raise ValueError("a lambda is only valid as a higher-order function argument")

    def callable(self):
        params, body = self.params, self.body

        def bind(*cols):
            mapping = {p: c._expr for p, c in zip(params, cols)}
            return Column(_transform(body, lambda e: mapping.get(e.col) if isinstance(e, ColRef) and not isinstance(
                e, QualRef) and e.col in mapping else None))
        if len(params) == 1:
            return lambda a: bind(a)
        if len(params) == 2:
            return lambda a, b: bind(a, b)
        if len(params) == 3:
            return lambda a, b, c: bind(a, b, c)
        raise SyntaxError("lambdas take 1 to 3 parameters")


class InSubquery(Expr):
    """``e IN (SELECT ...)``: the subquery runs once per evaluation; its single column's distinct
    values become the IN list."""

    def __init__(self, child: Expr, query):
        self.child, self.query = child, query

    def refs(self):
        return self.child.refs()

    def __str__(self):
        return f"({self.child} IN (subquery))"

    def eval(self, frame):
        from .dataframe import column_to_python
        sub = _run_query(frame._session, self.query)
        if len(sub.columns) != 1:
            raise ValueError("IN subquery must return exactly one column")
        vals = []
        seen = set()
        for part in frame._comm.allgather_object(column_to_python(sub._column_data(sub.columns[0]))):
            for v in part:
                if v not in seen:
                    seen.add(v)
                    vals.append(v)
        acc = Lit(False)
        for v in vals:
            acc = BinOp("or", acc, BinOp("==", self.child, Lit(v)))
        return acc.eval(frame)


@dataclass
class Source:
    name: Optional[str] = None
    sub: Optional[object] = None  # a query
    alias: Optional[str] = None
    sample: Optional[tuple] = None  # TABLESAMPLE: ("percent", p) | ("rows", n)


@dataclass
class JoinClause:
    how: str
    right: Source
    on: Optional[Expr] = None
    using: Optional[List[str]] = None


@dataclass
class Select:
    items: List[Tuple[Expr, Optional[str]]]
    table: Optional[str]
    where: Optional[Expr] = None
    group_by: List[Expr] = field(default_factory=list)
    having: Optional[Expr] = None
    order_by: List[SortOrder] = field(default_factory=list)
    limit: Optional[int] = None
    distinct: bool = False
    subquery: Optional["Select"] = None
    source: Optional[Source] = None
    joins: List[JoinClause] = field(default_factory=list)
    grouping_sets: Optional[List[List[Expr]]] = None  # ROLLUP / CUBE / GROUPING SETS


@dataclass
class SetOp:
    op: str          # union | union all | intersect | except
    left: object
    right: object
    order_by: List[SortOrder] = field(default_factory=list)
    limit: Optional[int] = None


def parse_select(sql: str):
    p = Parser(tokenize(sql))
    q = _query(p)
    if p.peek() is not None:
        raise SyntaxError(f"unexpected trailing SQL: {p.peek().val!r}")
    return q


def _query(p: Parser):
    """select (UNION [ALL] | INTERSECT | EXCEPT | MINUS) select ... ; a trailing ORDER BY / LIMIT of
    the last select applies to the whole set operation."""
    left = _select(p)
    while p.at_word("UNION", "INTERSECT", "EXCEPT", "MINUS"):
        op = p.take().val.upper()
        if op == "UNION" and p.at_word("ALL"):
            p.take()
            op = "UNION ALL"
        elif p.at_kw("DISTINCT"):
            p.take()
        right = _select(p)
        left = SetOp(op.lower().replace("minus", "except"), left, right)
        if isinstance(right, Select) and (right.order_by or right.limit is not None):
            left.order_by, left.limit = right.order_by, right.limit
            right.order_by, right.limit = [], None
    return left


def _source(p: Parser) -> Source:
    if p.at_op("("):
        p.take()
        sub = _query(p)
        p.expect_op(")")
        src = Source(sub=sub)
    else:
        src = Source(name=p.take().val)
    if p.at_word("TABLESAMPLE"):
        p.take()
        p.expect_op("(")
        v = float(p.take().val)
        unit = p.take().val.upper()
        if unit not in ("PERCENT", "ROWS"):
            raise SyntaxError("TABLESAMPLE supports (n PERCENT) and (n ROWS)")
        p.expect_op(")")
        src.sample = ("percent", v) if unit == "PERCENT" else ("rows", int(v))
    if p.at_kw("AS"):
        p.take()
        src.alias = p.take().val
    elif p.peek() is not None and p.peek().kind == "ident" and not p.at_word(
            "JOIN", "INNER", "LEFT", "RIGHT", "FULL", "CROSS", "SEMI", "ANTI", "ON", "USING", "UNION", "INTERSECT",
            "EXCEPT", "MINUS", "OUTER", "NATURAL"):
        src.alias = p.take().val
    return src


_JOIN_WORDS = ("JOIN", "INNER", "LEFT", "RIGHT", "FULL", "CROSS", "SEMI", "ANTI")


def _join(p: Parser) -> Optional[JoinClause]:
    if not p.at_word(*_JOIN_WORDS) and not p.at_op(","):
        return None
    if p.at_op(","):  # FROM a, b  ==  CROSS JOIN
        p.take()
        return JoinClause("cross", _source(p))
    words = []
    while not p.at_word("JOIN"):
        words.append(p.take().val.upper())
    p.take()
    words = [w for w in words if w != "OUTER"]
    how = {(): "inner", ("INNER",): "inner", ("LEFT",): "left", ("RIGHT",): "right", ("FULL",): "full",
           ("CROSS",): "cross", ("LEFT", "SEMI"): "leftsemi", ("SEMI",): "leftsemi", ("LEFT", "ANTI"): "leftanti",
           ("ANTI",): "leftanti"}.get(tuple(words))
    if how is None:
        raise SyntaxError(f"unsupported join type {' '.join(words)}")
    right = _source(p)
    jc = JoinClause(how, right)
    if p.at_word("ON"):
        p.take()
        jc.on = p.expr()
    elif p.at_word("USING"):
        p.take()
        p.expect_op("(")
        cols = [p.take().val]
        while p.at_op(","):
            p.take()
            cols.append(p.take().val)
        p.expect_op(")")
        jc.using = cols
    elif how != "cross":
        raise SyntaxError("JOIN needs ON or USING")
    return jc


def _select(p: Parser) -> Select:
    if p.at_op("("):
        p.take()
        q = _query(p)
        p.expect_op(")")
        return q
    p.expect_kw("SELECT")
    distinct = False
    if p.at_kw("DISTINCT"):
        p.take()
        distinct = True
    items = [_select_item(p)]
    while p.at_op(","):
        p.take()
        items.append(_select_item(p))
    sel = Select(items, None, distinct=distinct)
    if p.at_kw("FROM"):
        p.take()
        sel.source = _source(p)
        sel.table = sel.source.name
        while True:
            jc = _join(p)
            if jc is None:
                break
            sel.joins.append(jc)
    if p.at_kw("WHERE"):
        p.take()
        sel.where = p.expr()
    if p.at_kw("GROUP"):
        p.take()
        p.expect_kw("BY")
        _group_by(p, sel)
    if p.at_kw("HAVING"):
        p.take()
        sel.having = p.expr()
    if p.at_kw("ORDER"):
        p.take()
        p.expect_kw("BY")
        while True:
            e = p.expr()
            asc = True
            if p.at_kw("ASC", "DESC"):
                asc = p.take().val == "ASC"
            nulls_first = None
            if p.at_kw("NULLS"):
                p.take()
                nulls_first = p.take().val == "FIRST"
            sel.order_by.append(SortOrder(e, asc, nulls_first))
            if not p.at_op(","):
                break
            p.take()
    if p.at_kw("LIMIT"):
        p.take()
        sel.limit = int(p.take().val)
    return sel


def _paren_list(p: Parser) -> List[Expr]:
    p.expect_op("(")
    out: List[Expr] = []
    if not p.at_op(")"):
        out.append(p.expr())
        while p.at_op(","):
            p.take()
            out.append(p.expr())
    p.expect_op(")")
    return out


def _rollup_sets(keys: List[Expr]) -> List[List[Expr]]:
    return [keys[:i] for i in range(len(keys), -1, -1)]


def _cube_sets(keys: List[Expr]) -> List[List[Expr]]:
    n = len(keys)
    return [[k for j, k in enumerate(keys) if not (mask >> (n - 1 - j)) & 1] for mask in range(2 ** n)]


def _group_by(p: Parser, sel: Select) -> None:
    """GROUP BY e, ... | ROLLUP(e, ...) | CUBE(e, ...) | GROUPING SETS ((e, ...), e, ()) | e, ... WITH ROLLUP|CUBE."""
    nxt = p.peek(1)
    if p.at_word("ROLLUP", "CUBE") and nxt is not None and nxt.kind == "op" and nxt.val == "(":
        kind = p.take().val.upper()
        keys = _paren_list(p)
        sel.group_by = keys
        sel.grouping_sets = _rollup_sets(keys) if kind == "ROLLUP" else _cube_sets(keys)
        return
    if p.at_word("GROUPING") and nxt is not None and nxt.kind == "ident" and nxt.val.upper() == "SETS":
        p.take(), p.take()
        p.expect_op("(")
        sets: List[List[Expr]] = []
        while True:
            sets.append(_paren_list(p) if p.at_op("(") else [p.expr()])
            if not p.at_op(","):
                break
            p.take()
        p.expect_op(")")
        keys: List[Expr] = []
        for st in sets:
            for k in st:
                if str(k) not in {str(x) for x in keys}:
                    keys.append(k)
        sel.group_by, sel.grouping_sets = keys, sets
        return
    sel.group_by.append(p.expr())
    while p.at_op(","):
        p.take()
        sel.group_by.append(p.expr())
    if p.at_word("WITH") and p.peek(1) is not None and p.peek(1).val.upper() in ("ROLLUP", "CUBE"):
        p.take()
        kind = p.take().val.upper()
        sel.grouping_sets = _rollup_sets(sel.group_by) if kind == "ROLLUP" else _cube_sets(sel.group_by)


class _QualStar(Expr):
    def __init__(self, qual: str):
        self.qual = qual

    def refs(self):
        return []

    def __str__(self):
        return f"{self.qual}.*"


def _select_item(p: Parser):
    tok, nxt = p.peek(), p.peek(1)
    if tok is not None and tok.kind == "ident" and nxt is not None and nxt.kind == "op" and nxt.val == "." \
            and p.peek(2) is not None and p.peek(2).val == "*":
        p.take(), p.take(), p.take()
        return _QualStar(tok.val), None
    e = p.expr()
    alias = None
    if p.at_kw("AS"):
        p.take()
        alias = p.take().val
    elif p.peek() is not None and p.peek().kind == "ident" and not p.at_word("FROM"):
        alias = p.take().val
    return e, alias


def parse_expression(sql: str) -> Expr:
    p = Parser(tokenize(sql))
    e = p.expr()
    if p.peek() is not None:
        raise SyntaxError(f"unexpected trailing tokens in expression: {p.peek().val!r}")
    return e


def parse_select_item(sql: str) -> Expr:
    p = Parser(tokenize(sql))
    e, alias = _select_item(p)
    return Alias(e, alias) if alias else e


# ---------------------------------------------------------------------------------------- statements

def execute(session, sql: str):
    """Run one SQL statement against the session catalog; returns a DataFrame.

    Queries: SELECT with joins (INNER / LEFT / RIGHT / FULL [OUTER], CROSS, LEFT SEMI / ANTI, ON or
    USING), set operations (UNION [ALL], INTERSECT, EXCEPT), WITH common table expressions, IN
    subqueries, GROUP BY with expressions. Statements: CREATE [OR REPLACE] [TEMP] VIEW .. AS,
    CREATE TABLE .. AS, INSERT INTO / OVERWRITE, DROP TABLE / VIEW, SHOW TABLES, DESCRIBE."""
    p = Parser(tokenize(sql))
    if p.at_word("WITH"):
        p.take()
        ctes = []
        while True:
            name = p.take().val
            p.expect_kw("AS")
            p.expect_op("(")
            ctes.append((name, _query(p)))
            p.expect_op(")")
            if not p.at_op(","):
                break
            p.take()
        q = _query(p)
        _expect_end(p)
        cat = session.catalog
        saved = {n: cat._views.get(n) for n, _ in ctes}
        try:
            for n, cq in ctes:
                cat._register_view(n, _run_query(session, cq), True)
            return _run_query(session, q)
        finally:
            for n, v in saved.items():
                if v is None:
                    cat._views.pop(n, None)
                else:
                    cat._views[n] = v
    if p.at_word("CREATE"):
        return _create(session, p)
    if p.at_word("INSERT"):
        p.take()
        mode = "append"
        if p.at_word("OVERWRITE"):
            p.take()
            mode = "overwrite"
        else:
            p.expect_word("INTO")
        if p.at_word("TABLE"):
            p.take()
        name = p.take().val
        df = _run_query(session, _query(p))
        _expect_end(p)
        target = session.table(name)
        df = df.toDF(*target.columns) if len(df.columns) == len(target.columns) else df
        session.catalog._save_table(name, df, mode)
        return session.createDataFrame([], T.StructType([]))
    if p.at_word("DROP"):
        p.take()
        kind = p.take().val.upper()
        if p.at_word("IF"):
            p.take()
            p.expect_word("EXISTS")
        name = p.take().val
        _expect_end(p)
        if kind == "VIEW":
            session.catalog.dropTempView(name)
        else:
            session.catalog.dropTable(name)
        return session.createDataFrame([], T.StructType([]))
    if p.at_word("SHOW"):
        p.take()
        p.take()  # TABLES | VIEWS
        _expect_end(p)
        rows = [(t.database or "", t.name, t.isTemporary) for t in session.catalog.listTables()]
        return session.createDataFrame(rows, "namespace STRING, tableName STRING, isTemporary BOOLEAN")
    if p.at_word("DESCRIBE", "DESC"):
        p.take()
        if p.at_word("TABLE"):
            p.take()
        name = p.take().val
        _expect_end(p)
        df = session.table(name)
        rows = [(f.name, f.dataType.simpleString(), None) for f in df.schema.fields]
        return session.createDataFrame(rows, "col_name STRING, data_type STRING, comment STRING")
    q = _query(p)
    _expect_end(p)
    return _run_query(session, q)


def _expect_end(p: Parser) -> None:
    if p.peek() is not None:
        raise SyntaxError(f"unexpected trailing SQL: {p.peek().val!r}")


def _create(session, p: Parser):
    p.take()  # CREATE
    replace = False
    if p.at_kw("OR"):
        p.take()
        p.expect_word("REPLACE")
        replace = True
    if p.at_word("GLOBAL"):
        p.take()
    if p.at_word("TEMP", "TEMPORARY"):
        p.take()
    kind = p.take().val.upper()
    if_not_exists = False
    if p.at_word("IF"):
        p.take()
        p.expect_kw("NOT")
        p.expect_word("EXISTS")
        if_not_exists = True
    name = p.take().val
    if p.at_word("USING"):
        p.take()
        p.take()
    p.expect_kw("AS")
    q = _query(p)
    _expect_end(p)
    df = _run_query(session, q)
    if kind == "VIEW":
        session.catalog._register_view(name, df, replace)
    elif kind == "TABLE":
        if session.catalog.tableExists(name):
            if if_not_exists:
                return session.createDataFrame([], T.StructType([]))
            raise ValueError(f"table {name} already exists")
        session.catalog._save_table(name, df, "overwrite")
    else:
        raise SyntaxError(f"CREATE {kind} is not supported")
    return session.createDataFrame([], T.StructType([]))


def _run_query(session, q):
    if isinstance(q, SetOp):
        left, right = _run_query(session, q.left), _run_query(session, q.right)
        if q.op == "union all":
            df = left.union(right)
        elif q.op == "union":
            df = left.union(right).distinct()
        elif q.op == "intersect":
            df = left.intersect(right)
        else:
            df = left.subtract(right)
        if q.order_by:
            df = df.orderBy(*q.order_by)
        if q.limit is not None:
            df = df.limit(q.limit)
        return df
    return _run(session, q)


def _source_frame(session, src: Source):
    df = _run_query(session, src.sub) if src.sub is not None else session.table(src.name)
    if src.sample is not None:
        kind, v = src.sample
        df = df.sample(fraction=min(max(v / 100.0, 0.0), 1.0), seed=0) if kind == "percent" else df.limit(v)
    return df, (src.alias or src.name)


def _split_on(cond: Expr, lcols, rcols):
    """ON condition -> ([(left col, right col)] equi keys, residual conjuncts)."""
    conj = []

    def flat(e):
        if isinstance(e, BinOp) and e.op == "and":
            flat(e.left)
            flat(e.right)
        else:
            conj.append(e)
    flat(cond)
    keys, rest = [], []
    for c in conj:
        if isinstance(c, BinOp) and c.op == "==" and isinstance(c.left, ColRef) and isinstance(c.right, ColRef):
            a, b = c.left, c.right
            side = lambda r, cols: (getattr(r, "qual", None), r.col, r.col in cols)  # noqa: E731
            la, lb = side(a, lcols), side(b, rcols)
            if la[2] and lb[2]:
                keys.append((a, b))
                continue
            la, lb = side(b, lcols), side(a, rcols)
            if la[2] and lb[2]:
                keys.append((b, a))
                continue
        rest.append(c)
    return keys, rest


def _join_frames(left, lq, right, rq, how: str, lkeys: List[str], rkeys: List[str], using: bool):
    """Equi-join keeping both sides' columns; names present on both sides become
    ``alias.column`` (USING keys appear once). Device path: relational_fast (joint key codes,
    per-code match ranges; right side broadcast as ``DataFrame.join``), row loop otherwise."""
    from . import relational_fast as RF
    lnames = left.columns
    rnames = right.columns
    r_out = [n for n in rnames if not (using and n in rkeys)]
    both = set(lnames) & set(r_out)
    lq, rq = lq or "l", rq or "r"
    out_l = [f"{lq}.{n}" if n in both else n for n in lnames]
    out_r = [f"{rq}.{n}" if n in both else n for n in r_out]
    semi = how in ("leftsemi", "leftanti")
    fields = [T.StructField(n, left.schema[o].dataType, True) for n, o in zip(out_l, lnames)]
    if not semi:
        fields += [T.StructField(n, right.schema[o].dataType, True) for n, o in zip(out_r, r_out)]
    schema = T.StructType(fields)
    df = None
    if RF.ENABLED:
        rcols, n_right = RF._gather_frame(right)
        r = RF.join_indices(left, rcols, n_right, list(lkeys), list(rkeys), how)
        if r is not None:
            li, ri = r
            fill = list(zip(lkeys, rkeys)) if using else []
            df = RF.build_join(left, rcols, li, ri, list(zip(out_l, lnames)),
                               [] if semi else list(zip(out_r, r_out)), fill, schema)
    if df is None:
        df = _join_rows(left, right, how, lkeys, rkeys, using, lnames, r_out, schema, semi)
    src = dict(getattr(left, "_sql_sources", {}) or {lq: out_l})
    if not semi:
        src[rq] = out_r
    df._sql_sources = src
    return df


def _join_rows(left, right, how, lkeys, rkeys, using, lnames, r_out, schema, semi):
    """Row-loop join for keys without device codes (vectors, arrays, ...)."""
    from .builder import frame_from_pycolumns
    from .group import _hashable
    rnames, rrows, _ = right._gather_host()
    lcols = left._local_rows_host()
    ridx = [rnames.index(k) for k in rkeys]
    index = {}
    for j, r in enumerate(rrows):
        key = tuple(_hashable(r[i]) for i in ridx)
        if any(v is None for v in key):
            continue
        index.setdefault(key, []).append(j)
    r_pos = [rnames.index(n) for n in r_out]
    rows, matched = [], set()
    for i in range(left._nrows):
        lrow = [lcols[n][i] for n in lnames]
        key = tuple(_hashable(lcols[k][i]) for k in lkeys)
        hits = list(range(len(rrows))) if how == "cross" else ([] if any(v is None for v in key)
                                                               else index.get(key, []))
        if semi:
            if bool(hits) == (how == "leftsemi"):
                rows.append(lrow)
            continue
        if hits:
            for j in hits:
                matched.add(j)
                rows.append(lrow + [rrows[j][t] for t in r_pos])
        elif how in ("left", "full"):
            rows.append(lrow + [None] * len(r_pos))
    if how in ("right", "full"):
        allm = set()
        for part in left._comm.allgather_object(sorted(matched)):
            allm |= set(part)
        if left._comm.rank == left._comm.world_size - 1:
            for j, r in enumerate(rrows):
                if j not in allm:
                    lrow = [None] * len(lnames)
                    if using:
                        for k_l, k_r in zip(lkeys, rkeys):
                            lrow[lnames.index(k_l)] = r[rnames.index(k_r)]
                    rows.append(lrow + [r[t] for t in r_pos])
    pycols = {f.name: [r[j] for r in rows] for j, f in enumerate(schema.fields)}
    counts = left._comm.allgather_object(len(rows))
    off = sum(counts[: left._comm.rank])
    return frame_from_pycolumns(left._session, schema, pycols, list(range(off, off + len(rows))))


def _apply_join(session, df, lq, jc: JoinClause):
    right, rq = _source_frame(session, jc.right)
    if jc.how == "cross":
        out = _join_frames(df, lq, right, rq, "cross", [], [], False)
        return out if jc.on is None else out.filter(Column(jc.on))
    if jc.using is not None:
        return _join_frames(df, lq, right, rq, jc.how, jc.using, jc.using, True)
    keys, rest = _split_on(jc.on, set(df.columns), set(right.columns))
    if not keys:
        if jc.how != "inner":
            raise NotImplementedError("non-equi outer joins are not supported")
        return _join_frames(df, lq, right, rq, "cross", [], [], False).filter(Column(jc.on))
    if rest and jc.how != "inner":
        raise NotImplementedError("outer joins with non-equality ON conditions are not supported")
    out = _join_frames(df, lq, right, rq, jc.how, [a.col for a, _ in keys], [b.col for _, b in keys], False)
    for c in rest:
        out = out.filter(Column(c))
    return out


def _transform(e: Expr, fn) -> Expr:
    """Bottom-up rewrite of an expression tree (fn returns a replacement or None)."""
    from .column import Func
    r = fn(e)
    if r is not None:
        return r
    if isinstance(e, BinOp):
        return BinOp(e.op, _transform(e.left, fn), _transform(e.right, fn))
    if isinstance(e, Unary):
        return Unary(e.op, _transform(e.child, fn))
    if isinstance(e, Alias):
        return Alias(_transform(e.child, fn), e.alias)
    if isinstance(e, Cast):
        return Cast(_transform(e.child, fn), e.to)
    if isinstance(e, When):
        return When([(_transform(c, fn), _transform(v, fn)) for c, v in e.branches],
                    _transform(e.other, fn) if e.other is not None else None)
    if isinstance(e, Func):
        nf = Func(e.fname, [_transform(a, fn) for a in e.args], e.impl)
        if hasattr(e, "params"):
            nf.params = e.params
        return nf
    if isinstance(e, GetField):
        return GetField(_transform(e.child, fn), e.field)
    if isinstance(e, Subscript):
        return Subscript(_transform(e.child, fn), _transform(e.index, fn))
    return e


def _grouped(df, sel: Select, exprs: List[Expr], null_keys=(), all_keys=None):
    """GROUP BY with arbitrary expressions: aggregates and non-column keys are computed first under
    internal names, then the select items (expressions over keys and aggregates), HAVING and ORDER
    BY are evaluated on that frame. For one grouping set of ROLLUP / CUBE / GROUPING SETS,
    ``null_keys`` are the keys rolled up (null in the output) and ``grouping()`` / ``grouping_id()``
    resolve against ``all_keys``."""
    from .functions_extra import GroupingMarker
    from .group import aggregate
    null_str = {str(k): k for k in null_keys}
    null_types = {sk: k.eval(df).dtype for sk, k in null_str.items()}
    all_names = [str(k) for k in (all_keys if all_keys is not None else sel.group_by)]
    in_set = [str(k) for k in sel.group_by]
    keys, key_names = [], []
    for j, k in enumerate(sel.group_by):
        if isinstance(k, ColRef) and not isinstance(k, QualRef):
            keys.append(k)
            key_names.append(k.col)
        else:
            nm = f"__key{j}"
            keys.append(Alias(k, nm))
            key_names.append(nm)
    key_str = {str(k.child if isinstance(k, Alias) else k): n for k, n in zip(keys, key_names)}
    aggs: List[Expr] = []

    def grab(e):
        if isinstance(e, GroupingMarker):
            v, dt = e.value(all_names, in_set)
            return Cast(Lit(v), dt)
        if not isinstance(e, (Lit, Alias)) and str(e) in null_str:
            return Cast(Lit(None), null_types[str(e)])
        if isinstance(e, AggExpr):
            s_ = str(e)
            for i, a in enumerate(aggs):
                if str(a) == s_:
                    return ColRef(f"__agg{i}")
            aggs.append(e)
            return ColRef(f"__agg{len(aggs) - 1}")
        if not isinstance(e, (Lit,)) and str(e) in key_str and not isinstance(e, Alias):
            return ColRef(key_str[str(e)])
        if isinstance(e, QualRef) and e.col in key_str:
            return ColRef(key_str[e.col])
        return None
    items = [_transform(x, grab) for x in exprs]
    # unaliased items keep their SQL text as the column name (e.g. "sum(v)"), not the internal one
    items = [Alias(it, x.name()) if not isinstance(x, Alias) and it.name() != x.name() else it
             for x, it in zip(exprs, items)]
    having = _transform(sel.having, grab) if sel.having is not None else None
    orders = [SortOrder(_transform(o.expr, grab), o.ascending, o.nulls_first) for o in sel.order_by]
    # ORDER BY an output alias
    out_names = {x.name(): x for x in items}
    orders = [SortOrder(ColRef(o.expr.col), o.ascending, o.nulls_first)
              if isinstance(o.expr, ColRef) and o.expr.col in out_names else o for o in orders]
    agg_df = aggregate(df, keys, [ColRef(n) for n in key_names] + [Alias(a, f"__agg{i}") for i, a in enumerate(aggs)])
    if having is not None:
        agg_df = agg_df.filter(Column(having))
    if orders:
        tmp = agg_df.select(*[Column(c) for c in agg_df.columns], *[Column(x) for x in items
                                                                    if x.name() not in agg_df.columns])
        tmp = tmp.orderBy(*orders)
        return tmp.select(*[Column(ColRef(x.name())) for x in items]), True
    return agg_df.select(*[Column(x) for x in items]), False


def _run(session, sel: Select):
    if sel.source is not None:
        df, lq = _source_frame(session, sel.source)
        for jc in sel.joins:
            df = _apply_join(session, df, lq, jc)
            lq = None
    elif sel.subquery is not None:
        df = _run_query(session, sel.subquery)
    elif sel.table is not None:
        df = session.table(sel.table)
    else:
        df = session.range(1)
    if sel.where is not None:
        df = df.filter(Column(sel.where))
    exprs: List[Expr] = []
    sources = getattr(df, "_sql_sources", None) or {}
    for e, alias in sel.items:
        if isinstance(e, ColRef) and e.col == "*" and not isinstance(e, QualRef):
            exprs += [ColRef(n) for n in df.columns]
        elif isinstance(e, _QualStar):
            cols = sources.get(e.qual)
            if cols is None:
                if e.qual in (sel.table, getattr(sel.source, "alias", None)):
                    cols = df.columns
                else:
                    raise ValueError(f"unknown table alias {e.qual!r}")
            exprs += [Alias(ColRef(c), c.split(".", 1)[1]) if c.startswith(e.qual + ".") else ColRef(c) for c in cols]
        else:
            exprs.append(Alias(e, alias) if alias else e)
    ordered = False
    if sel.grouping_sets is not None:
        import dataclasses
        out = None
        for gs in sel.grouping_sets:
            in_set = {str(k) for k in gs}
            sub = dataclasses.replace(sel, group_by=list(gs), grouping_sets=None, order_by=[], limit=None)
            part, _ = _grouped(df, sub, exprs, null_keys=[k for k in sel.group_by if str(k) not in in_set],
                               all_keys=sel.group_by)
            out = part if out is None else out.union(part)
        df = out
    elif sel.group_by or any(x.is_aggregate() for x in exprs):
        df, ordered = _grouped(df, sel, exprs)
    else:
        out_names = {x.name() for x in exprs}
        if sel.order_by and not sel.distinct and any(
                r not in out_names for o in sel.order_by for r in o.expr.refs()):
            # ORDER BY a source column that is not projected: sort first, then project
            df = df.orderBy(*sel.order_by)
            ordered = True
        df = df.select(*[Column(x) for x in exprs])
    if sel.distinct:
        df = df.distinct()
    if sel.order_by and not ordered:
        df = df.orderBy(*[SortOrder(_rewrite_aggs(o.expr, exprs), o.ascending, o.nulls_first)
                          for o in sel.order_by])
    if sel.limit is not None:
        df = df.limit(sel.limit)
    return df


def _rewrite_aggs(e: Expr, items: List[Expr]) -> Expr:
    """Replace aggregate sub-expressions by references to the matching output column."""
    if isinstance(e, AggExpr):
        s = str(e)
        for it in items:
            inner = it.child if isinstance(it, Alias) else it
            if str(inner) == s:
                return ColRef(it.name())
        return ColRef(s)
    if isinstance(e, BinOp):
        return BinOp(e.op, _rewrite_aggs(e.left, items), _rewrite_aggs(e.right, items))
    if isinstance(e, Unary):
        return Unary(e.op, _rewrite_aggs(e.child, items))
    return e
