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
from .column import AggExpr, Alias, BinOp, Cast, ColRef, Column, Expr, Lit, SortOrder, Unary, When

_TOKEN = re.compile(r"""
    \s*(?:
      (?P<num>\d+\.\d*(?:[eE][-+]?\d+)?|\.\d+(?:[eE][-+]?\d+)?|\d+(?:[eE][-+]?\d+)?)
    | (?P<str>'(?:[^']|'')*')
    | (?P<dstr>"(?:[^"]|"")*")
    | (?P<ident>`[^`]+`|[A-Za-z_][A-Za-z_0-9]*(?:\.[A-Za-z_][A-Za-z_0-9]*)*)
    | (?P<op><=>|<=|>=|<>|!=|==|\|\||[-+*/%(),=<>.])
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
            elif self.at_op("=", "==", "!=", "<>", "<", "<=", ">", ">=", "<=>"):
                op = self.take().val
                op = {"=": "==", "<>": "!=", "<=>": "=="}.get(op, op)
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
            else:
                e = BinOp(op, e, rhs)
        return e

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
        return self.primary()

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
            name = tok.val.split(".")[-1] if "." in tok.val else tok.val
            return ColRef(name)
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
        distinct = False
        if self.at_kw("DISTINCT"):
            self.take()
            distinct = True
        args: List[Expr] = []
        if self.at_op("*"):
            self.take()
            args = []
        elif not self.at_op(")"):
            args.append(self.expr())
            while self.at_op(","):
                self.take()
                args.append(self.expr())
        self.expect_op(")")
        e = self._call_expr(name, lname, args, distinct)
        if self.at_word("OVER"):
            self.take()
            from .window import WindowExpr
            e = WindowExpr(e, self.window_spec())
        return e

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
        fn = getattr(F, lname, None)
        if fn is None:
            raise SyntaxError(f"unknown function {name}")
        lit_pos = _LIT_ARGS.get(lname, ())
        cols = [a.value if (i in lit_pos and isinstance(a, Lit)) else Column(a) for i, a in enumerate(args)]
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


def parse_select(sql: str) -> Select:
    p = Parser(tokenize(sql))
    sel = _select(p)
    if p.peek() is not None:
        raise SyntaxError(f"unexpected trailing SQL: {p.peek().val!r}")
    return sel


def _select(p: Parser) -> Select:
    p.expect_kw("SELECT")
    distinct = False
    if p.at_kw("DISTINCT"):
        p.take()
        distinct = True
    items = [_select_item(p)]
    while p.at_op(","):
        p.take()
        items.append(_select_item(p))
    table, sub = None, None
    if p.at_kw("FROM"):
        p.take()
        if p.at_op("("):
            p.take()
            sub = _select(p)
            p.expect_op(")")
        else:
            table = p.take().val
        if p.at_kw("AS"):
            p.take()
            p.take()
        elif p.peek() is not None and p.peek().kind == "ident":
            p.take()  # table alias
    sel = Select(items, table, distinct=distinct, subquery=sub)
    if p.at_kw("WHERE"):
        p.take()
        sel.where = p.expr()
    if p.at_kw("GROUP"):
        p.take()
        p.expect_kw("BY")
        sel.group_by.append(p.expr())
        while p.at_op(","):
            p.take()
            sel.group_by.append(p.expr())
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


def _select_item(p: Parser):
    e = p.expr()
    alias = None
    if p.at_kw("AS"):
        p.take()
        alias = p.take().val
    elif p.peek() is not None and p.peek().kind == "ident":
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


def execute(session, sql: str):
    """Run a SELECT against the session catalog; returns a DataFrame."""
    sel = parse_select(sql)
    return _run(session, sel)


def _run(session, sel: Select):
    from .dataframe import DataFrame
    if sel.subquery is not None:
        df = _run(session, sel.subquery)
    elif sel.table is not None:
        df = session.table(sel.table)
    else:
        df = session.range(1)
    if sel.where is not None:
        df = df.filter(Column(sel.where))
    exprs: List[Expr] = []
    for e, alias in sel.items:
        if isinstance(e, ColRef) and e.col == "*":
            exprs += [ColRef(n) for n in df.columns]
        else:
            exprs.append(Alias(e, alias) if alias else e)
    ordered = False
    if sel.group_by or any(x.is_aggregate() for x in exprs):
        from .group import aggregate
        out = aggregate(df, sel.group_by, exprs)
        if sel.having is not None:
            out = out.filter(Column(_rewrite_aggs(sel.having, exprs)))
        df = out
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
