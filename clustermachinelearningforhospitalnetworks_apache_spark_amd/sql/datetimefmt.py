"""Spark datetime patterns (java.time.format.DateTimeFormatter letters, as used by ``date_format``,
``to_timestamp(col, fmt)``, ``to_date(col, fmt)``, ``unix_timestamp(col, fmt)``, ``from_unixtime``
and the CSV/JSON ``timestampFormat`` option) compiled once into a formatter and a regex parser.

Supported letters: y (year: yyyy / yy), M / L (month: M, MM, MMM, MMMM), d, D (day of year), H, h, k, K,
m, s, S… (fraction), a (AM/PM), E (EEE / EEEE), and 'quoted literals' ('' for a quote). Zone
letters (X, x, Z, z, V, O) format as UTC / parse an offset. A value that does not parse gives
null, like Spark's non-ANSI mode.
"""
from __future__ import annotations

import datetime as _dt
import re
from functools import lru_cache
from typing import Callable, List, Optional, Tuple

_MONTHS = ["January", "February", "March", "April", "May", "June", "July", "August", "September", "October",
           "November", "December"]
_DAYS = ["Monday", "Tuesday", "Wednesday", "Thursday", "Friday", "Saturday", "Sunday"]


def _tokens(pattern: str) -> List[Tuple[str, str]]:
    """[(kind, text)]: kind 'lit' or a pattern letter run such as 'yyyy'."""
    out: List[Tuple[str, str]] = []
    i, n = 0, len(pattern)
    while i < n:
        ch = pattern[i]
        if ch == "'":
            j = i + 1
            lit = []
            while j < n:
                if pattern[j] == "'":
                    if j + 1 < n and pattern[j + 1] == "'":
                        lit.append("'")
                        j += 2
                        continue
                    break
                lit.append(pattern[j])
                j += 1
            out.append(("lit", "".join(lit) if j > i + 1 else "'"))
            i = j + 1
        elif ch.isalpha():
            j = i
            while j < n and pattern[j] == ch:
                j += 1
            out.append((ch, pattern[i:j]))
            i = j
        else:
            out.append(("lit", ch))
            i += 1
    return out


def _fmt_token(kind: str, run: str, t: _dt.datetime) -> str:
    w = len(run)
    if kind == "lit":
        return run
    if kind in "yu":
        return f"{t.year % 100:02d}" if w == 2 else f"{t.year:0{w}d}"
    if kind in "ML":
        if w >= 4:
            return _MONTHS[t.month - 1]
        if w == 3:
            return _MONTHS[t.month - 1][:3]
        return f"{t.month:0{w}d}"
    if kind == "d":
        return f"{t.day:0{w}d}"
    if kind == "D":
        return f"{t.timetuple().tm_yday:0{w}d}"
    if kind == "H":
        return f"{t.hour:0{w}d}"
    if kind == "k":
        return f"{t.hour or 24:0{w}d}"
    if kind == "h":
        return f"{(t.hour % 12) or 12:0{w}d}"
    if kind == "K":
        return f"{t.hour % 12:0{w}d}"
    if kind == "m":
        return f"{t.minute:0{w}d}"
    if kind == "s":
        return f"{t.second:0{w}d}"
    if kind == "S":
        return f"{t.microsecond:06d}"[:w].ljust(w, "0")
    if kind == "a":
        return "AM" if t.hour < 12 else "PM"
    if kind == "E":
        name = _DAYS[t.weekday()]
        return name if w >= 4 else name[:3]
    if kind in "XxZOVz":
        if kind == "X":
            return "Z"
        if kind == "Z":
            return "+0000"
        if kind == "x":
            return "+00"
        return "UTC"
    raise ValueError(f"unsupported datetime pattern letter {kind!r}")


@lru_cache(maxsize=256)
def formatter(pattern: str) -> Callable[[_dt.datetime], str]:
    toks = _tokens(pattern)
    for kind, run in toks:
        if kind != "lit":
            _fmt_token(kind, run, _dt.datetime(2000, 1, 1))  # validate letters once

    def fmt(t) -> str:
        if isinstance(t, _dt.date) and not isinstance(t, _dt.datetime):
            t = _dt.datetime(t.year, t.month, t.day)
        return "".join(_fmt_token(k, r, t) for k, r in toks)
    return fmt


def _rx_token(kind: str, run: str) -> Tuple[str, Optional[str]]:
    w = len(run)
    if kind == "lit":
        return re.escape(run), None
    if kind in "yu":
        return (r"(\d{2})", "yy") if w == 2 else (r"([+-]?\d{4,9})" if w >= 4 else r"(\d{1,9})", "y")
    if kind in "ML":
        if w >= 4:
            return "(" + "|".join(_MONTHS) + ")", "MMMM"
        if w == 3:
            return "(" + "|".join(m[:3] for m in _MONTHS) + ")", "MMM"
        return (r"(\d{1,2})" if w == 1 else r"(\d{2})"), "M"
    if kind in "dHhkKms":
        return (r"(\d{1,2})" if w == 1 else r"(\d{2})"), kind
    if kind == "D":
        return r"(\d{1,3})", "D"
    if kind == "S":
        return rf"(\d{{1,{max(w, 1)}}})", "S"
    if kind == "a":
        return r"(AM|PM|am|pm)", "a"
    if kind == "E":
        return "(" + "|".join(_DAYS + [d[:3] for d in _DAYS]) + ")", None
    if kind in "XxZOVz":
        return r"(Z|UTC|GMT|[+-]\d{2}:?\d{2}|[+-]\d{2})", "zone"
    raise ValueError(f"unsupported datetime pattern letter {kind!r}")


@lru_cache(maxsize=256)
def parser(pattern: str) -> Callable[[str], Optional[_dt.datetime]]:
    """str -> naive UTC datetime, or None when the text does not match the whole pattern."""
    parts, fields = [], []
    for kind, run in _tokens(pattern):
        rx, f = _rx_token(kind, run)
        parts.append(rx)
        if f is not None:
            fields.append(f)
    rx = re.compile("^" + "".join(parts) + "$")

    def parse(s) -> Optional[_dt.datetime]:
        if s is None:
            return None
        m = rx.match(str(s).strip())
        if m is None:
            return None
        v = dict(year=1970, month=1, day=1, hour=0, minute=0, second=0, us=0)
        pm = None
        hour12 = None
        off = None
        doy = None
        for f, g in zip(fields, m.groups()):
            if f == "y":
                v["year"] = int(g)
            elif f == "yy":
                v["year"] = 2000 + int(g)
            elif f == "M":
                v["month"] = int(g)
            elif f == "MMM":
                v["month"] = [x[:3] for x in _MONTHS].index(g) + 1
            elif f == "MMMM":
                v["month"] = _MONTHS.index(g) + 1
            elif f == "d":
                v["day"] = int(g)
            elif f == "D":
                doy = int(g)
            elif f in "Hk":
                v["hour"] = int(g) % 24
            elif f in "hK":
                hour12 = int(g) % 12
            elif f == "m":
                v["minute"] = int(g)
            elif f == "s":
                v["second"] = int(g)
            elif f == "S":
                v["us"] = int(g.ljust(6, "0")[:6])
            elif f == "a":
                pm = g.upper() == "PM"
            elif f == "zone":
                if g in ("Z", "UTC", "GMT"):
                    off = 0
                else:
                    sign = -1 if g[0] == "-" else 1
                    digits = g[1:].replace(":", "")
                    off = sign * (int(digits[:2]) * 60 + (int(digits[2:4]) if len(digits) >= 4 else 0))
        if hour12 is not None:
            v["hour"] = hour12 + (12 if pm else 0)
        elif pm is not None and pm and v["hour"] < 12:
            v["hour"] += 12
        try:
            t = _dt.datetime(v["year"], v["month"], v["day"], v["hour"], v["minute"], v["second"], v["us"])
            if doy is not None:
                t = t.replace(month=1, day=1) + _dt.timedelta(days=doy - 1)
        except ValueError:
            return None
        if off:
            t = t - _dt.timedelta(minutes=off)
        return t
    return parse


__all__ = ["formatter", "parser"]
