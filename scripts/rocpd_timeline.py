"""Summaries of a rocprofv3 rocpd database (run_results.db): per-kernel stats and a timeline.

usage: python scripts/rocpd_timeline.py DB [--after NAME_SUBSTR] [--limit N] [--stats]
--after: start the timeline at the first kernel whose name contains NAME_SUBSTR (e.g. the first
row-norm kernel of the timed fit); --stats: per-kernel totals of the (selected) range instead."""
import argparse
import re
import sqlite3
from collections import defaultdict


def short(n):
    n = re.sub(r"\(anonymous namespace\)::", "", n)
    n = re.sub(r"^void ", "", n)
    return n.split("(")[0][:80]


ap = argparse.ArgumentParser()
ap.add_argument("db")
ap.add_argument("--after", default=None)
ap.add_argument("--skip", type=int, default=0, help="skip this many matches of --after")
ap.add_argument("--limit", type=int, default=200)
ap.add_argument("--stats", action="store_true")
a = ap.parse_args()
rows = sqlite3.connect(a.db).execute("select name, start, end from kernels order by start").fetchall()
i0 = 0
if a.after:
    hits = [i for i, r in enumerate(rows) if a.after in r[0]]
    i0 = hits[min(a.skip, len(hits) - 1)] if hits else 0
sel = rows[i0:i0 + a.limit] if not a.stats else rows[i0:]
if a.stats:
    agg = defaultdict(lambda: [0, 0])
    for name, s, e in sel:
        agg[short(name)][0] += 1
        agg[short(name)][1] += e - s
    tot = sum(v[1] for v in agg.values())
    for k, (c, t) in sorted(agg.items(), key=lambda kv: -kv[1][1])[:a.limit]:
        print(f"{k:80s} {c:6d} {t / 1e6:10.3f} ms {100 * t / tot:6.2f}%")
else:
    t0 = sel[0][1]
    prev = t0
    for name, s, e in sel:
        print(f"{(s - t0) / 1e6:10.3f} gap {(s - prev) / 1e6:7.3f} dur {(e - s) / 1e6:8.3f}  {short(name)}")
        prev = e
