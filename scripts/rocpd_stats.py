"""Kernel statistics from a rocprofv3 rocpd database (``--kernel-trace``; rocprofv3 of ROCm 7 writes
``*_results.db``): whole run, or the window between the i-th and (i+1)-th dispatch of a marker kernel
(e.g. the row pass that opens every KMeans fit), with GPU-busy vs wall time of the window.

    python scripts/rocpd_stats.py DB [--marker row_pass_kernel --index 1] [--top 30] [--timeline]
"""
import argparse
import re
import sqlite3
from collections import defaultdict


def short(name: str) -> str:
    name = re.sub(r"\(anonymous namespace\)::", "", name)
    name = re.sub(r"^void ", "", name)
    return name.split("(")[0] if not name.startswith("__") else name


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("db")
    ap.add_argument("--marker", default=None)
    ap.add_argument("--index", type=int, default=0)
    ap.add_argument("--top", type=int, default=30)
    ap.add_argument("--timeline", action="store_true")
    a = ap.parse_args()
    c = sqlite3.connect(a.db)
    rows = list(c.execute("select name, start, end from kernels order by start"))
    lo, hi = rows[0][1], rows[-1][2]
    if a.marker:
        marks = [r[1] for r in rows if a.marker in r[0]]
        lo = marks[a.index]
        hi = marks[a.index + 1] if a.index + 1 < len(marks) else hi
    sel = [r for r in rows if lo <= r[1] < hi]
    tot = defaultdict(lambda: [0, 0.0])
    busy = 0.0
    last_end = lo
    for n, s, e in sel:
        t = (e - s) / 1e6
        tot[short(n)][0] += 1
        tot[short(n)][1] += t
        busy += max(0.0, (e - max(s, last_end)) / 1e6)
        last_end = max(last_end, e)
    wall = (sel[-1][2] - sel[0][1]) / 1e6 if sel else 0.0
    print(f"window: {len(sel)} dispatches, first start -> last end {wall:.3f} ms, GPU busy {busy:.3f} ms")
    for name, (cnt, t) in sorted(tot.items(), key=lambda kv: -kv[1][1])[: a.top]:
        print(f"{name[:88]:88s} {cnt:6d} {t:10.3f} ms {100 * t / max(busy, 1e-9):6.2f}%")
    if a.timeline:
        for n, s, e in sel:
            print(f"{(s - lo) / 1e6:10.3f} {(e - s) / 1e6:9.3f}  {short(n)[:90]}")


if __name__ == "__main__":
    main()
