"""Merged timeline of one window of a rocprofv3 database (``--kernel-trace --runtime-trace
[--marker-trace]``): kernels (start offset, gap before, duration), blocking HIP runtime calls and roctx
ranges, in time order, between the i-th and (i+1)-th dispatch of a marker kernel.

    python scripts/rocpd_timeline.py DB --marker row_pass_kernel --index 1 [--gap-apis US]

``--gap-apis US``: after the timeline, every idle gap of at least US microseconds between kernels with the HIP
runtime calls the host made during it (name, count, total time): what the host was doing while the GPU waited.
"""
import argparse
import re
import sqlite3

BLOCKING = ("hipMemcpyWithStream", "hipMemcpy", "hipStreamSynchronize", "hipDeviceSynchronize",
            "hipEventSynchronize", "hipMemcpyDtoH", "hipMemset", "hipMemcpyAsync")


def short(n):
    n = re.sub(r"\(anonymous namespace\)::", "", n)
    n = re.sub(r"^void ", "", n)
    return n.split("(")[0][:70]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("db")
    ap.add_argument("--marker", default="row_pass_kernel")
    ap.add_argument("--index", type=int, default=1)
    ap.add_argument("--end-marker", default=None, help="window ends at the next dispatch of this kernel")
    ap.add_argument("--gap-apis", type=float, default=0.0)
    ap.add_argument("--gap-detail", type=float, default=0.0, help="gaps of at least this many us: every call listed")
    a = ap.parse_args()
    c = sqlite3.connect(a.db)
    ks = list(c.execute("select name, start, end from kernels order by start"))
    marks = [s for n, s, e in ks if a.marker in n]
    lo = marks[a.index]
    hi = marks[a.index + 1] if a.index + 1 < len(marks) else ks[-1][2] + 1
    sel = [(n, s, e) for n, s, e in ks if lo <= s < hi]
    ev = [(s, "K", short(n), e - s) for n, s, e in sel]
    try:
        regs = list(c.execute("select name, start, end from regions where start >= ? and start < ?",
                              (lo - 5_000_000, sel[-1][2])))
    except sqlite3.Error:
        regs = []
    for n, s, e in regs:
        if n in BLOCKING:
            ev.append((s, "B", n, e - s))
        elif n.startswith(("kmeans", "kinit", "fit", "lloyd")):
            ev.append((s, "R", n, e - s))
    ev.sort()
    t0 = lo
    kend = lo
    busy = 0
    for t, kind, name, dur in ev:
        if kind == "K":
            gap = max(0, t - kend)
            print(f"{(t - t0) / 1e6:9.3f} K gap {gap / 1e3:7.1f}us dur {dur / 1e3:8.1f}us  {name}")
            kend = max(kend, t + dur)
            busy += dur
        else:
            print(f"{(t - t0) / 1e6:9.3f} {kind} {'':17s} dur {dur / 1e3:8.1f}us  [{name}]")
    span = sel[-1][2] - lo
    print(f"window {span / 1e6:.3f} ms, {len(sel)} kernels, kernel time {busy / 1e6:.3f} ms")
    if a.gap_apis > 0:
        try:
            api = list(c.execute("select name, start, end from regions where start >= ? and start < ? order by start",
                                 (lo, sel[-1][2])))
        except sqlite3.Error:
            api = []
        kend = lo
        for n, s0, e0 in sel:
            if s0 - kend >= a.gap_apis * 1e3:
                agg = {}
                for an, as_, ae in api:
                    if kend <= as_ < s0:
                        c_, t_ = agg.get(an, (0, 0))
                        agg[an] = (c_ + 1, t_ + ae - as_)
                top = sorted(agg.items(), key=lambda kv: -kv[1][1])[:8]
                desc = ", ".join(f"{k} x{v[0]} {v[1] / 1e3:.0f}us" for k, v in top)
                print(f"gap {(kend - lo) / 1e6:9.3f} -> {(s0 - lo) / 1e6:9.3f} ms ({(s0 - kend) / 1e3:6.1f} us) "
                      f"before {short(n)}: {desc or 'no runtime calls'}")
                if a.gap_detail > 0 and s0 - kend >= a.gap_detail * 1e3:
                    for an, as_, ae in api:
                        if kend - 50_000 <= as_ < s0 and an not in ("hipGetDevice", "hipSetDevice", "hipGetLastError"):
                            print(f"      {(as_ - lo) / 1e6:9.3f} ms  {(ae - as_) / 1e3:7.1f} us  {an}")
            kend = max(kend, e0)


if __name__ == "__main__":
    main()
