"""Host synchronisation inside a window of a rocprofv3 trace (``--kernel-trace --runtime-trace``):
blocking HIP runtime calls (synchronous copies, stream/device/event synchronize) between the i-th and
(i+1)-th dispatch of a marker kernel, and the GPU idle gaps longer than a threshold in that window.

    python scripts/rocpd_syncs.py DB --marker row_pass_kernel --index 1 [--gap-us 20]
"""
import argparse
import sqlite3

BLOCKING = ("hipMemcpyWithStream", "hipMemcpy", "hipStreamSynchronize", "hipDeviceSynchronize",
            "hipEventSynchronize", "hipMemcpyDtoH", "hipMemset")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("db")
    ap.add_argument("--marker", default="row_pass_kernel")
    ap.add_argument("--index", type=int, default=1)
    ap.add_argument("--gap-us", type=float, default=20.0)
    ap.add_argument("--after-ms", type=float, default=0.0, help="only gaps this far into the window")
    ap.add_argument("--show", type=int, default=40)
    a = ap.parse_args()
    c = sqlite3.connect(a.db)
    ks = list(c.execute("select name, start, end from kernels order by start"))
    marks = [s for n, s, e in ks if a.marker in n]
    lo = marks[a.index]
    hi = marks[a.index + 1] if a.index + 1 < len(marks) else ks[-1][2]
    sel = [(n, s, e) for n, s, e in ks if lo <= s < hi]
    print(f"window {(sel[-1][2] - lo) / 1e6:.3f} ms, {len(sel)} kernels")
    calls = list(c.execute("select name, start, end from regions where start >= ? and start < ? order by start",
                           (lo, sel[-1][2])))
    cnt = {}
    for n, s, e in calls:
        if n in BLOCKING:
            cnt[n] = cnt.get(n, 0) + 1
    print("blocking runtime calls in the window:", cnt)
    gaps = []
    end = sel[0][2]
    for n, s, e in sel[1:]:
        if s - end > a.gap_us * 1e3 and (end - lo) / 1e6 >= a.after_ms:
            gaps.append(((s - end) / 1e3, (end - lo) / 1e6, n[:60]))
        end = max(end, e)
    tot = sum(g[0] for g in gaps)
    print(f"GPU idle gaps > {a.gap_us:g} us after {a.after_ms:g} ms: {len(gaps)}, total {tot / 1e3:.3f} ms")
    for g in gaps[: a.show]:
        print(f"  {g[0]:8.1f} us at {g[1]:8.3f} ms before {g[2]}")


if __name__ == "__main__":
    main()
