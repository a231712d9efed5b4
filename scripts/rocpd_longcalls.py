"""Longest host runtime calls in a rocprofv3 trace (``--kernel-trace --runtime-trace``), with the kernels
dispatched in the 2 ms after each: ``python scripts/rocpd_longcalls.py DB [--top 20] [--min-ms 1]``."""
import argparse
import sqlite3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("db")
    ap.add_argument("--top", type=int, default=20)
    ap.add_argument("--min-ms", type=float, default=1.0)
    a = ap.parse_args()
    c = sqlite3.connect(a.db)
    t0 = c.execute("select min(start) from regions").fetchone()[0]
    rows = list(c.execute("select name, start, end from regions where end - start >= ? order by end - start desc "
                          "limit ?", (int(a.min_ms * 1e6), a.top)))
    for n, s, e in rows:
        ks = [k for k, in c.execute("select name from kernels where start >= ? and start < ? order by start limit 3",
                                    (s, e + 2_000_000))]
        print(f"{(e - s) / 1e6:9.2f} ms at {(s - t0) / 1e6:10.2f} ms  {n:32s} next: {'; '.join(k[:60] for k in ks)}")


if __name__ == "__main__":
    main()
