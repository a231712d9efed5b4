"""Collective/compute overlap from a rocprofv3 kernel trace (run_results.db).

usage: python scripts/rocpd_streams.py DB [--after NAME_SUBSTR] [--skip N] [--limit N]
For every RCCL kernel (name contains "nccl"/"rccl") after the marker kernel: its queue, start/duration,
and the compute kernels of OTHER queues that overlap it in time (with the overlapped microseconds).
The summary line gives total collective time and the part of it hidden under compute."""
import argparse
import re
import sqlite3


def short(n):
    n = re.sub(r"\(anonymous namespace\)::", "", n)
    n = re.sub(r"^void ", "", n)
    return n.split("(")[0][:60]


ap = argparse.ArgumentParser()
ap.add_argument("db")
ap.add_argument("--after", default="row_pass_kernel")
ap.add_argument("--skip", type=int, default=1)
ap.add_argument("--limit", type=int, default=60)
a = ap.parse_args()
rows = sqlite3.connect(a.db).execute("select name, start, end, queue_id from kernels order by start").fetchall()
hits = [i for i, r in enumerate(rows) if a.after in r[0]]
i0 = hits[min(a.skip, len(hits) - 1)] if hits else 0
rows = rows[i0:]
t0 = rows[0][1] if rows else 0
coll = [r for r in rows if re.search(r"nccl|rccl", r[0], re.I)]
comp = [r for r in rows if not re.search(r"nccl|rccl", r[0], re.I)]
tot = hid = 0
print(f"{len(coll)} collective kernels after '{a.after}' #{a.skip}; queues: collective "
      f"{sorted({r[3] for r in coll})}, compute {sorted({r[3] for r in comp})}")
for j, (name, s, e, q) in enumerate(coll):
    ov = []
    cover = 0
    for (cn, cs, ce, cq) in comp:
        if cq != q and cs < e and ce > s:
            o = min(e, ce) - max(s, cs)
            cover += o
            ov.append(f"{short(cn)} {o / 1e3:.1f}us")
    cover = min(cover, e - s)
    tot += e - s
    hid += cover
    if j < a.limit:
        print(f"{(s - t0) / 1e6:10.3f} ms q{q} dur {(e - s) / 1e3:8.1f} us  {short(name)}  | overlaps: "
              + ("; ".join(ov[:4]) if ov else "none"))
print(f"collective time {tot / 1e6:.3f} ms, overlapped with compute on other queues {hid / 1e6:.3f} ms "
      f"({100.0 * hid / max(tot, 1):.1f}%)")
