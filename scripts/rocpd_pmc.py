"""Summarise rocprofv3 PMC databases (rocpd sqlite): per kernel (name filter), the counter values of
each dispatch (summed over instances) and the mean over dispatches.
Usage: python scripts/rocpd_pmc.py <db> [<db> ...] [--kernel SUBSTR]"""
import argparse
import collections
import sqlite3


def summarise(path, sub):
    db = sqlite3.connect(path)
    rows = db.execute("select dispatch_id, kernel_name, counter_name, sum(value), max(duration), "
                      "max(vgpr_count), max(accum_vgpr_count), max(sgpr_count), max(lds_block_size) "
                      "from counters_collection group by dispatch_id, counter_name").fetchall()
    per = collections.defaultdict(dict)
    meta = {}
    for did, kname, cname, val, dur, vg, ag, sg, lds in rows:
        if sub and sub not in kname:
            continue
        per[(did, kname)][cname] = val
        meta[(did, kname)] = (dur, vg, ag, sg, lds)
    by_kernel = collections.defaultdict(list)
    for (did, kname), c in per.items():
        by_kernel[kname].append((did, c, meta[(did, kname)]))
    for kname, lst in by_kernel.items():
        lst.sort()
        print(f"== {kname[:140]}")
        dur, vg, ag, sg, lds = lst[-1][2]
        print(f"   dispatches {len(lst)}  vgpr {vg} agpr {ag} sgpr {sg} lds {lds}")
        names = sorted({n for _, c, _ in lst for n in c})
        for n in names:
            vals = [c[n] for _, c, _ in lst if n in c]
            print(f"   {n:32s} mean {sum(vals) / len(vals):16.4g}   last {vals[-1]:16.4g}")


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("db", nargs="+")
    ap.add_argument("--kernel", default="")
    a = ap.parse_args()
    for p in a.db:
        print(f"# {p}")
        summarise(p, a.kernel)
