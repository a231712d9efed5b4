"""Profile analysis for rocprofv3 output: one tool, one subcommand per view.

rocpd databases (``rocprofv3 ... -d DIR -o NAME`` writes ``DIR/NAME_results.db``):

    python scripts/prof.py stats DB [--marker row_pass_kernel --index 1] [--top 30] [--timeline]
        per-kernel time of the whole run or of the window between the i-th and (i+1)-th dispatch of a marker
        kernel (the row pass opens every KMeans fit), with GPU-busy vs wall time of the window
    python scripts/prof.py timeline DB [--marker M --index I] [--gap-apis US] [--gap-detail US]
        merged kernel / blocking HIP call / roctx timeline of the window (``--runtime-trace --marker-trace``);
        --gap-apis lists the host calls made during every idle gap of at least US microseconds
    python scripts/prof.py syncs DB [--marker M --index I] [--gap-us 20] [--show 40]
        blocking runtime calls and GPU idle gaps in the window
    python scripts/prof.py streams DB [--after row_pass_kernel] [--skip 1]
        every RCCL kernel, and the compute kernels of other queues that overlap it
    python scripts/prof.py longcalls DB [--top 20] [--min-ms 1]
        longest host runtime calls, with the kernels dispatched right after each
    python scripts/prof.py pmc DB [DB ...] [--kernel SUBSTR]
        PMC databases (``--pmc``): counter values per dispatch and their mean per kernel

CSV output (``--output-format csv``):

    python scripts/prof.py pmccsv DIR [SUBSTR]
        per-dispatch clock, MFMA busy share, wave-cycle split and HBM rate from ``*/*counter_collection.csv``
    python scripts/prof.py kcsv kernel_stats.csv [N]
        top N rows of a ``--stats`` kernel table with short names

Static:

    python scripts/prof.py kres SRC.hip [FILTER]
        VGPRs / spills / occupancy per kernel of a .hip file for gfx950 (hipcc resource-usage remarks)
"""
import argparse
import collections
import csv
import glob
import os
import re
import sqlite3
import subprocess

BLOCKING = ("hipMemcpyWithStream", "hipMemcpy", "hipStreamSynchronize", "hipDeviceSynchronize",
            "hipEventSynchronize", "hipMemcpyDtoH", "hipMemset")


def short(name: str, width: int = 90) -> str:
    name = re.sub(r"\(anonymous namespace\)::", "", name)
    name = re.sub(r"^void ", "", name)
    return (name.split("(")[0] if not name.startswith("__") else name)[:width]


def kernels(db):
    return list(db.execute("select name, start, end from kernels order by start"))


def window(ks, marker, index):
    """[lo, hi) between the index-th and (index+1)-th dispatch of the marker kernel (the whole run without one)."""
    if not marker:
        return ks[0][1], ks[-1][2] + 1
    marks = [s for n, s, e in ks if marker in n]
    lo = marks[index]
    return lo, (marks[index + 1] if index + 1 < len(marks) else ks[-1][2] + 1)


def regions(db, lo, hi):
    try:
        return list(db.execute("select name, start, end from regions where start >= ? and start < ? order by start",
                               (lo, hi)))
    except sqlite3.Error:  # no --runtime-trace in this database
        return []


def cmd_stats(a):
    ks = kernels(sqlite3.connect(a.db))
    lo, hi = window(ks, a.marker, a.index)
    sel = [r for r in ks if lo <= r[1] < hi]
    tot = collections.defaultdict(lambda: [0, 0.0])
    busy, last_end = 0.0, lo
    for n, s, e in sel:
        tot[short(n)][0] += 1
        tot[short(n)][1] += (e - s) / 1e6
        busy += max(0.0, (e - max(s, last_end)) / 1e6)
        last_end = max(last_end, e)
    wall = (sel[-1][2] - sel[0][1]) / 1e6 if sel else 0.0
    print(f"window: {len(sel)} dispatches, first start -> last end {wall:.3f} ms, GPU busy {busy:.3f} ms")
    for name, (cnt, t) in sorted(tot.items(), key=lambda kv: -kv[1][1])[: a.top]:
        print(f"{name[:88]:88s} {cnt:6d} {t:10.3f} ms {100 * t / max(busy, 1e-9):6.2f}%")
    if a.timeline:
        for n, s, e in sel:
            print(f"{(s - lo) / 1e6:10.3f} {(e - s) / 1e6:9.3f}  {short(n)}")


def cmd_timeline(a):
    db = sqlite3.connect(a.db)
    ks = kernels(db)
    lo, hi = window(ks, a.marker, a.index)
    sel = [(n, s, e) for n, s, e in ks if lo <= s < hi]
    ev = [(s, "K", short(n, 70), e - s) for n, s, e in sel]
    for n, s, e in regions(db, lo - 5_000_000, sel[-1][2]):
        if n in BLOCKING or n == "hipMemcpyAsync":
            ev.append((s, "B", n, e - s))
        elif n.startswith(("kmeans", "kinit", "fit", "lloyd")):
            ev.append((s, "R", n, e - s))
    ev.sort()
    kend, busy = lo, 0
    for t, kind, name, dur in ev:
        if kind == "K":
            print(f"{(t - lo) / 1e6:9.3f} K gap {max(0, t - kend) / 1e3:7.1f}us dur {dur / 1e3:8.1f}us  {name}")
            kend = max(kend, t + dur)
            busy += dur
        else:
            print(f"{(t - lo) / 1e6:9.3f} {kind} {'':17s} dur {dur / 1e3:8.1f}us  [{name}]")
    print(f"window {(sel[-1][2] - lo) / 1e6:.3f} ms, {len(sel)} kernels, kernel time {busy / 1e6:.3f} ms")
    if a.gap_apis <= 0:
        return
    api = regions(db, lo, sel[-1][2])
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
                  f"before {short(n, 70)}: {desc or 'no runtime calls'}")
            if a.gap_detail > 0 and s0 - kend >= a.gap_detail * 1e3:
                for an, as_, ae in api:
                    if kend - 50_000 <= as_ < s0 and an not in ("hipGetDevice", "hipSetDevice", "hipGetLastError"):
                        print(f"      {(as_ - lo) / 1e6:9.3f} ms  {(ae - as_) / 1e3:7.1f} us  {an}")
        kend = max(kend, e0)


def cmd_syncs(a):
    db = sqlite3.connect(a.db)
    ks = kernels(db)
    lo, hi = window(ks, a.marker, a.index)
    sel = [(n, s, e) for n, s, e in ks if lo <= s < hi]
    print(f"window {(sel[-1][2] - lo) / 1e6:.3f} ms, {len(sel)} kernels")
    cnt = collections.Counter(n for n, s, e in regions(db, lo, sel[-1][2]) if n in BLOCKING)
    print("blocking runtime calls in the window:", dict(cnt))
    gaps, end = [], sel[0][2]
    for n, s, e in sel[1:]:
        if s - end > a.gap_us * 1e3 and (end - lo) / 1e6 >= a.after_ms:
            gaps.append(((s - end) / 1e3, (end - lo) / 1e6, n[:60]))
        end = max(end, e)
    print(f"GPU idle gaps > {a.gap_us:g} us after {a.after_ms:g} ms: {len(gaps)}, "
          f"total {sum(g[0] for g in gaps) / 1e3:.3f} ms")
    for g in gaps[: a.show]:
        print(f"  {g[0]:8.1f} us at {g[1]:8.3f} ms before {g[2]}")


def cmd_streams(a):
    rows = sqlite3.connect(a.db).execute("select name, start, end, queue_id from kernels order by start").fetchall()
    hits = [i for i, r in enumerate(rows) if a.after in r[0]]
    rows = rows[hits[min(a.skip, len(hits) - 1)]:] if hits else rows
    t0 = rows[0][1] if rows else 0
    is_coll = lambda n: re.search(r"nccl|rccl", n, re.I)  # noqa: E731
    coll = [r for r in rows if is_coll(r[0])]
    comp = [r for r in rows if not is_coll(r[0])]
    tot = hid = 0
    print(f"{len(coll)} collective kernels after '{a.after}' #{a.skip}; queues: collective "
          f"{sorted({r[3] for r in coll})}, compute {sorted({r[3] for r in comp})}")
    for j, (name, s, e, q) in enumerate(coll):
        ov, cover = [], 0
        for cn, cs, ce, cq in comp:
            if cq != q and cs < e and ce > s:
                o = min(e, ce) - max(s, cs)
                cover += o
                ov.append(f"{short(cn, 60)} {o / 1e3:.1f}us")
        tot += e - s
        hid += min(cover, e - s)
        if j < a.limit:
            print(f"{(s - t0) / 1e6:10.3f} ms q{q} dur {(e - s) / 1e3:8.1f} us  {short(name, 60)}  | overlaps: "
                  + ("; ".join(ov[:4]) if ov else "none"))
    print(f"collective time {tot / 1e6:.3f} ms, overlapped with compute on other queues {hid / 1e6:.3f} ms "
          f"({100.0 * hid / max(tot, 1):.1f}%)")


def cmd_longcalls(a):
    db = sqlite3.connect(a.db)
    t0 = db.execute("select min(start) from regions").fetchone()[0]
    rows = list(db.execute("select name, start, end from regions where end - start >= ? order by end - start desc "
                           "limit ?", (int(a.min_ms * 1e6), a.top)))
    for n, s, e in rows:
        ks = [k for k, in db.execute("select name from kernels where start >= ? and start < ? order by start limit 3",
                                     (s, e + 2_000_000))]
        print(f"{(e - s) / 1e6:9.2f} ms at {(s - t0) / 1e6:10.2f} ms  {n:32s} next: {'; '.join(k[:60] for k in ks)}")


def cmd_pmc(a):
    for path in a.db:
        print(f"# {path}")
        rows = sqlite3.connect(path).execute(
            "select dispatch_id, kernel_name, counter_name, sum(value), max(duration), max(vgpr_count), "
            "max(accum_vgpr_count), max(sgpr_count), max(lds_block_size) from counters_collection "
            "group by dispatch_id, counter_name").fetchall()
        per, meta = collections.defaultdict(dict), {}
        for did, kname, cname, val, dur, vg, ag, sg, lds in rows:
            if a.kernel and a.kernel not in kname:
                continue
            per[(did, kname)][cname] = val
            meta[(did, kname)] = (vg, ag, sg, lds)
        by_kernel = collections.defaultdict(list)
        for (did, kname), c in per.items():
            by_kernel[kname].append((did, c, meta[(did, kname)]))
        for kname, lst in by_kernel.items():
            lst.sort()
            vg, ag, sg, lds = lst[-1][2]
            print(f"== {kname[:140]}\n   dispatches {len(lst)}  vgpr {vg} agpr {ag} sgpr {sg} lds {lds}")
            for n in sorted({n for _, c, _ in lst for n in c}):
                vals = [c[n] for _, c, _ in lst if n in c]
                print(f"   {n:32s} mean {sum(vals) / len(vals):16.4g}   last {vals[-1]:16.4g}")


def cmd_pmccsv(a):
    disp = collections.defaultdict(dict)
    fs = glob.glob(os.path.join(a.dir, "*", "*counter_collection.csv")) + \
        glob.glob(os.path.join(a.dir, "*counter_collection.csv"))
    for f in sorted(fs):
        tag = os.path.basename(os.path.dirname(f))
        for r in csv.DictReader(open(f)):
            if a.sub not in r["Kernel_Name"]:
                continue
            d = disp[(tag, int(r["Dispatch_Id"]))]
            d["ms"] = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6
            d["vgpr"] = r["VGPR_Count"]
            d[r["Counter_Name"]] = d.get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
    by_tag = collections.defaultdict(list)
    for (tag, did), d in sorted(disp.items()):
        by_tag[tag].append((did, d))
    for tag, rows in by_tag.items():
        print(f"== {tag}")
        for did, d in rows:
            out = [f"dispatch {did} {d['ms']:.3f} ms vgpr {d['vgpr']}"]
            if "GRBM_GUI_ACTIVE" in d:
                cyc = d["GRBM_GUI_ACTIVE"] / 8  # the counter sums the 8 XCDs
                out.append(f"clock {cyc / d['ms'] / 1e6:.2f} GHz")
                if "SQ_VALU_MFMA_BUSY_CYCLES" in d:
                    out.append(f"MFMA busy {d['SQ_VALU_MFMA_BUSY_CYCLES'] / 1024 / cyc * 100:.0f}%")
                if "SQ_INSTS_VALU" in d:  # a wave64 VALU op holds its 16-lane SIMD 4 cycles (more for f64/trans)
                    out.append(f"VALU issue >= {4 * d['SQ_INSTS_VALU'] / 1024 / cyc * 100:.0f}% of SIMD cycles")
            if "SQ_WAIT_ANY" in d:
                tot = d["SQ_WAIT_ANY"] + d["SQ_WAIT_INST_ANY"] + d["SQ_ACTIVE_INST_ANY"]
                out.append("waves: wait {:.0f}% issue-stall {:.0f}% active {:.0f}%".format(
                    *(100 * d[k] / tot for k in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY"))))
            if "SQ_LDS_BANK_CONFLICT" in d:
                out.append(f"LDS conflict {d['SQ_LDS_BANK_CONFLICT']:.3g} VALU {d.get('SQ_INSTS_VALU', 0):.3g} "
                           f"LDS {d.get('SQ_INSTS_LDS', 0):.3g} coexec {d.get('SQ_VALU_MFMA_COEXEC_CYCLES', 0):.3g}")
            if "FETCH_SIZE" in d:  # FETCH_SIZE is half the streamed bytes on gfx950 (MI355X_MICROARCH.md)
                out.append(f"HBM {2 * d['FETCH_SIZE'] * 1024 / d['ms'] / 1e9:.2f} TB/s (2 x FETCH_SIZE)")
            print(" | ".join(out))


def cmd_kcsv(a):
    for r in list(csv.DictReader(open(a.csv)))[: a.n]:
        print(f"{short(r['Name']):90s} {int(r['Calls']):6d} {float(r['AverageNs']) / 1e6:9.3f} ms "
              f"{float(r['TotalDurationNs']) / 1e6:10.2f} ms {float(r['Percentage']):6.2f}%")


def cmd_kres(a):
    inc = os.path.dirname(a.src) or "."
    r = subprocess.run(["hipcc", "-O3", "-std=c++17", "--offload-arch=gfx950", "--cuda-device-only", "-I", inc, "-c",
                        a.src, "-o", "/tmp/kres.o", "-Rpass-analysis=kernel-resource-usage"],
                       capture_output=True, text=True)
    cur, rows = {}, []
    for line in r.stderr.splitlines():
        m = re.search(r"remark:\s+(Function Name|VGPRs|VGPRs Spill|Occupancy \[waves/SIMD\]|LDS Size \[bytes/block\]): "
                      r"(.*?) \[", line)
        if not m:
            if "error" in line:
                print(line)
            continue
        if m.group(1) == "Function Name":
            cur = {"name": subprocess.run(["c++filt", m.group(2)], capture_output=True, text=True).stdout.strip()}
            rows.append(cur)
        else:
            cur[m.group(1)] = m.group(2)
    for c in rows:
        name = short(c["name"], 70)
        if a.filter in name:
            print(f"{name:70s} vgpr={c.get('VGPRs')} spill={c.get('VGPRs Spill')} "
                  f"occ={c.get('Occupancy [waves/SIMD]')}")


def main(argv=None):
    ap = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    sub = ap.add_subparsers(dest="cmd", required=True)

    def windowed(name, marker=None, index=0):
        p = sub.add_parser(name)
        p.add_argument("db")
        p.add_argument("--marker", default=marker)
        p.add_argument("--index", type=int, default=index)
        return p

    p = windowed("stats")
    p.add_argument("--top", type=int, default=30)
    p.add_argument("--timeline", action="store_true")
    p = windowed("timeline", "row_pass_kernel", 1)
    p.add_argument("--gap-apis", type=float, default=0.0)
    p.add_argument("--gap-detail", type=float, default=0.0, help="gaps of at least this many us: every call listed")
    p = windowed("syncs", "row_pass_kernel", 1)
    p.add_argument("--gap-us", type=float, default=20.0)
    p.add_argument("--after-ms", type=float, default=0.0, help="only gaps this far into the window")
    p.add_argument("--show", type=int, default=40)
    p = sub.add_parser("streams")
    p.add_argument("db")
    p.add_argument("--after", default="row_pass_kernel")
    p.add_argument("--skip", type=int, default=1)
    p.add_argument("--limit", type=int, default=60)
    p = sub.add_parser("longcalls")
    p.add_argument("db")
    p.add_argument("--top", type=int, default=20)
    p.add_argument("--min-ms", type=float, default=1.0)
    p = sub.add_parser("pmc")
    p.add_argument("db", nargs="+")
    p.add_argument("--kernel", default="")
    p = sub.add_parser("pmccsv")
    p.add_argument("dir")
    p.add_argument("sub", nargs="?", default="kmeans_assign")
    p = sub.add_parser("kcsv")
    p.add_argument("csv")
    p.add_argument("n", nargs="?", type=int, default=15)
    p = sub.add_parser("kres")
    p.add_argument("src")
    p.add_argument("filter", nargs="?", default="")
    a = ap.parse_args(argv)
    globals()["cmd_" + a.cmd](a)


if __name__ == "__main__":
    main()
