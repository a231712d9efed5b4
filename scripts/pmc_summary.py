"""Summarise rocprofv3 --pmc CSVs of the assign dispatches (scripts/gpu_pmc_assign.sh).

usage: python scripts/pmc_summary.py gpurun_out/pmc_TAG [name-substring]
Per dispatch: duration, counters, and derived clock (GRBM_GUI_ACTIVE / 8 XCDs / time), MFMA busy share
(SQ_VALU_MFMA_BUSY_CYCLES / 1024 SIMDs / kernel cycles), wave-cycle split, HBM rate (FETCH_SIZE is half the
streamed bytes on gfx950, MI355X_MICROARCH.md §HBM)."""
import csv
import glob
import os
import sys
from collections import defaultdict

root = sys.argv[1]
sub = sys.argv[2] if len(sys.argv) > 2 else "kmeans_assign"
disp = defaultdict(dict)
for f in sorted(glob.glob(os.path.join(root, "*", "*counter_collection.csv"))):
    tag = os.path.basename(os.path.dirname(f))
    for r in csv.DictReader(open(f)):
        if sub not in r["Kernel_Name"]:
            continue
        key = (tag, int(r["Dispatch_Id"]))
        d = disp[key]
        d["ms"] = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6
        d["vgpr"] = r["VGPR_Count"]
        d[r["Counter_Name"]] = d.get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
by_tag = defaultdict(list)
for (tag, did), d in sorted(disp.items()):
    by_tag[tag].append((did, d))
for tag, rows in by_tag.items():
    print(f"== {tag}")
    for i, (did, d) in enumerate(rows):
        kind = "full" if i < 3 else "compute-only"
        out = [f"dispatch {did} {kind:12s} {d['ms']:.3f} ms vgpr {d['vgpr']}"]
        if "GRBM_GUI_ACTIVE" in d:
            cyc = d["GRBM_GUI_ACTIVE"] / 8
            out.append(f"clock {cyc / d['ms'] / 1e6:.2f} GHz")
            if "SQ_VALU_MFMA_BUSY_CYCLES" in d:
                out.append(f"MFMA busy {d['SQ_VALU_MFMA_BUSY_CYCLES'] / 1024 / cyc * 100:.0f}%")
        if "SQ_WAIT_ANY" in d:
            tot = d["SQ_WAIT_ANY"] + d["SQ_WAIT_INST_ANY"] + d["SQ_ACTIVE_INST_ANY"]
            out.append("waves: wait {:.0f}% issue-stall {:.0f}% active {:.0f}%".format(
                *(100 * d[k] / tot for k in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY"))))
            out.append(f"LDS conflict {d['SQ_LDS_BANK_CONFLICT']:.3g} VALU {d.get('SQ_INSTS_VALU', 0):.3g} "
                       f"LDS {d.get('SQ_INSTS_LDS', 0):.3g} coexec {d['SQ_VALU_MFMA_COEXEC_CYCLES']:.3g}")
        if "FETCH_SIZE" in d:
            out.append(f"HBM {2 * d['FETCH_SIZE'] * 1024 / d['ms'] / 1e9:.2f} TB/s (2 x FETCH_SIZE)")
        print(" | ".join(out))
