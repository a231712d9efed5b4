"""K9r full pass (20M x 256 bf16, k = 256) with its rows from HBM, from L2 (stride-0 X: every row the same row),
MFMA only and without the LDS-DMA (kmeans_rr.h dbg ablations), 6 launches each — run under rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES
(scripts/gpu.sh clock) to compare the clock and the MFMA busy share of the two.

    python scripts/mb_k9r_clock.py            (under the profiler)
    python scripts/mb_k9r_clock.py show DIR   (per-dispatch table from the profiler's counter CSV)
"""
import csv
import glob
import os
import sys

if len(sys.argv) > 2 and sys.argv[1] == "show":
    rows = {}
    for f in sorted(glob.glob(os.path.join(sys.argv[2], "**", "*counter_collection.csv"), recursive=True)):
        for r in csv.DictReader(open(f)):
            if "kmeans_assign_rr" not in r["Kernel_Name"]:
                continue
            d = rows.setdefault(int(r["Dispatch_Id"]), {})
            d["ns"] = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
            d[r["Counter_Name"]] = d.get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
    ids = sorted(rows)
    names = ["rows from HBM", "rows from L2 ", "MFMA only    ", "no DMA       "]
    for i, did in enumerate(ids):
        d = rows[did]
        ns = d["ns"]
        clk = d.get("GRBM_GUI_ACTIVE", 0.0) / 8 / ns  # GHz: the counter sums the 8 XCDs
        mf = d.get("SQ_VALU_MFMA_BUSY_CYCLES", 0.0) / 1024 / (clk * ns) if clk else 0.0
        src = names[min(i // 6, len(names) - 1)]
        print(f"dispatch {did:5d} {src}: {ns / 1e6:.3f} ms, clock {clk:.2f} GHz, MFMA busy {mf:.1%}, "
              f"SQ_BUSY_CYCLES {d.get('SQ_BUSY_CYCLES', 0):.3g}")
    sys.exit(0)

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import bench  # noqa: E402
from clustermachinelearningforhospitalnetworks_apache_spark_amd.models.kmeans import LloydEngine  # noqa: E402
from clustermachinelearningforhospitalnetworks_apache_spark_amd.ops import kmeans_ops as K  # noqa: E402

n, D, KC = 20_000_000, 256, 256
x = bench.make_blobs(n, D, KC, seed=1000, device=torch.device("cuda"))
eng = LloydEngine(x, D, KC, use_graph=False)
eng.set_centers(x[:KC].to(torch.float32).double().cpu().numpy())
x0 = torch.as_strided(eng.x, (n, eng.dp), (0, 1))
from clustermachinelearningforhospitalnetworks_apache_spark_amd import _native  # noqa: E402
lib = _native.kernels()
# rows from HBM, rows from L2, then the ablations (kmeans_rr.h dbg bits): MFMA only (5), no DMA (1)
for xx, dbg in ((eng.x, 0), (x0, 0), (eng.x, 5), (eng.x, 1)):
    lib.cml_kmeans_set_rr_debug(dbg)
    for _ in range(6):
        K.assign_bf16(xx, n, eng.dp, eng.cb, eng.cnorm, eng.aplan, eng.labels, None, eng.cost_part, eng.hist,
                      eng.rank, xnorm=eng.xnorm)
    torch.cuda.synchronize()
lib.cml_kmeans_set_rr_debug(0)
print("done", flush=True)
