"""K9r ablation: time the assign with parts of the pipeline switched off (kmeans_rr.h `dbg` bits:
1 no LDS-DMA, 2 no MFMA/keys, 4 no finalize). usage: python scripts/mb_assign_rr_dbg.py N D K [fp8]
(fp8: e4m3 rows, the MX pass unless CML_KMEANS_FP8_MX=0)"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import bench  # noqa: E402
from clustermachinelearningforhospitalnetworks_apache_spark_amd import _native  # noqa: E402
from clustermachinelearningforhospitalnetworks_apache_spark_amd.models.kmeans import LloydEngine  # noqa: E402
from clustermachinelearningforhospitalnetworks_apache_spark_amd.ops import kmeans_ops as K  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 20_000_000
D = int(sys.argv[2]) if len(sys.argv) > 2 else 256
KC = int(sys.argv[3]) if len(sys.argv) > 3 else 256
FP8 = len(sys.argv) > 4 and sys.argv[4] == "fp8"
K.set_assign_variant(8)
x = bench.make_blobs(n, D, KC, seed=1000, device=torch.device("cuda"))
if FP8:
    x = (x.float() / 3.2).clamp(-440, 440).to(torch.float8_e4m3fn)
eng = LloydEngine(x, D, KC, use_graph=False)
eng.set_centers(x[:KC].to(torch.float32).double().cpu().numpy())
x0 = torch.as_strided(eng.x, (n, eng.dp), (0, 1))
lib = _native.kernels()
print(f"n={n} d={D} k={KC} rr_ct={eng.aplan.rr_ct} grid={eng.aplan.grid} fp8={FP8} mx={eng._mx}", flush=True)
ROWB = eng.dp * (1 if FP8 else 2)


def timed(xx, reps=5):
    ts = []
    for _ in range(reps):
        a, b = torch.cuda.Event(True), torch.cuda.Event(True)
        a.record()
        K.assign_bf16(xx, n, eng.dp, eng.cb, eng.cnorm, eng.aplan, eng.labels, None, eng.cost_part, eng.hist,
                      eng.rank, xnorm=eng.xnorm)
        b.record()
        torch.cuda.synchronize()
        ts.append(a.elapsed_time(b))
    return sorted(ts)[len(ts) // 2]


res = {}
for rnd in range(3):
    for dbg in (0, 1, 2, 4, 3, 6, 5):
        lib.cml_kmeans_set_rr_debug(dbg)
        res.setdefault((dbg, "full"), []).append(timed(eng.x))
        res.setdefault((dbg, "compute"), []).append(timed(x0))
lib.cml_kmeans_set_rr_debug(0)
names = {0: "all on", 1: "no DMA", 2: "no MFMA", 4: "no finalize", 3: "finalize only", 6: "DMA only",
         5: "MFMA only"}
for dbg in (0, 1, 2, 4, 3, 6, 5):
    f = sorted(res[(dbg, "full")])[1]
    c = sorted(res[(dbg, "compute")])[1]
    print(f"dbg {dbg} {names[dbg]:14s}: full {f:.3f} ms ({n * ROWB / f / 1e9:.2f} TB/s)  compute-only {c:.3f} ms",
          flush=True)
