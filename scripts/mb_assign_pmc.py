"""Dispatches for a PMC pass: the assign over N x D (k centres) three times with the HBM stream, then
three times with every row aliasing row 0 (compute only). Identify them in the counter CSV by order.

usage: python scripts/mb_assign_pmc.py [variant] [n] [d] [k] [rr-debug-bits]   (variant: 0 = K9, 8 = K9r)"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import bench  # noqa: E402
from clustermachinelearningforhospitalnetworks_apache_spark_amd.models.kmeans import LloydEngine  # noqa: E402
from clustermachinelearningforhospitalnetworks_apache_spark_amd.ops import kmeans_ops as K  # noqa: E402

v = int(sys.argv[1]) if len(sys.argv) > 1 else 0
n = int(sys.argv[2]) if len(sys.argv) > 2 else 20_000_000
d = int(sys.argv[3]) if len(sys.argv) > 3 else 256
k = int(sys.argv[4]) if len(sys.argv) > 4 else 256
dbg = int(sys.argv[5]) if len(sys.argv) > 5 else 0
K.set_assign_variant(v)
if dbg:
    from clustermachinelearningforhospitalnetworks_apache_spark_amd import _native  # noqa: E402
    _native.kernels().cml_kmeans_set_rr_debug(dbg)
x = bench.make_blobs(n, d, k, seed=1000, device=torch.device("cuda"))
eng = LloydEngine(x, d, k, use_graph=False)
eng.set_centers(x[:k].double().cpu().numpy())
torch.cuda.synchronize()
x0 = torch.as_strided(eng.x, (n, eng.dp), (0, 1))
for xx in (eng.x, x0):
    for _ in range(3):
        K.assign_bf16(xx, n, eng.dp, eng.cb, eng.cnorm, eng.aplan, eng.labels, None, eng.cost_part, eng.hist,
                      eng.rank, xnorm=eng.xnorm)
    torch.cuda.synchronize()
print("done", flush=True)
