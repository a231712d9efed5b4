"""Dispatches for a PMC pass: K9 assign over 20M x 256 (k = 256) three times with the HBM stream, then three
times with every row aliasing row 0 (compute only). Identify them in the counter CSV by order."""
import torch
import bench
from clustermachinelearningforhospitalnetworks_apache_spark_amd.models.kmeans import LloydEngine
from clustermachinelearningforhospitalnetworks_apache_spark_amd.ops import kmeans_ops as K

n = 20_000_000
x = bench.make_blobs(n, 256, 256, seed=1000, device=torch.device("cuda"))
eng = LloydEngine(x, 256, 256, use_graph=False)
eng.set_centers(x[:256].double().cpu().numpy())
torch.cuda.synchronize()
x0 = torch.as_strided(eng.x, (n, eng.dp), (0, 1))
for xx in (eng.x, x0):
    for _ in range(3):
        K.assign_bf16(xx, n, eng.dp, eng.cb, eng.cnorm, eng.aplan, eng.labels, None, eng.cost_part, eng.hist,
                      eng.rank, xnorm=eng.xnorm)
    torch.cuda.synchronize()
print("done", flush=True)
