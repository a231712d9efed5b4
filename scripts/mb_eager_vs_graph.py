"""Per-step time of the Lloyd step at an 8-GPU shard size (12.5M x 256, k = 256) eager vs HIP graph,
with the multi-rank chunking (2 row chunks): how much of a rank's step is host launch cost."""
import time
import torch
import bench
from clustermachinelearningforhospitalnetworks_apache_spark_amd.models.kmeans import LloydEngine

n = 12_500_000
x = bench.make_blobs(n, 256, 256, seed=1000, device=torch.device("cuda"))
for chunks in (1, 2):
    for graph in (False, True):
        eng = LloydEngine(x, 256, 256, row_chunks=chunks, use_graph=graph)
        eng.set_centers(eng.init_kmeans_parallel(seed=42))
        for _ in range(4):
            eng.step()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(20):
            eng.step()
        t_host = (time.perf_counter() - t0) / 20
        torch.cuda.synchronize()
        t_all = (time.perf_counter() - t0) / 20
        print(f"chunks={chunks} graph={graph}: {1e3 * t_all:.3f} ms/step (host enqueue {1e3 * t_host:.3f} ms/step)",
              flush=True)
        del eng
        torch.cuda.empty_cache()
