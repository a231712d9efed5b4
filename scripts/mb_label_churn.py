"""Fraction of rows whose KMeans label changes per Lloyd iteration on the bench data (100M x 256, k=256)."""
import sys
import torch
sys.argv += [] 
import bench
from clustermachinelearningforhospitalnetworks_apache_spark_amd.models.kmeans import LloydEngine

n = int(sys.argv[1]) if len(sys.argv) > 1 else 20_000_000
x = bench.make_blobs(n, 256, 256, seed=1000, device=torch.device("cuda"))
eng = LloydEngine(x, 256, 256, use_graph=False)
eng.set_centers(eng.init_kmeans_parallel(seed=42))
prev = None
for it in range(25):
    eng.step()
    lab = eng.labels[:n].clone()
    if prev is not None:
        ch = int((lab != prev).sum().item())
        print(f"iter {it}: changed {ch} ({100.0 * ch / n:.3f}%)", flush=True)
    prev = lab
