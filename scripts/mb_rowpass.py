"""K12 row pass on 100M x 256 bf16 rows (norms + first k-means|| costs + max norm + exponent range):
best of 10 timed launches. CML_ROWPASS_PACKED=1 selects the packed-FMA variant (read once per process)."""
import os
import torch
from clustermachinelearningforhospitalnetworks_apache_spark_amd.ops import kmeans_ops as K

n, dp = 100_000_000, 256
x = torch.empty((n, dp), dtype=torch.bfloat16, device="cuda")
for s in range(0, n, 1 << 24):
    x[s:s + (1 << 24)] = torch.randn((min(1 << 24, n - s), dp), device="cuda").to(torch.bfloat16)
xn = torch.empty(n, device="cuda")
cost = torch.empty(n, device="cuda")
near = torch.empty(n, dtype=torch.int32, device="cuda")
c0 = x[7].float().contiguous()
c0n = float((c0.double() ** 2).sum())
mx = torch.zeros(1, device="cuda")
best = 1e30
for _ in range(10):
    er = torch.tensor([2 ** 31 - 1, -1], dtype=torch.int32, device="cuda")
    a, b = torch.cuda.Event(True), torch.cuda.Event(True)
    a.record()
    K.row_pass(x, n, dp, xn, c0, c0n, cost, near, xn_max=mx, erange=er)
    b.record()
    torch.cuda.synchronize()
    best = min(best, a.elapsed_time(b))
print(f"packed={os.environ.get('CML_ROWPASS_PACKED', '0')} row_pass {best:.3f} ms {n * dp * 2 / best / 1e9:.2f} TB/s "
      f"erange={er.tolist()}", flush=True)
