"""K9r under PMC counters: mode 0 (or argv[4]) at n x d, k centres, 3 launches. Run under
rocprofv3 --pmc ... -- python3 scripts/mb_k9r_pmc.py n d k mode."""
import sys

import torch

from clustermachinelearningforhospitalnetworks_apache_spark_amd.models.kmeans import LloydEngine, to_device_matrix
from clustermachinelearningforhospitalnetworks_apache_spark_amd.ops import kmeans_ops as K

n = int(sys.argv[1]) if len(sys.argv) > 1 else 20_000_000
d = int(sys.argv[2]) if len(sys.argv) > 2 else 256
k = int(sys.argv[3]) if len(sys.argv) > 3 else 256
mode = int(sys.argv[4]) if len(sys.argv) > 4 else 0
g = torch.Generator(device="cuda").manual_seed(0)
cen = torch.randn(k, d, device="cuda", generator=g) * 4
x = torch.empty((n, d), dtype=torch.bfloat16, device="cuda")
for s in range(0, n, 1 << 22):
    m = min(1 << 22, n - s)
    x[s:s + m] = (cen[torch.randint(0, k, (m,), device="cuda", generator=g)] +
                  torch.randn(m, d, device="cuda", generator=g)).to(torch.bfloat16)
x = to_device_matrix(x, d)
dp = x.shape[1]
kp = -(-k // 32) * 32
cb = torch.zeros((kp, dp), dtype=torch.bfloat16, device="cuda")
cn = torch.zeros(kp, device="cuda")
K.update_centers(None, k, d, cen.double().clone(), cb, dp, kp, cn, None)
xn = torch.empty(n, device="cuda")
K.row_pass(x, n, dp, xn)
plan = K.plan_assign(n, dp, k)
lab = torch.zeros(n, dtype=torch.int32, device="cuda")
cp = torch.zeros(plan.grid, dtype=torch.float64, device="cuda")
best = torch.empty(n, device="cuda")
ub = torch.zeros(n, device="cuda")
lb = torch.zeros(n, device="cuda")
mc = torch.tensor([float(cn[:k].max())], device="cuda")
tau = LloydEngine.prune_tau(dp)
for _ in range(3):
    if mode == 0:
        K.assign_bf16(x, n, dp, cb, cn, plan, lab, best, cp, xnorm=xn)
    else:
        K.assign_rr_ext(1, x, n, dp, cb, cn, plan, xn, lab, cp, ub, lb, mc, tau)
torch.cuda.synchronize()
print("plan", plan, flush=True)
