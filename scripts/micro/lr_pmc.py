"""Workload for one rocprofv3 --pmc pass over K13 (`logreg_grad_kernel`): 50M x 512 e4m3 rows (the config-5
shape), then 50M x 256 bf16 rows (config 4), three dispatches each.

    cd /tmp && rocprofv3 --pmc <counters> --kernel-trace --output-format csv -d /tmp/pm -o pm -- \
        python3 $REPO/scripts/micro/lr_pmc.py
    python3 scripts/prof.py pmccsv /tmp/pm logreg_grad
"""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", ".."))
import torch  # noqa: E402

from clustermachinelearningforhospitalnetworks_apache_spark_amd.ops import glm_ops  # noqa: E402
from clustermachinelearningforhospitalnetworks_apache_spark_amd.utils import synth  # noqa: E402

dev = torch.device("cuda", 0)
n = int(os.environ.get("LR_ROWS", "50000000"))
for d, dt in ((512, torch.float8_e4m3fn), (256, torch.bfloat16)):
    x = synth.synth_rows(0, n, d, seed=3, dtype=torch.bfloat16, device=dev)
    if dt != torch.bfloat16:  # synth_rows writes bf16 / f32; e4m3 rows are rounded from those
        x = x.to(dt)
    g = torch.Generator(device=dev)
    g.manual_seed(1)
    y = torch.randint(0, 2, (n,), generator=g, device=dev).double()
    coef = torch.randn(d + 1, generator=g, device=dev, dtype=torch.float64) * 0.05
    for _ in range(3):
        glm_ops.logreg_grad(x, d, y, coef, None)
    torch.cuda.synchronize()
    print("dtype", dt, "d", d, flush=True)
    del x, y
    torch.cuda.empty_cache()
