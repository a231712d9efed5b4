"""Workload for one rocprofv3 --pmc pass over the K13m MFMA forms (100M x 256 bf16 rows, C = 8): the 16-class
tile (mode 0) and the 32-class tile (mode 3), three dispatches each, in that order.

    cd /tmp && rocprofv3 --pmc <counters> --kernel-trace --output-format csv -d /tmp/pm -o pm -- \
        python3 $REPO/scripts/micro/mn_pmc.py
    python3 scripts/prof.py pmccsv --dir /tmp/pm --sub multinomial
"""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", ".."))
import torch  # noqa: E402

from clustermachinelearningforhospitalnetworks_apache_spark_amd import _native  # noqa: E402
from clustermachinelearningforhospitalnetworks_apache_spark_amd.ops import glm_ops  # noqa: E402
from clustermachinelearningforhospitalnetworks_apache_spark_amd.utils import synth  # noqa: E402

dev = torch.device("cuda", 0)
n, d, C = int(os.environ.get("MN_ROWS", "100000000")), 256, 8
x = synth.synth_rows(0, n, d, seed=3, dtype=torch.bfloat16, device=dev)
g = torch.Generator(device=dev)
g.manual_seed(1)
y = torch.randint(0, C, (n,), generator=g, device=dev).double()
coef = torch.randn(C, d + 1, generator=g, device=dev, dtype=torch.float64) * 0.05
lib = _native.kernels()
for mode in (0, 3):
    prev = glm_ops.set_multinomial_mfma_mode(mode)
    cp, dp = lib.cml_multinomial_mfma_supported(d, 0, C), lib.cml_multinomial_mfma_dpad(d, C)
    for _ in range(3):
        glm_ops._multinomial_mfma(x, d, y, coef, None, C, cp, dp)
    torch.cuda.synchronize()
    glm_ops.set_multinomial_mfma_mode(prev)
    print("mode", mode, "cp", cp, flush=True)
