"""K8 (scale_apply) rates at the config-4/5 shapes: 50M x 512 bf16 -> e4m3 (the pipeline's StandardScaler
transform) and 50M x 256 bf16 -> bf16; one pass each, best of 5, read + write bytes.

    PYTHONPATH=$PWD python3 scripts/micro/scale_ab.py
"""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import torch  # noqa: E402

from mb_ml import best_ms, rows_x  # noqa: E402
from clustermachinelearningforhospitalnetworks_apache_spark_amd.ops import glm_ops  # noqa: E402

for n, d, out in ((50_000_000, 512, torch.float8_e4m3fn), (50_000_000, 256, torch.bfloat16)):
    x = rows_x(n, d, torch.bfloat16)
    mean = torch.zeros(d, dtype=torch.float64, device="cuda")
    inv = torch.ones(d, dtype=torch.float64, device="cuda")
    gb = n * d * (2 + torch.tensor([], dtype=out).element_size()) / 1e9
    for _ in range(2):
        t = best_ms(lambda: glm_ops.scale_apply(x, d, mean, inv, True, out))
        print(f"bf16 -> {out} n={n} d={d}: {t:.3f} ms {gb / t:.2f} TB/s (r+w)", flush=True)
    del x
    torch.cuda.empty_cache()
