"""K7 (column moments) prefetch depth A/B: 50M x 256 bf16, 50M x 512 e4m3, 25M x 256 f32 rows; one pass each,
best of 5, at 1 and 2 row groups in flight per wave (the same accumulation order, so the same bits).

    PYTHONPATH=$PWD python3 scripts/micro/moments_ring.py
"""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import torch  # noqa: E402

from mb_ml import best_ms, rows_x  # noqa: E402
from clustermachinelearningforhospitalnetworks_apache_spark_amd.ops import glm_ops  # noqa: E402

for d, dt, n in ((256, torch.bfloat16, 50_000_000), (512, torch.float8_e4m3fn, 50_000_000),
                 (256, torch.float32, 25_000_000)):
    x = rows_x(n, d, dt)
    gb = x.numel() * x.element_size() / 1e9
    ref = None
    for u in (1, 2, 1, 2):
        glm_ops.set_moments_unroll(u)
        m = glm_ops.moments(x, d)
        got = torch.cat([m[1], m[2]])
        ref = got.clone() if ref is None else ref
        same = bool(torch.equal(got, ref))
        t = best_ms(lambda: glm_ops.moments(x, d))
        print(f"{dt} d={d} n={n} U={u}: {t:.3f} ms {gb / t:.2f} TB/s same_bits={same}", flush=True)
    glm_ops.set_moments_unroll(0)
    del x
    torch.cuda.empty_cache()
