"""K24 (linear_predict, logistic link) rates: 50M x 256 bf16, 50M x 512 e4m3, 25M x 256 f32 rows; one pass
each, best of 5, at each prefetch depth the library offers (the ring variant measured in
profiles/r6/k13_ring/predict_ring_ab.log had a `set_predict_unroll` knob; it was not kept, so today this
measures the one K24 form).

    PYTHONPATH=$PWD python3 scripts/micro/predict_ab.py
"""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import torch  # noqa: E402

from mb_ml import best_ms, glm_inputs, rows_x  # noqa: E402
from clustermachinelearningforhospitalnetworks_apache_spark_amd.ops import glm_ops  # noqa: E402

try:
    glm_ops.set_predict_unroll(0)
    depths = (1, 2, 1, 2)
except (AttributeError, KeyError):
    depths = (None, None)
for d, dt, n in ((256, torch.bfloat16, 50_000_000), (512, torch.float8_e4m3fn, 50_000_000),
                 (256, torch.float32, 25_000_000)):
    x = rows_x(n, d, dt)
    _, coef = glm_inputs(1, d)
    gb = x.numel() * x.element_size() / 1e9
    ref = None
    for u in depths:
        if u is not None:
            glm_ops.set_predict_unroll(u)
        p = glm_ops.linear_predict(x, d, coef, "logistic")
        ref = p.clone() if ref is None else ref
        t = best_ms(lambda: glm_ops.linear_predict(x, d, coef, "logistic"))
        print(f"{dt} d={d} n={n} U={u}: {t:.3f} ms {gb / t:.2f} TB/s same_bits={bool(torch.equal(p, ref))}",
              flush=True)
    if depths[0] is not None:
        glm_ops.set_predict_unroll(0)
    del x
    torch.cuda.empty_cache()
