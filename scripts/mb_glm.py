"""Microbenchmark of the GLM kernels (K7 moments, K8 scale_apply, K13 logreg_grad, K24 linear_predict)."""
import torch
from clustermachinelearningforhospitalnetworks_apache_spark_amd.ops import glm_ops


def timeit(fn, reps=5):
    fn(); torch.cuda.synchronize()
    best = 1e30
    for _ in range(reps):
        s, e = torch.cuda.Event(True), torch.cuda.Event(True)
        s.record(); fn(); e.record(); torch.cuda.synchronize()
        best = min(best, s.elapsed_time(e))
    return best


for n, d, dt in [(20_000_000, 512, torch.float8_e4m3fn), (20_000_000, 256, torch.bfloat16), (10_000_000, 256, torch.float32), (20_000_000, 4, torch.float64),
                 (20_000_000, 512, torch.bfloat16)]:
    x = torch.randn(n, d, device="cuda").to(dt) if dt != torch.float8_e4m3fn else torch.randn(n, d, device="cuda").to(torch.bfloat16).to(dt)
    y = (torch.rand(n, device="cuda") > 0.5).double()
    coef = torch.randn(d + 1, device="cuda", dtype=torch.float64) * 0.05
    gb = x.numel() * x.element_size() / 1e9
    t = timeit(lambda: glm_ops.moments(x, d))
    print(f"n={n} d={d} {dt}: moments {t:.3f} ms {gb/t:.2f} TB/s", flush=True)
    mean = torch.zeros(d, dtype=torch.float64, device="cuda"); inv = torch.ones(d, dtype=torch.float64, device="cuda")
    t = timeit(lambda: glm_ops.scale_apply(x, d, mean, inv, True, dt))
    print(f"n={n} d={d} {dt}: scale_apply {t:.3f} ms {2*gb/t:.2f} TB/s (r+w)", flush=True)
    t = timeit(lambda: glm_ops.logreg_grad(x, d, y, coef, None))
    print(f"n={n} d={d} {dt}: logreg_grad {t:.3f} ms {gb/t:.2f} TB/s", flush=True)
    t = timeit(lambda: glm_ops.linear_predict(x, d, coef, "logistic"))
    print(f"n={n} d={d} {dt}: linear_predict {t:.3f} ms {gb/t:.2f} TB/s", flush=True)
    if d <= 30:
        t = timeit(lambda: glm_ops.gram(x, d, y, None))
        print(f"n={n} d={d} {dt}: gram {t:.3f} ms {gb/t:.2f} TB/s", flush=True)
    del x, y
    torch.cuda.empty_cache()
