"""fp8 x 512 GLM kernels by streaming layout (chunks per lane: 1 = auto/round 3, 2, 4): K13 logreg_grad,
K7 moments, K24 linear_predict — bytes in flight per wave vs VGPRs."""
import torch

from clustermachinelearningforhospitalnetworks_apache_spark_amd.ops import glm_ops


def timeit(fn, reps=5):
    fn()
    torch.cuda.synchronize()
    best = 1e30
    for _ in range(reps):
        s, e = torch.cuda.Event(True), torch.cuda.Event(True)
        s.record()
        fn()
        e.record()
        torch.cuda.synchronize()
        best = min(best, s.elapsed_time(e))
    return best


n, d = 50_000_000, 512
x = torch.randn(n, d, device="cuda").to(torch.bfloat16).to(torch.float8_e4m3fn)
y = (torch.rand(n, device="cuda") > 0.5).double()
coef = torch.randn(d + 1, device="cuda", dtype=torch.float64) * 0.05
gb = x.numel() / 1e9
ref = None
for nch in (0, 2, 4):
    glm_ops.set_fp8_nch(nch)
    g = glm_ops.logreg_grad(x, d, y, coef, None)
    if ref is None:
        ref = g.clone()
    err = float((g - ref).abs().max() / ref.abs().max())
    t = timeit(lambda: glm_ops.logreg_grad(x, d, y, coef, None))
    tm = timeit(lambda: glm_ops.moments(x, d))
    tp = timeit(lambda: glm_ops.linear_predict(x, d, coef, "logistic"))
    print(f"fp8 nch={nch or 'auto'}: logreg_grad {t:.3f} ms {gb / t:.2f} TB/s (rel diff {err:.1e}); "
          f"moments {gb / tm:.2f} TB/s; linear_predict {gb / tp:.2f} TB/s", flush=True)
glm_ops.set_fp8_nch(0)
