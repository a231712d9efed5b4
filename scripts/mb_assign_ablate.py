"""K9 ablation: full vs compute-only (ldx=0: every row is row 0, L1/L2 hits) vs memory-heavy (k=32)."""
import sys
import torch
from clustermachinelearningforhospitalnetworks_apache_spark_amd import _native
from clustermachinelearningforhospitalnetworks_apache_spark_amd.ops import kmeans_ops as K
from clustermachinelearningforhospitalnetworks_apache_spark_amd.models.kmeans import to_device_matrix


def timeit(fn, reps=5):
    fn(); torch.cuda.synchronize()
    best = 1e30
    for _ in range(reps):
        s, e = torch.cuda.Event(True), torch.cuda.Event(True)
        s.record(); fn(); e.record(); torch.cuda.synchronize()
        best = min(best, s.elapsed_time(e))
    return best


lib = _native.kernels()
shapes = [(20_000_000, 256, 256), (20_000_000, 16, 5), (10_000_000, 128, 64)]
variants = [int(v) for v in sys.argv[1:]] or [0, 1, 2, 3, 4, 5]
for (n, d, k) in shapes:
    x = torch.randn(n, d, device="cuda", dtype=torch.bfloat16)
    dp = x.shape[1]
    xn = K.row_sqnorm(x, n, dp)
    for kk in sorted({k, 32}, reverse=True):
        kp = (kk + 31) // 32 * 32
        cb = torch.randn(kp, dp, device="cuda").to(torch.bfloat16)
        cn = (cb.float() ** 2).sum(1)
        lab = torch.empty(n, dtype=torch.int32, device="cuda")
        for v in variants:
            K.set_assign_variant(v)
            ap = K.plan_assign(n, dp, kk)
            cost = torch.zeros(ap.grid, dtype=torch.float64, device="cuda")
            for ldx, tag in ((x.stride(0), "full"), (0, "ldx0")):
                if tag == "ldx0" and kk != k:
                    continue
                def run():
                    st = lib.cml_kmeans_assign_bf16(x.data_ptr(), n, ldx, dp, cb.data_ptr(), dp, ap.kc, ap.kp, 0,
                                                    cn.data_ptr(), xn.data_ptr(), lab.data_ptr(), 0, 1, 1,
                                                    cost.data_ptr(), 0, 0, ap.grid, 0, 0)
                    _native.check(st, "assign")
                t = timeit(run)
                print(f"n={n} d={d} k={kk} v{v} grid={ap.grid}x{ap.nwaves}w {tag:5s}: {t:.3f} ms "
                      f"{n*dp*2/t/1e9:.2f} TB/s {2*n*dp*kp/t/1e9:.0f} TF/s", flush=True)
    del x, xn
    torch.cuda.empty_cache()
