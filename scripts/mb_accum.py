"""Microbenchmark of the KMeans kernels (one process, cuda events)."""
import torch
from clustermachinelearningforhospitalnetworks_apache_spark_amd.ops import kmeans_ops as K
from clustermachinelearningforhospitalnetworks_apache_spark_amd.models.kmeans import LloydEngine


def timeit(fn, reps=3):
    fn(); torch.cuda.synchronize()
    best = 1e30
    for _ in range(reps):
        s, e = torch.cuda.Event(True), torch.cuda.Event(True)
        s.record(); fn(); e.record(); torch.cuda.synchronize()
        best = min(best, s.elapsed_time(e))
    return best


for (n, d, k) in [(20_000_000, 256, 256), (10_000_000, 128, 64), (20_000_000, 16, 5), (4_000_000, 512, 128),
                  (1_250_000, 128, 64), (100_000, 16, 5)]:
    g = torch.Generator(device="cuda"); g.manual_seed(0)
    cen = torch.randn(k, d, device="cuda", generator=g) * 4
    x = (cen[torch.randint(0, k, (n,), device="cuda", generator=g)] + torch.randn(n, d, device="cuda", generator=g)).to(torch.bfloat16)
    del cen
    gb = n * d * 2 / 1e9
    for mode in (None, "priv"):
        K.set_assign_variant(0)
        try:
            eng = LloydEngine(x, d, k, accum_mode=mode)
        except ValueError as e:
            print(f"n={n} d={d} k={k} mode={mode}: {e}")
            continue
        eng.set_centers(x[:k].double().cpu().numpy())
        if mode is None:
            for v in (0,):
                K.set_assign_variant(v)
                ap = K.plan_assign(n, eng.dp, k)
                t_as = timeit(lambda: K.assign_bf16(x, n, eng.dp, eng.cb, eng.cnorm, ap, eng.labels, eng.best,
                                                    eng.cost_part, xnorm=eng.xnorm))
                print(f"n={n} d={d} k={k} variant {v} grid {ap.grid}x{ap.nwaves}w: assign {t_as:.3f} ms "
                      f"({gb/t_as:.2f} TB/s, {2*n*d*k/t_as/1e9:.0f} TF/s)", flush=True)
            K.set_assign_variant(0)
        for g in (False, True):
            eng.use_graph = g
            t_st = timeit(lambda: eng.step(), reps=5)
            print(f"n={n} d={d} k={k} {eng.cplan} graph={g}: step {t_st:.3f} ms -> {n/t_st/1e6:.2f} Gsamples/s",
                  flush=True)
        del eng
        torch.cuda.empty_cache()
    del x
    torch.cuda.empty_cache()
