"""K13 logreg_grad ablation: rows in flight per wave (U = 1 / 2) x batch size, plus K7 moments."""
import json
import sys

import torch
from clustermachinelearningforhospitalnetworks_apache_spark_amd.ops import glm_ops


def timeit(fn, reps=20, graph=True):
    """Median ms per call; with graph=True the calls are captured into one HIP graph and replayed,
    so host launch overhead (Python + ctypes, tens of µs) does not hide the kernel time."""
    fn(); torch.cuda.synchronize()
    if graph:
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            for _ in range(reps):
                fn()
        g.replay(); torch.cuda.synchronize()
        ts = []
        for _ in range(5):
            s, e = torch.cuda.Event(True), torch.cuda.Event(True)
            s.record(); g.replay(); e.record(); torch.cuda.synchronize()
            ts.append(s.elapsed_time(e) / reps)
        return min(ts)
    ts = []
    for _ in range(reps):
        s, e = torch.cuda.Event(True), torch.cuda.Event(True)
        s.record(); fn(); e.record(); torch.cuda.synchronize()
        ts.append(s.elapsed_time(e))
    ts.sort()
    return ts[len(ts) // 2]


res = []
for d, dt in [(256, torch.bfloat16), (512, torch.float8_e4m3fn), (256, torch.float32)]:
    n = 50_000_000 if dt != torch.float32 else 25_000_000
    x = torch.randn(n, d, device="cuda").to(torch.bfloat16).to(dt)
    y = (torch.rand(n, device="cuda") > 0.5).double()
    coef = torch.randn(d + 1, device="cuda", dtype=torch.float64) * 0.05
    base = torch.zeros((), dtype=torch.int64, device="cuda")
    for u in (1,):
        glm_ops.set_logreg_unroll(u)
        for b in (16384, 131072, 1048576, n):
            t = timeit(lambda: glm_ops.logreg_grad(x, d, y, coef, None, batch=b, row_base=base), reps=20 if b < n else 3)
            gb = b * d * x.element_size() / 1e9
            r = {"dtype": str(dt), "d": d, "U": u, "rows": b, "ms": round(t, 4), "TB/s": round(gb / t, 2)}
            res.append(r)
            print(json.dumps(r), flush=True)
    glm_ops.set_logreg_unroll(0)
    part = torch.randn(1024, d + 3, dtype=torch.float64, device="cuda")
    t = timeit(lambda: glm_ops.partial_colsum(part))
    print(json.dumps({"op": "partial_colsum", "shape": [1024, d + 3], "us": round(t * 1e3, 2)}), flush=True)
    t = timeit(lambda: glm_ops.moments(x, d), reps=5, graph=False)
    r = {"dtype": str(dt), "d": d, "op": "moments", "rows": n, "ms": round(t, 3),
         "TB/s": round(n * d * x.element_size() / 1e9 / t, 2)}
    res.append(r)
    print(json.dumps(r), flush=True)
    del x, y
    torch.cuda.empty_cache()
if len(sys.argv) > 1:
    json.dump(res, open(sys.argv[1], "w"), indent=1)
