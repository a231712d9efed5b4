"""Random-forest fit time on the GPU (ForestEngine, 20 trees, depth 5, 32 bins): reference-shaped data
(4 features) at scale and a wide table; prints per-fit seconds and the phase split."""
import time
import torch
from clustermachinelearningforhospitalnetworks_apache_spark_amd.models import trees as TR

for n, d, task in [(10_000_000, 4, "regression"), (10_000_000, 4, "classification"), (2_000_000, 64, "regression")]:
    g = torch.Generator(device="cuda")
    g.manual_seed(0)
    x = torch.randn(n, d, device="cuda", dtype=torch.float64, generator=g)
    if task == "regression":
        y = 2 * x[:, 0] + (x[:, 1 % d] > 0).double() + 0.1 * torch.randn(n, device="cuda", dtype=torch.float64,
                                                                           generator=g)
        imp = "variance"
    else:
        y = ((x[:, 0] + 0.5 * x[:, 2 % d]) > 0).double()
        imp = "gini"
    p = TR.TreeParams(task=task, num_classes=2, impurity=imp, num_trees=20, seed=1, feature_subset="auto")
    times = {}
    eng = TR.ForestEngine(x, y, p)
    for name in ("find_splits", "binize", "histogram", "best_splits", "route"):
        fn = getattr(eng, name)

        def wrap(*a, _fn=fn, _name=name, **k):
            torch.cuda.synchronize()
            t = time.perf_counter()
            r = _fn(*a, **k)
            torch.cuda.synchronize()
            times[_name] = times.get(_name, 0.0) + time.perf_counter() - t
            return r
        setattr(eng, name, wrap)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    trees = eng.fit()
    torch.cuda.synchronize()
    t = time.perf_counter() - t0
    nodes = sum(TR.num_nodes(r) for r in trees)
    print(f"RF{task[:5]} n={n} d={d}: fit {t:.3f} s ({nodes} nodes) " +
          " ".join(f"{k}={v:.3f}s" for k, v in times.items()), flush=True)
    del x, y, eng
    torch.cuda.empty_cache()
