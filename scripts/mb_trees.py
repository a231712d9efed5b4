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
    for rep in ("cold", "warm"):  # the first fit of a process also loads every kernel it launches
        times.clear()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        trees = eng.fit()
        torch.cuda.synchronize()
        t = time.perf_counter() - t0
        nodes = sum(TR.num_nodes(r) for r in trees)
        print(f"RF{task[:5]} n={n} d={d} ({rep}): fit {t:.3f} s ({nodes} nodes) " +
              " ".join(f"{k}={v:.3f}s" for k, v in times.items()), flush=True)
    del x, y, eng
    torch.cuda.empty_cache()

# gradient boosting: 20 boosting iterations of depth-5 regression trees (GBTRegressor defaults) / logistic loss
for n, d, loss in [(10_000_000, 4, "squared"), (10_000_000, 4, "logistic"), (2_000_000, 64, "squared")]:
    g = torch.Generator(device="cuda")
    g.manual_seed(0)
    x = torch.randn(n, d, device="cuda", dtype=torch.float64, generator=g)
    y = torch.sin(2 * x[:, 0]) + (x[:, 1 % d] > 0).double() + 0.1 * torch.randn(n, device="cuda",
                                                                                 dtype=torch.float64, generator=g)
    if loss == "logistic":
        y = torch.where(y > 0.5, 1.0, -1.0).double()
    p = TR.TreeParams(max_depth=5, seed=1)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    trees, tw = TR.fit_gbt(x, y, p, 20, 0.1, loss)
    torch.cuda.synchronize()
    t = time.perf_counter() - t0
    f = TR.predict_forest(trees, x, "variance", 1, False, False, tw)[:, 0]
    err = float(TR.gbt_loss(loss, f, y).mean())
    print(f"GBT-{loss} n={n} d={d}: fit {t:.3f} s for {len(trees)} trees ({t / len(trees) * 1e3:.1f} ms/tree), "
          f"train loss {err:.4f}", flush=True)
    del x, y
    torch.cuda.empty_cache()
