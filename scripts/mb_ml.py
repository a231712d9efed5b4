"""Estimator-kernel microbenchmarks (GLM family and trees): one driver, one subcommand per experiment.

    python scripts/mb_ml.py glm [--scale S]
        K7 moments, K8 scale_apply, K13 logreg_grad, K24 linear_predict (and K15 gram for narrow rows) on five
        shapes from 20M x 512 fp8 to 20M x 4 f64; best-of-5 ms and TB/s
    python scripts/mb_ml.py glm-fp8 [--rows 50000000]
        fp8 x 512 GLM kernels by streaming layout (chunks per lane: auto, 2, 4) with the gradient's relative diff
    python scripts/mb_ml.py logreg [--scale S] [--out FILE.json]
        K13 logreg_grad by batch size (16K rows .. the whole shard; small batches replayed from one HIP graph so
        launch cost does not hide the kernel), partial_colsum, and K7 moments
    python scripts/mb_ml.py multinomial [--rows 100000000] [--dim 256]
        K13m multinomial loss + gradient passes over bf16 rows for C = 4, 8 (VALU kernel), 16, 32, 64 (MFMA kernel):
        best-of-3 ms, HBM TB/s of the row bytes, and the MFMA-form FLOP rate
    python scripts/mb_ml.py trees [--scale S]
        ForestEngine fits (20 trees, depth 5, 32 bins) with the phase split, cold and warm; GBT fits (20 iterations)
    python scripts/mb_ml.py tree-transform [--rows 2000000]
        the reference workflow's tree fits and transforms (ref.py:130-160) through the public API, each between
        device syncs; the first RF-regression transform also under cProfile

``--scale`` multiplies every row count (e.g. 0.05 for a quick check).
"""
import argparse
import cProfile
import io
import json
import os
import pstats
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from clustermachinelearningforhospitalnetworks_apache_spark_amd.ops import glm_ops  # noqa: E402


def best_ms(fn, reps=5):
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


def graph_ms(fn, reps=20):
    """ms per call with the calls captured into one HIP graph and replayed (best of 5 replays)."""
    fn()
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for _ in range(reps):
            fn()
    g.replay()
    torch.cuda.synchronize()
    ts = []
    for _ in range(5):
        s, e = torch.cuda.Event(True), torch.cuda.Event(True)
        s.record()
        g.replay()
        e.record()
        torch.cuda.synchronize()
        ts.append(s.elapsed_time(e) / reps)
    return min(ts)


def rows_x(n, d, dt):
    x = torch.randn(n, d, device="cuda")
    return (x.to(torch.bfloat16) if dt == torch.float8_e4m3fn else x).to(dt)


def glm_inputs(n, d):
    y = (torch.rand(n, device="cuda") > 0.5).double()
    return y, torch.randn(d + 1, device="cuda", dtype=torch.float64) * 0.05


def cmd_glm(argv):
    ap = argparse.ArgumentParser(prog="mb_ml.py glm")
    ap.add_argument("--scale", type=float, default=1.0)
    a = ap.parse_args(argv)
    shapes = [(20_000_000, 512, torch.float8_e4m3fn), (20_000_000, 256, torch.bfloat16),
              (10_000_000, 256, torch.float32), (20_000_000, 4, torch.float64), (20_000_000, 512, torch.bfloat16)]
    for n, d, dt in shapes:
        n = int(n * a.scale)
        x = rows_x(n, d, dt)
        y, coef = glm_inputs(n, d)
        gb = x.numel() * x.element_size() / 1e9
        mean = torch.zeros(d, dtype=torch.float64, device="cuda")
        inv = torch.ones(d, dtype=torch.float64, device="cuda")
        ops = [("moments", lambda: glm_ops.moments(x, d), 1),
               ("scale_apply", lambda: glm_ops.scale_apply(x, d, mean, inv, True, dt), 2),
               ("logreg_grad", lambda: glm_ops.logreg_grad(x, d, y, coef, None), 1),
               ("linear_predict", lambda: glm_ops.linear_predict(x, d, coef, "logistic"), 1)]
        if d <= 30:
            ops.append(("gram", lambda: glm_ops.gram(x, d, y, None), 1))
        for name, fn, passes in ops:
            t = best_ms(fn)
            print(f"n={n} d={d} {dt}: {name} {t:.3f} ms {passes * gb / t:.2f} TB/s{' (r+w)' if passes == 2 else ''}",
                  flush=True)
        del x, y
        torch.cuda.empty_cache()


def cmd_glm_fp8(argv):
    ap = argparse.ArgumentParser(prog="mb_ml.py glm-fp8")
    ap.add_argument("--rows", type=int, default=50_000_000)
    a = ap.parse_args(argv)
    n, d = a.rows, 512
    x = rows_x(n, d, torch.float8_e4m3fn)
    y, coef = glm_inputs(n, d)
    gb = x.numel() / 1e9
    ref = None
    for nch in (0, 2, 4):
        glm_ops.set_fp8_nch(nch)
        g = glm_ops.logreg_grad(x, d, y, coef, None)
        ref = g.clone() if ref is None else ref
        err = float((g - ref).abs().max() / ref.abs().max())
        t = best_ms(lambda: glm_ops.logreg_grad(x, d, y, coef, None))
        tm = best_ms(lambda: glm_ops.moments(x, d))
        tp = best_ms(lambda: glm_ops.linear_predict(x, d, coef, "logistic"))
        print(f"fp8 nch={nch or 'auto'}: logreg_grad {t:.3f} ms {gb / t:.2f} TB/s (rel diff {err:.1e}); "
              f"moments {gb / tm:.2f} TB/s; linear_predict {gb / tp:.2f} TB/s", flush=True)
    glm_ops.set_fp8_nch(0)


def cmd_logreg(argv):
    ap = argparse.ArgumentParser(prog="mb_ml.py logreg")
    ap.add_argument("--scale", type=float, default=1.0)
    ap.add_argument("--out", default=None)
    ap.add_argument("--unroll", type=int, default=1, help="K13 rows in flight per wave (1, 2; 0 = automatic)")
    a = ap.parse_args(argv)
    res = []
    glm_ops.set_logreg_unroll(a.unroll)
    for d, dt in ((256, torch.bfloat16), (512, torch.float8_e4m3fn), (256, torch.float32)):
        n = int((25_000_000 if dt == torch.float32 else 50_000_000) * a.scale)
        x = rows_x(n, d, dt)
        y, coef = glm_inputs(n, d)
        base = torch.zeros((), dtype=torch.int64, device="cuda")
        for b in sorted({min(b, n) for b in (16384, 131072, 1048576, n)}):
            t = graph_ms(lambda: glm_ops.logreg_grad(x, d, y, coef, None, batch=b, row_base=base),
                         reps=20 if b < n else 3)
            r = {"dtype": str(dt), "d": d, "U": a.unroll, "rows": b, "ms": round(t, 4),
                 "TB/s": round(b * d * x.element_size() / 1e9 / t, 2)}
            res.append(r)
            print(json.dumps(r), flush=True)
        part = torch.randn(1024, d + 3, dtype=torch.float64, device="cuda")
        t = graph_ms(lambda: glm_ops.partial_colsum(part))
        print(json.dumps({"op": "partial_colsum", "shape": [1024, d + 3], "us": round(t * 1e3, 2)}), flush=True)
        ts = sorted(best_ms(lambda: glm_ops.moments(x, d), 1) for _ in range(5))
        t = ts[2]
        r = {"dtype": str(dt), "d": d, "op": "moments", "rows": n, "ms": round(t, 3),
             "TB/s": round(n * d * x.element_size() / 1e9 / t, 2)}
        res.append(r)
        print(json.dumps(r), flush=True)
        del x, y
        torch.cuda.empty_cache()
    glm_ops.set_logreg_unroll(0)
    if a.out:
        json.dump(res, open(a.out, "w"), indent=1)


def cmd_trees(argv):
    from clustermachinelearningforhospitalnetworks_apache_spark_amd.models import trees as TR
    ap = argparse.ArgumentParser(prog="mb_ml.py trees")
    ap.add_argument("--scale", type=float, default=1.0)
    a = ap.parse_args(argv)

    def data(n, d):
        g = torch.Generator(device="cuda")
        g.manual_seed(0)
        x = torch.randn(n, d, device="cuda", dtype=torch.float64, generator=g)
        return x, 0.1 * torch.randn(n, device="cuda", dtype=torch.float64, generator=g)

    def timed(fn):
        torch.cuda.synchronize()
        t = time.perf_counter()
        r = fn()
        torch.cuda.synchronize()
        return time.perf_counter() - t, r

    for n, d, task in ((10_000_000, 4, "regression"), (10_000_000, 4, "classification"), (2_000_000, 64, "regression")):
        n = int(n * a.scale)
        x, noise = data(n, d)
        if task == "regression":
            y, imp = 2 * x[:, 0] + (x[:, 1 % d] > 0).double() + noise, "variance"
        else:
            y, imp = ((x[:, 0] + 0.5 * x[:, 2 % d]) > 0).double(), "gini"
        p = TR.TreeParams(task=task, num_classes=2, impurity=imp, num_trees=20, seed=1, feature_subset="auto")
        times = {}
        eng = TR.ForestEngine(x, y, p)
        for name in ("find_splits", "binize", "histogram", "best_splits", "route"):
            def wrap(*args, _fn=getattr(eng, name), _name=name, **kw):
                t, r = timed(lambda: _fn(*args, **kw))
                times[_name] = times.get(_name, 0.0) + t
                return r
            setattr(eng, name, wrap)
        for rep in ("cold", "warm"):  # the first fit of a process also loads every kernel it launches
            times.clear()
            t, trees = timed(eng.fit)
            nodes = sum(TR.num_nodes(r) for r in trees)
            print(f"RF{task[:5]} n={n} d={d} ({rep}): fit {t:.3f} s ({nodes} nodes) " +
                  " ".join(f"{k}={v:.3f}s" for k, v in times.items()), flush=True)
        del x, y, eng
        torch.cuda.empty_cache()
    # gradient boosting: 20 iterations of depth-5 regression trees (GBTRegressor defaults) / logistic loss
    for n, d, loss in ((10_000_000, 4, "squared"), (10_000_000, 4, "logistic"), (2_000_000, 64, "squared")):
        n = int(n * a.scale)
        x, noise = data(n, d)
        y = torch.sin(2 * x[:, 0]) + (x[:, 1 % d] > 0).double() + noise
        if loss == "logistic":
            y = torch.where(y > 0.5, 1.0, -1.0).double()
        t, (trees, tw) = timed(lambda: TR.fit_gbt(x, y, TR.TreeParams(max_depth=5, seed=1), 20, 0.1, loss))
        f = TR.predict_forest(trees, x, "variance", 1, False, False, tw)[:, 0]
        err = float(TR.gbt_loss(loss, f, y).mean())
        print(f"GBT-{loss} n={n} d={d}: fit {t:.3f} s for {len(trees)} trees ({t / len(trees) * 1e3:.1f} ms/tree), "
              f"train loss {err:.4f}", flush=True)
        del x, y
        torch.cuda.empty_cache()


def cmd_tree_transform(argv):
    from clustermachinelearningforhospitalnetworks_apache_spark_amd.ml.classification import (
        DecisionTreeClassifier, RandomForestClassifier)
    from clustermachinelearningforhospitalnetworks_apache_spark_amd.ml.feature import VectorAssembler
    from clustermachinelearningforhospitalnetworks_apache_spark_amd.ml.regression import (
        DecisionTreeRegressor, RandomForestRegressor)
    from clustermachinelearningforhospitalnetworks_apache_spark_amd.sql import SparkSession
    ap = argparse.ArgumentParser(prog="mb_ml.py tree-transform")
    ap.add_argument("--rows", type=int, default=int(os.environ.get("MB_ROWS", 2_000_000)))
    a = ap.parse_args(argv)
    n = a.rows
    spark = SparkSession.builder.master("mi355x" if torch.cuda.is_available() else "local[4]").getOrCreate()
    dev = spark._device
    g = torch.Generator(device=dev).manual_seed(0)
    cols = {c: torch.randint(0, 100, (n,), generator=g, device=dev).to(torch.int32)
            for c in ("admission_count", "current_occupancy", "emergency_visits")}
    cols["seasonality_index"] = torch.rand(n, generator=g, device=dev, dtype=torch.float64)
    los = (cols["admission_count"].double() * 0.05 + cols["seasonality_index"] * 3
           + torch.rand(n, generator=g, device=dev, dtype=torch.float64))
    cols["length_of_stay"] = los
    cols["LOS_binary"] = (los > 5.0).to(torch.int32)
    df = spark.createDataFrameFromTensors(cols)
    feats = ["admission_count", "current_occupancy", "emergency_visits", "seasonality_index"]

    def sync():
        if torch.cuda.is_available():
            torch.cuda.synchronize()

    def timed(name, fn):
        sync()
        t = time.perf_counter()
        out = fn()
        sync()
        print(f"{name:36s} {1000 * (time.perf_counter() - t):9.2f} ms", flush=True)
        return out

    va = VectorAssembler(inputCols=feats, outputCol="features")
    tr, te = va.transform(df).select("features", "length_of_stay").randomSplit([0.7, 0.3], seed=42)
    dt = timed("DecisionTreeRegressor.fit",
               lambda: DecisionTreeRegressor(featuresCol="features", labelCol="length_of_stay").fit(tr))
    timed("DecisionTreeRegressionModel.transform", lambda: dt.transform(te))
    rf = timed("RandomForestRegressor.fit",
               lambda: RandomForestRegressor(featuresCol="features", labelCol="length_of_stay").fit(tr))
    print("rf trees", len(rf._trees), "nodes", rf.totalNumNodes, "depths", [rf.trees[i].depth for i in range(3)])
    pr = cProfile.Profile()
    sync()
    pr.enable()
    timed("RandomForestRegressionModel.transform", lambda: rf.transform(te))
    pr.disable()
    s = io.StringIO()
    pstats.Stats(pr, stream=s).sort_stats("cumulative").print_stats(25)
    print(s.getvalue())
    for _ in range(2):
        timed("RandomForestRegressionModel.transform", lambda: rf.transform(te))
    ctr, cte = va.transform(df).select("features", "LOS_binary").randomSplit([0.7, 0.3], seed=42)
    rfc = timed("RandomForestClassifier.fit",
                lambda: RandomForestClassifier(featuresCol="features", labelCol="LOS_binary").fit(ctr))
    timed("RandomForestClassificationModel.transform", lambda: rfc.transform(cte))
    dtc = timed("DecisionTreeClassifier.fit",
                lambda: DecisionTreeClassifier(featuresCol="features", labelCol="LOS_binary").fit(ctr))
    timed("DecisionTreeClassificationModel.transform", lambda: dtc.transform(cte))


def _mode_run(mode, x, d, y, coef, C, cp, dp):
    prev = glm_ops.set_multinomial_mfma_mode(mode)
    try:
        lib = glm_ops._native.kernels()
        code = glm_ops._CODE[x.dtype]
        cp, dp = lib.cml_multinomial_mfma_supported(d, code, C), lib.cml_multinomial_mfma_dpad(d, C)
        if cp <= 0:
            return None
        return glm_ops._multinomial_mfma(x, d, y, coef, None, C, cp, dp)
    finally:
        glm_ops.set_multinomial_mfma_mode(prev)


def cmd_multinomial(argv):
    ap = argparse.ArgumentParser(prog="mb_ml.py multinomial")
    ap.add_argument("--rows", type=int, default=100_000_000)
    ap.add_argument("--dim", type=int, default=256)
    ap.add_argument("--dtype", default="bf16", choices=["bf16", "fp8"], help="row storage (fp8: OCP e4m3)")
    ap.add_argument("--classes", default="4,8,16,32,64")
    a = ap.parse_args(argv)
    from clustermachinelearningforhospitalnetworks_apache_spark_amd.utils import synth
    dev = torch.device("cuda", 0)
    n, d = a.rows, a.dim
    x = synth.synth_rows(0, n, d, seed=3, dtype=torch.bfloat16, device=dev)
    code, esz = 0, 2
    if a.dtype == "fp8":
        x = x.to(torch.float8_e4m3fn)
        code, esz = 3, 1
    lib = __import__("clustermachinelearningforhospitalnetworks_apache_spark_amd._native",
                     fromlist=["kernels"]).kernels()
    g = torch.Generator(device=dev)
    g.manual_seed(1)
    for C in (int(c) for c in a.classes.split(",")):
        y = torch.randint(0, C, (n,), generator=g, device=dev).to(torch.float64)
        coef = torch.randn(C, d + 1, generator=g, device=dev, dtype=torch.float64) * 0.05
        # MFMA form: margins + gradient on the padded class tile (16, 32 or 64 classes)
        flop = 4.0 * n * d * (16 if C <= 16 else 32 if C <= 32 else 64)  # (mode 3: 32 for C <= 16 too)
        runs = []
        if lib.cml_multinomial_supported(d, code, C) > 0:
            runs.append(("valu", lambda: glm_ops.multinomial_grad(x, d, y, coef, prefer_valu=True)))
        cp = lib.cml_multinomial_mfma_supported(d, code, C)
        if cp > 0:  # every MFMA form (mode 0, the first, is the default route)
            dp = lib.cml_multinomial_mfma_dpad(d, C)
            for mode, name in ((0, "mfma-bf16x3"), (3, "mfma-bf16x3-32tile"), (2, "mfma-bf16x3-regsplit"),
                               (1, "mfma-f32")):
                if (mode == 3 and C > 16) or (code == 3 and mode in (1, 2)):  # (e4m3 rows: bf16 forms only)
                    continue
                runs.append((name, (lambda m: lambda: _mode_run(m, x, d, y, coef, C, cp, dp))(mode)))
        if not runs:
            runs.append(("torch-chunks", lambda: glm_ops.multinomial_grad(x, d, y, coef)))
        if code == 0 and lib.cml_multinomial_predict_lds(d, 0, C) > 0:  # K13t: transform (raw + probability, f64 [n, C] each)
            ms = best_ms(lambda: glm_ops.multinomial_predict(x, d, coef), reps=3)
            byts = n * d * 2 + 2 * n * C * 8
            print(f"multinomial transform {n}x{d} bf16 C={C:2d} [K13t f64 mfma]: {ms:8.3f} ms, "
                  f"{byts / ms / 1e9:6.2f} TB/s (rows in + raw/prob out)", flush=True)
        for name, fn in runs:
            ms = best_ms(fn, reps=3)
            print(f"multinomial {n}x{d} {a.dtype} C={C:2d} [{name}]: {ms:8.3f} ms, {n * d * esz / ms / 1e9:6.2f} TB/s rows"
                  + (f", {flop / ms / 1e9:7.1f} useful TFLOP/s" if name.startswith("mfma") else ""), flush=True)
        del y


COMMANDS = {"multinomial": cmd_multinomial, "glm": cmd_glm, "glm-fp8": cmd_glm_fp8, "logreg": cmd_logreg, "trees": cmd_trees,
            "tree-transform": cmd_tree_transform}

if __name__ == "__main__":
    if len(sys.argv) < 2 or sys.argv[1] not in COMMANDS:
        print(__doc__)
        sys.exit(2)
    COMMANDS[sys.argv[1]](sys.argv[2:])
