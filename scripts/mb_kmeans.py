"""KMeans engine microbenchmarks (Lloyd step, accumulate, row pass, pruning, precision paths): one driver, one
subcommand per experiment. The K9/K9r assign pass on its own is scripts/mb_k9r.py.

    python scripts/mb_kmeans.py accum [--scale S]
        one Lloyd step (assign + accumulate + update) eager and graph-replayed, both accumulate regimes, on six shapes
    python scripts/mb_kmeans.py segacc [--rows 50000000] [--reps 5]
        the sort-regime accumulate (K10 counting sort + segmented f64 sums) alone, plain and with the seeded step's
        upper-bound side output
    python scripts/mb_kmeans.py overlap [--rows 25000000]
        a chunk's accumulate and the next chunk's assign alone, serial, and on two HIP streams
    python scripts/mb_kmeans.py rowpass [--rows 100000000]
        the fused row pass (f32 + f64 norms, first k-means|| costs, max norm, exponent range) with checksums
    python scripts/mb_kmeans.py prune [--rows 100000000] [--dim 256] [--k 256] [--steps 10] [--warmup 3]
        pruned Lloyd steps: untraced ms/step, then per-phase device-synchronised ranges and candidates per step
    python scripts/mb_kmeans.py bounds [--rows 12500000] [--cand 0.03] [--k 256] [--reps 20]
        the K9p bounds pass alone against a device copy of its 12 B/row, and a check of its candidate lists
    python scripts/mb_kmeans.py churn [--rows 20000000]
        fraction of rows whose label changes per Lloyd iteration
    python scripts/mb_kmeans.py graph [--rows 12500000]
        Lloyd step eager vs HIP graph at one 8-GPU shard, with 1 and 2 row chunks (host enqueue vs step time)
    python scripts/mb_kmeans.py cert [--rows 10000000] [--dim 128] [--k 64] [--reps 3]
        certified f32 path (config-2 shape): public-API fit, transform's prediction column and computeCost, each
        checked bit for bit against exact_assign
    python scripts/mb_kmeans.py fp8-mx [--rows 20000000] [--dim 512] [--k 128] [--steps 8]
        fp8 rows: MX-scaled fp8 MFMAs against the bf16 widening pass, one assign pass and pruned steps each way
    python scripts/mb_kmeans.py host [--rows 12500000] [--dim 256] [--k 256] [--iters 20] [--top 45]
        cProfile of the timed public-API fit after two warm-ups (scripts/sync_audit.py lists its blocking reads)
"""
import argparse
import cProfile
import io
import os
import pstats
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
from clustermachinelearningforhospitalnetworks_apache_spark_amd.models.kmeans import LloydEngine  # noqa: E402
from clustermachinelearningforhospitalnetworks_apache_spark_amd.ops import kmeans_ops as K  # noqa: E402

DEV = torch.device("cuda", 0)


def event_list(fn, reps):
    ts = []
    for _ in range(reps):
        s, e = torch.cuda.Event(True), torch.cuda.Event(True)
        s.record()
        fn()
        e.record()
        torch.cuda.synchronize()
        ts.append(s.elapsed_time(e))
    return ts


def best_ms(fn, reps=3):
    fn()
    torch.cuda.synchronize()
    return min(event_list(fn, reps))


def blobs(n, d, k, g):
    cen = torch.randn(k, d, device="cuda", generator=g) * 4
    return (cen[torch.randint(0, k, (n,), device="cuda", generator=g)] +
            torch.randn(n, d, device="cuda", generator=g)).to(torch.bfloat16)


def parse(name, argv, **opts):
    ap = argparse.ArgumentParser(prog=f"mb_kmeans.py {name}")
    for key, default in opts.items():
        ap.add_argument("--" + key.replace("_", "-"), type=type(default), default=default)
    return ap.parse_args(argv)


def cmd_accum(argv):
    a = parse("accum", argv, scale=1.0)
    for n, d, k in ((20_000_000, 256, 256), (10_000_000, 128, 64), (20_000_000, 16, 5), (4_000_000, 512, 128),
                    (1_250_000, 128, 64), (100_000, 16, 5)):
        n = max(k, int(n * a.scale))
        x = blobs(n, d, k, torch.Generator(device="cuda").manual_seed(0))
        gb = n * d * 2 / 1e9
        for mode in (None, "priv"):
            try:
                eng = LloydEngine(x, d, k, accum_mode=mode)
            except ValueError as e:
                print(f"n={n} d={d} k={k} mode={mode}: {e}")
                continue
            eng.set_centers(x[:k].double().cpu().numpy())
            if mode is None:
                ap = K.plan_assign(n, eng.dp, k)
                t = best_ms(lambda: K.assign_bf16(x, n, eng.dp, eng.cb, eng.cnorm, ap, eng.labels, eng.best,
                                                  eng.cost_part, xnorm=eng.xnorm))
                print(f"n={n} d={d} k={k} grid {ap.grid}x{ap.nwaves}w: assign {t:.3f} ms ({gb / t:.2f} TB/s, "
                      f"{2 * n * d * k / t / 1e9:.0f} TF/s)", flush=True)
            for graph in (False, True):
                eng.use_graph = graph
                t = best_ms(eng.step, reps=5)
                print(f"n={n} d={d} k={k} {eng.cplan} graph={graph}: step {t:.3f} ms -> {n / t / 1e6:.2f} Gsamples/s",
                      flush=True)
            del eng
            torch.cuda.empty_cache()
        del x
        torch.cuda.empty_cache()


def cmd_segacc(argv):
    a = parse("segacc", argv, rows=50_000_000, reps=5)
    n, d, k = a.rows, 256, 256
    x = bench.make_blobs(n, d, k, seed=1, device=DEV)
    eng = LloydEngine(x, d, k, prune=False, use_graph=False)
    eng.set_centers(x[:k].double().cpu().numpy())
    eng.step()  # labels, ranks and histograms of a full K9r pass
    torch.cuda.synchronize()
    msg = torch.zeros_like(eng.msgs[0])
    ub = torch.empty(n, dtype=torch.float32, device=DEV)
    print(f"sum grid scale {eng._qscale!r} (0: plain f64 sums)")

    def run(with_ub):
        K.accumulate_sort(x, n, eng.dp, d, eng.labels, eng.rank, eng.hist, eng.aplan, k, eng.cost_part, eng.off,
                          eng.seg, eng.perm, eng.cplan, msg, eng.slots, ub_centres=eng.cb if with_ub else None,
                          ub=ub if with_ub else None, qscale=eng._qscale)

    for with_ub in (False, True):
        run(with_ub)
        torch.cuda.synchronize()
        ts = sorted(event_list(lambda: run(with_ub), a.reps))
        print(f"accumulate_sort n={n} d={d} k={k} ub={with_ub}: best {ts[0]:.3f} ms, median {ts[len(ts) // 2]:.3f} ms"
              f" ({n * d * 2 / 1e9 / ts[0]:.2f} TB/s of rows)", flush=True)


def cmd_overlap(argv):
    a = parse("overlap", argv, rows=25_000_000)
    n, d, k = a.rows, 256, 256
    g = torch.Generator(device="cuda").manual_seed(0)
    cen = torch.randn(k, d, device="cuda", generator=g) * 4
    xs = [(cen[torch.randint(0, k, (n,), device="cuda", generator=g)] +
           torch.randn(n, d, device="cuda", generator=g)).to(torch.bfloat16) for _ in range(2)]
    init = xs[0][:k].double().cpu().numpy()
    s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()
    ea, eb = [LloydEngine(x, d, k, accum_mode="sort", use_graph=False) for x in xs]
    for e in (ea, eb):
        e.set_centers(init)
        e.step()

    def assign(e, stream=None):
        K.assign_bf16(e.x, e.n, e.dp, e.cb, e.cnorm, e.aplan, e.labels, e._best(0, e.n), e.cost_part, e.hist,
                      e.rank, stream=stream, xnorm=e.xnorm)

    def accum(e, stream=None):
        K.accumulate_sort(e.x, e.n, e.dp, e.d, e.labels, e.rank, e.hist, e.aplan, e.k, e.cost_part, e.off, e.seg,
                          e.perm, e.cplan, e.msgs[0], e.slots, stream=stream)

    def both():
        cur = torch.cuda.current_stream()
        s1.wait_stream(cur)
        s2.wait_stream(cur)
        assign(eb, s1)
        accum(ea, s2)
        cur.wait_stream(s1)
        cur.wait_stream(s2)

    ta, tc = best_ms(lambda: assign(eb)), best_ms(lambda: accum(ea))
    ts = best_ms(lambda: (assign(eb), accum(ea)))
    tb = best_ms(both)
    print(f"grid {eb.aplan.grid}: assign {ta:.3f} ms, accumulate {tc:.3f} ms, serial {ts:.3f} ms, two streams "
          f"{tb:.3f} ms (overlap saves {ts - tb:.3f} ms)", flush=True)


def cmd_rowpass(argv):
    a = parse("rowpass", argv, rows=100_000_000)
    n, dp = a.rows, 256
    x = torch.empty((n, dp), dtype=torch.bfloat16, device="cuda")
    for s in range(0, n, 1 << 24):
        x[s:s + (1 << 24)] = torch.randn((min(1 << 24, n - s), dp), device="cuda").to(torch.bfloat16)
    xn = torch.empty(n, device="cuda")
    xn64 = torch.empty(n, dtype=torch.float64, device="cuda")
    cost = torch.empty(n, device="cuda")
    near = torch.empty(n, dtype=torch.int32, device="cuda")
    c0 = x[7].float().contiguous()
    c0n = float((c0.double() ** 2).sum())
    mx = torch.zeros(1, device="cuda")
    best = 1e30
    for _ in range(10):
        er = torch.tensor([2 ** 31 - 1, -1], dtype=torch.int32, device="cuda")
        best = min(best, event_list(lambda: K.row_pass(x, n, dp, xn, c0, c0n, cost, near, xn_max=mx, erange=er,
                                                       xn64=xn64), 1)[0])
    print(f"row_pass {best:.3f} ms {n * dp * 2 / best / 1e9:.2f} TB/s erange={er.tolist()} "
          f"sum(xn)={float(xn.double().sum())!r} sum(xn64)={float(xn64.sum())!r} "
          f"sum(cost)={float(cost.double().sum())!r}", flush=True)


def cmd_prune(argv):
    from clustermachinelearningforhospitalnetworks_apache_spark_amd.utils.trace import TRACER
    a = parse("prune", argv, rows=100_000_000, dim=256, k=256, steps=10, warmup=3)
    x = bench.make_blobs(a.rows, a.dim, a.k, seed=1000, device=DEV)
    eng = LloydEngine(x, a.dim, a.k, prune=True)
    eng.set_centers(eng.init_kmeans_parallel(seed=42))
    for i in range(a.warmup):
        eng.step()
        print("warmup", i, eng.prune_stats(), flush=True)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(a.steps):
        eng.step()
    torch.cuda.synchronize()
    print(f"untraced: {1e3 * (time.perf_counter() - t0) / a.steps:.3f} ms/step", flush=True)
    TRACER.enable(sync=True)
    TRACER.reset()
    for i in range(a.steps):
        eng.step()
        print("step", i, eng.prune_stats(), flush=True)
    print(TRACER.report())


def cmd_bounds(argv):
    a = parse("bounds", argv, rows=12_500_000, cand=0.03, k=256, reps=20)
    n, k = a.rows, a.k
    g = torch.Generator(device=DEV).manual_seed(3)
    lab = torch.randint(0, k, (n,), generator=g, device=DEV, dtype=torch.int32)
    # offset-form bounds: ub - cu[label], lb + cl[label] with zero drifts; a row is proven when ub <= thr[label]
    thr = torch.full((k,), 1.0, device=DEV)
    ub = torch.where(torch.rand(n, generator=g, device=DEV) < a.cand, 2.0, 0.5).to(torch.float32)
    lb = torch.full((n,), 0.1, device=DEV)
    drift, dmax, cum = torch.zeros(k, device=DEV), torch.zeros(3, device=DEV), torch.zeros(2 * k, device=DEV)
    c2 = torch.full((1,), 1e-3, device=DEV)
    cand = torch.zeros(n + 1024, dtype=torch.int32, device=DEV)
    cand_lab = torch.zeros_like(cand)
    cand_xn = torch.zeros(n + 1024, device=DEV)
    xn = torch.rand(n, generator=g, device=DEV)
    count = torch.zeros(1, dtype=torch.int32, device=DEV)

    def run():
        K.prune_bounds(lab, ub, lb, drift, dmax, thr, c2, k, cand, count, xn=xn, cand_lab=cand_lab, cand_xn=cand_xn,
                       cum=cum)

    def med(fn):
        fn()
        torch.cuda.synchronize()
        return sorted(event_list(fn, a.reps))[a.reps // 2]

    t = med(run)
    src = torch.empty(3 * n, dtype=torch.int32, device=DEV)
    dst = torch.empty_like(src)
    tc = med(lambda: dst.copy_(src))
    print(f"bounds pass n={n} k={k} candidates {int(count.item())} ({a.cand:.0%}): {1e3 * t:.1f} us "
          f"({12 * n / t / 1e9:.2f} TB/s of bounds); copy of 12 B/row: {1e3 * tc:.1f} us "
          f"({24 * n / tc / 1e9:.2f} TB/s read+write)", flush=True)
    m = int(count.item())
    rows = cand[:m].long()
    want = torch.nonzero(ub > 1.0).flatten()
    ok = (torch.equal(torch.sort(rows).values, want) and torch.equal(cand_lab[:m], lab[rows])
          and torch.equal(cand_xn[:m], xn[rows]))
    print(f"candidate list (rows, labels, norms) correct: {ok}", flush=True)
    if not ok:
        raise SystemExit(1)


def cmd_churn(argv):
    a = parse("churn", argv, rows=20_000_000, iters=25)
    n = a.rows
    x = bench.make_blobs(n, 256, 256, seed=1000, device=DEV)
    eng = LloydEngine(x, 256, 256, use_graph=False)
    eng.set_centers(eng.init_kmeans_parallel(seed=42))
    prev = None
    for it in range(a.iters):
        eng.step()
        lab = eng.labels[:n].clone()
        if prev is not None:
            ch = int((lab != prev).sum().item())
            print(f"iter {it}: changed {ch} ({100.0 * ch / n:.3f}%)", flush=True)
        prev = lab


def cmd_graph(argv):
    a = parse("graph", argv, rows=12_500_000, steps=20)
    x = bench.make_blobs(a.rows, 256, 256, seed=1000, device=DEV)
    for chunks in (1, 2):
        for graph in (False, True):
            eng = LloydEngine(x, 256, 256, row_chunks=chunks, use_graph=graph)
            eng.set_centers(eng.init_kmeans_parallel(seed=42))
            for _ in range(4):
                eng.step()
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(a.steps):
                eng.step()
            t_host = (time.perf_counter() - t0) / a.steps
            torch.cuda.synchronize()
            t_all = (time.perf_counter() - t0) / a.steps
            print(f"chunks={chunks} graph={graph}: {1e3 * t_all:.3f} ms/step (host enqueue {1e3 * t_host:.3f} "
                  f"ms/step)", flush=True)
            del eng
            torch.cuda.empty_cache()


def _fit_frame(rows, dim, k, seed, dtype=None):
    from clustermachinelearningforhospitalnetworks_apache_spark_amd.sql import SparkSession
    spark = SparkSession.builder.master("mi355x").getOrCreate()
    x = bench.make_blobs(rows, dim, k, seed=seed, device=DEV)
    x = x.to(dtype) if dtype is not None else x
    return x, spark.createDataFrameFromTensors({"features": x})


def cmd_cert(argv):
    import numpy as np

    from clustermachinelearningforhospitalnetworks_apache_spark_amd.ml.clustering import KMeans
    a = parse("cert", argv, rows=10_000_000, dim=128, k=64, reps=3)
    x, df = _fit_frame(a.rows, a.dim, a.k, 1, torch.float32)
    km = KMeans(k=a.k, maxIter=20, tol=0.0, seed=42)
    km.fit(df)  # warm-up

    def wall(fn):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        out = fn()
        torch.cuda.synchronize()
        return 1e3 * (time.perf_counter() - t0), out

    fits = [wall(lambda: km.fit(df)) for _ in range(a.reps)]
    model = fits[-1][1]
    print(f"fit ms {[round(t, 2) for t, _ in fits]}", flush=True)
    tr = [wall(lambda: model.transform(df)._column_data("prediction").values) for _ in range(a.reps + 1)]
    pred = tr[-1][1]
    print(f"transform (prediction column materialised) ms {[round(t, 2) for t, _ in tr]}", flush=True)
    t, cost = wall(lambda: model.computeCost(df))
    print(f"computeCost {cost} in {t:.2f} ms", flush=True)
    cen = torch.as_tensor(np.stack(model.clusterCenters()), dtype=torch.float64, device=DEV)
    t, (lab_ex, d_ex) = wall(lambda: K.exact_assign(x, cen))
    print(f"exact_assign {t:.2f} ms; labels equal: {bool(torch.equal(lab_ex.long(), pred.long()))}; "
          f"cost equal: {cost == float(d_ex.sum().item())}", flush=True)


def cmd_fp8_mx(argv):
    a = parse("fp8-mx", argv, rows=20_000_000, dim=512, k=128, steps=8)
    n, d, k = a.rows, a.dim, a.k
    g = torch.Generator(device=DEV).manual_seed(7)
    cen = torch.randn(32, d, generator=g, device=DEV) * 3  # config-5 shaped: 32 standardised blobs in e4m3
    x8 = torch.empty((n, d), dtype=torch.float8_e4m3fn, device=DEV)
    for s0 in range(0, n, 1 << 21):
        m = min(1 << 21, n - s0)
        z = cen[torch.randint(0, 32, (m,), generator=g, device=DEV)] + torch.randn((m, d), generator=g, device=DEV)
        x8[s0:s0 + m] = (z / 3.2).clamp(-440, 440).to(torch.float8_e4m3fn)
        del z
    init = x8[torch.randperm(n, generator=torch.Generator().manual_seed(1))[:k].to(DEV)].float().double().cpu().numpy()
    torch.cuda.synchronize()

    def ms(fn, reps=5):
        fn()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(reps):
            fn()
        torch.cuda.synchronize()
        return 1e3 * (time.perf_counter() - t0) / reps

    labels = {}
    for mx in (True, False):
        K.set_fp8_mx(mx)
        eng = LloydEngine(x8, d, k, prune=True, use_graph=False)
        eng.set_centers(init)
        eng.step()  # first step (norms, state)
        lab = torch.empty(n, dtype=torch.int32, device=DEV)
        best = torch.empty(n, dtype=torch.float32, device=DEV)
        t_pass = ms(lambda: K.assign_bf16(x8, n, eng.dp, eng.cb, eng.cnorm, eng.aplan, lab, best, None,
                                          xnorm=eng.xnorm))
        times, full = [], []
        for _ in range(a.steps):
            t0 = time.perf_counter()
            eng.step()
            torch.cuda.synchronize()
            times.append(1e3 * (time.perf_counter() - t0))
            full.append(eng.prune_stats()["full"])
        labels[mx] = eng.labels[:n].clone()
        print(f"mx={mx}: K9r pass {t_pass:.2f} ms ({n * k * d * 2 / t_pass / 1e9:.0f} TFLOP/s); pruned steps ms "
              f"{[round(t, 2) for t in times]} full {full}", flush=True)
        del eng
        torch.cuda.empty_cache()
    K.set_fp8_mx(True)
    print("labels differing after the steps:", int((labels[True] != labels[False]).sum().item()), "of", n)


def cmd_host(argv):
    from clustermachinelearningforhospitalnetworks_apache_spark_amd.ml.clustering import KMeans
    a = parse("host", argv, rows=12_500_000, dim=256, k=256, iters=20, top=45)
    _, df = _fit_frame(a.rows, a.dim, a.k, 1)
    for _ in range(2):
        KMeans(k=a.k, maxIter=a.iters, tol=0.0, seed=42).fit(df)  # warm-up (kernel loads, allocator, norms)
    torch.cuda.synchronize()
    pr = cProfile.Profile()
    t0 = time.perf_counter()
    pr.enable()
    KMeans(k=a.k, maxIter=a.iters, tol=0.0, seed=42).fit(df)
    torch.cuda.synchronize()
    pr.disable()
    print(f"fit wall {1e3 * (time.perf_counter() - t0):.2f} ms (under cProfile)")
    for key in ("tottime", "cumulative"):
        s = io.StringIO()
        pstats.Stats(pr, stream=s).sort_stats(key).print_stats(a.top)
        print(f"=== by {key}")
        print("\n".join(line for line in s.getvalue().splitlines() if line.strip())[:20000])


COMMANDS = {"accum": cmd_accum, "segacc": cmd_segacc, "overlap": cmd_overlap, "rowpass": cmd_rowpass,
            "prune": cmd_prune, "bounds": cmd_bounds, "churn": cmd_churn, "graph": cmd_graph, "cert": cmd_cert,
            "fp8-mx": cmd_fp8_mx, "host": cmd_host}

if __name__ == "__main__":
    if len(sys.argv) < 2 or sys.argv[1] not in COMMANDS:
        print(__doc__)
        sys.exit(2)
    COMMANDS[sys.argv[1]](sys.argv[2:])
