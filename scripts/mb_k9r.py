"""K9 / K9r assign microbenchmarks (the fused MFMA distance + argmin pass, kmeans_rr.h): one driver, one
subcommand per experiment. Positional arguments default to the headline shape, 20M x 256 bf16, k = 256.

    python scripts/mb_k9r.py rr [N D K [VARIANTS [fp8]]]
        in-process A/B of assign variants (0 = K9, 8 = K9r, 9 = K9 with the K9r default off), alternated round by
        round so DVFS drift hits all; full pass and compute-only pass (every row aliases row 0: no HBM stream)
    python scripts/mb_k9r.py dbg [N D K [fp8]]
        K9r ablation by its `dbg` bits (1 no LDS-DMA, 2 no MFMA/keys, 4 no finalize, and their unions);
        fp8: e4m3 rows, the MX pass unless CML_KMEANS_FP8_MX=0
    python scripts/mb_k9r.py modes [N D K]
        the K9r modes: 0 (assign + counting-sort ranks), 1 (top-2 bounds), 2 (candidate rows at 2/5/20 %), the
        fused row pass, and the centre tiles per wave for k = 64..320
    python scripts/mb_k9r.py pmc [VARIANT N D K DBG]
        dispatches for a PMC pass: 3 full passes then 3 compute-only passes (identify them by order)
    python scripts/mb_k9r.py pmc-mode [N D K MODE]
        3 launches of K9r mode 0 or mode 1 (top-2) for a PMC pass
    python scripts/mb_k9r.py clock
        rows from HBM, from L2, MFMA only and without the LDS-DMA, 6 launches each (scripts/gpu.sh clock runs it
        under rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES)
    python scripts/mb_k9r.py clock-show DIR
        per-dispatch clock and MFMA busy share from that run's counter CSV (no GPU)
    python scripts/mb_k9r.py ablate [VARIANTS]
        K9 launch variants (kmeans_ops.set_assign_variant): full vs compute-only vs a 32-centre launch, three shapes
    python scripts/mb_k9r.py sched [N [SCHEDS]]
        K9 pass time vs partner-wave scheduling (kmeans_ops.set_assign_sched), plus its compute and memory bounds
"""
import csv
import glob
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def _arg(argv, i, default, conv=int):
    return conv(argv[i]) if len(argv) > i else default


def _env():
    import torch

    import bench
    from clustermachinelearningforhospitalnetworks_apache_spark_amd import _native
    from clustermachinelearningforhospitalnetworks_apache_spark_amd.models import kmeans as KM
    from clustermachinelearningforhospitalnetworks_apache_spark_amd.ops import kmeans_ops as K
    return torch, bench, _native, KM, K


def engine(n, d, k, fp8=False, scale=1.0):
    """Blobs of the bench's shape on the device, a LloydEngine on them with the first k rows as centres, and the
    stride-0 view of its rows (every row is row 0: the pass without its HBM stream)."""
    torch, bench, _, KM, _ = _env()
    x = bench.make_blobs(n, d, k, seed=1000, device=torch.device("cuda"))
    if fp8:
        x = (x.float() / scale).clamp(-440, 440).to(torch.float8_e4m3fn)
    eng = KM.LloydEngine(x, d, k, use_graph=False)
    eng.set_centers(x[:k].to(torch.float32).double().cpu().numpy())
    return eng, torch.as_strided(eng.x, (n, eng.dp), (0, 1))


def assign(eng, xx, plan=None):
    _, _, _, _, K = _env()
    K.assign_bf16(xx, xx.shape[0], eng.dp, eng.cb, eng.cnorm, plan or eng.aplan, eng.labels, None, eng.cost_part,
                  eng.hist, eng.rank, xnorm=eng.xnorm)


def event_ms(fn, reps=5):
    import torch
    ts = []
    for _ in range(reps):
        a, b = torch.cuda.Event(True), torch.cuda.Event(True)
        a.record()
        fn()
        b.record()
        torch.cuda.synchronize()
        ts.append(a.elapsed_time(b))
    return ts


def wall_ms(fn, reps=7):
    import torch
    fn()
    torch.cuda.synchronize()
    ts = []
    for _ in range(reps):
        t = time.perf_counter()
        fn()
        torch.cuda.synchronize()
        ts.append(time.perf_counter() - t)
    return 1000 * sorted(ts)[reps // 2]


def cmd_rr(argv):
    torch, _, _, _, K = _env()
    n, d, k = _arg(argv, 0, 20_000_000), _arg(argv, 1, 256), _arg(argv, 2, 256)
    variants = [int(v) for v in argv[3].split(",")] if len(argv) > 3 else [0, 8]
    fp8 = len(argv) > 4 and argv[4] == "fp8"
    eng, x0 = engine(n, d, k, fp8)
    print(f"n={n} d={d} (padded {eng.dp}) k={k} {'fp8' if fp8 else 'bf16'}", flush=True)
    plans = {}
    for v in variants:
        K.set_assign_variant(0 if v == 9 else v)
        K.set_rr_default(v != 9)
        plans[v] = K.plan_assign(n, eng.dp, k, fp8=fp8)
    K.set_assign_variant(0)
    K.set_rr_default(True)
    labels, res = {}, {(v, m): [] for v in variants for m in ("full", "compute")}
    for rnd in range(5):
        for v in variants:
            eng.labels.fill_(-1)
            assign(eng, eng.x, plans[v])
            torch.cuda.synchronize()
            if rnd == 0:
                labels[v] = eng.labels.clone()
            res[(v, "full")] += event_ms(lambda: assign(eng, eng.x, plans[v]))
            res[(v, "compute")] += event_ms(lambda: assign(eng, x0, plans[v]))
        print(f"round {rnd} done", flush=True)
    for v in variants:
        same = float((labels[v] == labels[variants[0]]).float().mean())
        for m in ("full", "compute"):
            ts = sorted(res[(v, m)])
            t = ts[len(ts) // 2]
            print(f"variant {v} (grid {plans[v].grid}, rr_ct {plans[v].rr_ct}) {m:8s}: median {t:.3f} ms "
                  f"(min {ts[0]:.3f}) -> {2 * n * d * k / t / 1e9:.0f} TF/s, "
                  f"{n * eng.dp * eng.x.element_size() / t / 1e9:.2f} TB/s; label agreement with variant "
                  f"{variants[0]}: {same:.6f}", flush=True)


def cmd_dbg(argv):
    _, _, _native, _, K = _env()
    n, d, k = _arg(argv, 0, 20_000_000), _arg(argv, 1, 256), _arg(argv, 2, 256)
    fp8 = len(argv) > 3 and argv[3] == "fp8"
    K.set_assign_variant(8)
    eng, x0 = engine(n, d, k, fp8, scale=3.2)
    lib = _native.kernels()
    print(f"n={n} d={d} k={k} rr_ct={eng.aplan.rr_ct} grid={eng.aplan.grid} fp8={fp8} mx={eng._mx}", flush=True)
    rowb = eng.dp * (1 if fp8 else 2)
    order = (0, 1, 2, 4, 3, 6, 5)
    names = {0: "all on", 1: "no DMA", 2: "no MFMA", 4: "no finalize", 3: "finalize only", 6: "DMA only",
             5: "MFMA only"}
    res = {}
    for _ in range(3):
        for bits in order:
            lib.cml_kmeans_set_rr_debug(bits)
            res.setdefault((bits, "full"), []).append(sorted(event_ms(lambda: assign(eng, eng.x)))[2])
            res.setdefault((bits, "compute"), []).append(sorted(event_ms(lambda: assign(eng, x0)))[2])
    lib.cml_kmeans_set_rr_debug(0)
    for bits in order:
        f, c = sorted(res[(bits, "full")])[1], sorted(res[(bits, "compute")])[1]
        print(f"dbg {bits} {names[bits]:14s}: full {f:.3f} ms ({n * rowb / f / 1e9:.2f} TB/s)  compute-only {c:.3f} ms",
              flush=True)


def _raw_problem(n, d, k, g):
    """Blobs built directly in bf16 (no bench helper), padded for the kernels, and k centres on the device."""
    torch, _, _, KM, K = _env()
    cen = torch.randn(k, d, device="cuda", generator=g) * 4
    x = torch.empty((n, d), dtype=torch.bfloat16, device="cuda")
    for s in range(0, n, 1 << 22):
        m = min(1 << 22, n - s)
        x[s:s + m] = (cen[torch.randint(0, k, (m,), device="cuda", generator=g)] +
                      torch.randn(m, d, device="cuda", generator=g)).to(torch.bfloat16)
    x = KM.to_device_matrix(x, d)
    dp = x.shape[1]
    kp = -(-k // 32) * 32
    cb = torch.zeros((kp, dp), dtype=torch.bfloat16, device="cuda")
    cn = torch.zeros(kp, device="cuda")
    K.update_centers(None, k, d, cen.double().clone(), cb, dp, kp, cn, None)
    return x, dp, cb, cn


def cmd_modes(argv):
    torch, _, _, KM, K = _env()
    n, d, k = _arg(argv, 0, 20_000_000), _arg(argv, 1, 256), _arg(argv, 2, 256)
    g = torch.Generator(device="cuda").manual_seed(0)
    x, dp, cb, cn = _raw_problem(n, d, k, g)
    xn = torch.empty(n, device="cuda")
    c0 = cb[0].float().contiguous()
    cost = torch.empty(n, device="cuda")
    near = torch.empty(n, dtype=torch.int32, device="cuda")
    mx = torch.zeros(1, device="cuda")
    er = torch.tensor([2 ** 31 - 1, -1], dtype=torch.int32, device="cuda")
    t = wall_ms(lambda: K.row_pass(x, n, dp, xn))
    print(f"row pass (norms)            {t:8.3f} ms  {n * dp * 2 / t / 1e9:6.2f} TB/s")
    t = wall_ms(lambda: K.row_pass(x, n, dp, xn, c0, float(cn[0]), cost, near, xn_max=mx, erange=er))
    print(f"row pass (fused init)       {t:8.3f} ms  {n * dp * 2 / t / 1e9:6.2f} TB/s")
    plan = K.plan_assign(n, dp, k)
    lab = torch.zeros(n, dtype=torch.int32, device="cuda")
    cp = torch.zeros(plan.grid, dtype=torch.float64, device="cuda")
    hist = torch.zeros(plan.grid * plan.kp, dtype=torch.int32, device="cuda")
    rank = torch.zeros(n, dtype=torch.int32, device="cuda")
    t0 = wall_ms(lambda: K.assign_bf16(x, n, dp, cb, cn, plan, lab, None, cp, hist, rank, xnorm=xn))
    print(f"K9r mode 0 (+ranks)         {t0:8.3f} ms")
    ub = torch.zeros(n, device="cuda")
    lb = torch.zeros(n, device="cuda")
    mc = torch.tensor([float(cn[:k].max())], device="cuda")
    tau = KM.LloydEngine.prune_tau(dp)
    t1 = wall_ms(lambda: K.assign_rr_ext(1, x, n, dp, cb, cn, plan, xn, lab, cp, ub, lb, mc, tau, hist=hist,
                                         rank=rank))
    print(f"K9r mode 1 (top-2, +ranks)  {t1:8.3f} ms  ({100 * (t1 / t0 - 1):+.1f} %)")
    t1b = wall_ms(lambda: K.assign_rr_ext(1, x, n, dp, cb, cn, plan, xn, lab, cp, ub, lb, mc, tau))
    print(f"K9r mode 1 (top-2, no ranks){t1b:8.3f} ms")
    for frac in (0.02, 0.05, 0.2):
        m = int(n * frac)
        tr = plan.round_rows
        cand = torch.sort(torch.randperm(n, device="cuda", generator=g)[:m]).values.to(torch.int32)
        pad = -(-m // tr) * tr + tr
        idx = torch.zeros(pad, dtype=torch.int32, device="cuda")
        idx[:m] = cand
        cl = torch.zeros(pad, dtype=torch.int32, device="cuda")
        cl[:m] = lab[cand.long()]
        cx = torch.zeros(pad, device="cuda")
        cx[:m] = xn[cand.long()]
        cnt = torch.tensor([m], dtype=torch.int32, device="cuda")
        t2 = wall_ms(lambda: K.assign_rr_ext(2, x, m, dp, cb, cn, plan, cx, lab, cp, ub, lb, mc, tau, idx=idx,
                                             n_dev=cnt, lab_in=cl))
        print(f"K9r mode 2, {100 * frac:4.1f} % rows     {t2:8.3f} ms  ({m * dp * 2 / t2 / 1e9:5.2f} TB/s of candidate "
              f"rows; full-pass share {t2 / t0:.3f})")
    for kk in (64, 128, 192, 256, 320):  # centre tiles per wave: the k-means|| candidate chunk sizes
        kpk = -(-kk // 32) * 32
        cbk = torch.zeros((kpk, dp), dtype=torch.bfloat16, device="cuda")
        cnk = torch.zeros(kpk, device="cuda")
        K.update_centers(None, kk, d, torch.randn(kk, d, device="cuda", generator=g).double() * 4, cbk, dp, kpk, cnk,
                         None)
        pl = K.plan_assign(n, dp, kk)
        bst = torch.empty(n, device="cuda")
        t = wall_ms(lambda: K.assign_bf16(x, n, dp, cbk, cnk, pl, lab, bst, None, xnorm=xn))
        print(f"K9r mode 0, k={kk:3d} (CT={pl.rr_ct})     {t:8.3f} ms")


def cmd_pmc(argv):
    torch, _, _native, _, K = _env()
    v, n, d, k, bits = (_arg(argv, 0, 0), _arg(argv, 1, 20_000_000), _arg(argv, 2, 256), _arg(argv, 3, 256),
                        _arg(argv, 4, 0))
    K.set_assign_variant(v)
    if bits:
        _native.kernels().cml_kmeans_set_rr_debug(bits)
    eng, x0 = engine(n, d, k)
    torch.cuda.synchronize()
    for xx in (eng.x, x0):
        for _ in range(3):
            assign(eng, xx)
        torch.cuda.synchronize()
    print("done", flush=True)


def cmd_pmc_mode(argv):
    torch, _, _, KM, K = _env()
    n, d, k, mode = _arg(argv, 0, 20_000_000), _arg(argv, 1, 256), _arg(argv, 2, 256), _arg(argv, 3, 0)
    x, dp, cb, cn = _raw_problem(n, d, k, torch.Generator(device="cuda").manual_seed(0))
    xn = torch.empty(n, device="cuda")
    K.row_pass(x, n, dp, xn)
    plan = K.plan_assign(n, dp, k)
    lab = torch.zeros(n, dtype=torch.int32, device="cuda")
    cp = torch.zeros(plan.grid, dtype=torch.float64, device="cuda")
    best = torch.empty(n, device="cuda")
    ub = torch.zeros(n, device="cuda")
    lb = torch.zeros(n, device="cuda")
    mc = torch.tensor([float(cn[:k].max())], device="cuda")
    tau = KM.LloydEngine.prune_tau(dp)
    for _ in range(3):
        if mode == 0:
            K.assign_bf16(x, n, dp, cb, cn, plan, lab, best, cp, xnorm=xn)
        else:
            K.assign_rr_ext(1, x, n, dp, cb, cn, plan, xn, lab, cp, ub, lb, mc, tau)
    torch.cuda.synchronize()
    print("plan", plan, flush=True)


CLOCK_RUNS = ("rows from HBM", "rows from L2 ", "MFMA only    ", "no DMA       ")


def cmd_clock(argv):
    torch, _, _native, _, _ = _env()
    eng, x0 = engine(20_000_000, 256, 256)
    lib = _native.kernels()
    for xx, bits in ((eng.x, 0), (x0, 0), (eng.x, 5), (eng.x, 1)):  # the order of CLOCK_RUNS
        lib.cml_kmeans_set_rr_debug(bits)
        for _ in range(6):
            assign(eng, xx)
        torch.cuda.synchronize()
    lib.cml_kmeans_set_rr_debug(0)
    print("done", flush=True)


def cmd_clock_show(argv):
    rows = {}
    for f in sorted(glob.glob(os.path.join(argv[0], "**", "*counter_collection.csv"), recursive=True)):
        for r in csv.DictReader(open(f)):
            if "kmeans_assign_rr" not in r["Kernel_Name"]:
                continue
            d = rows.setdefault(int(r["Dispatch_Id"]), {})
            d["ns"] = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
            d[r["Counter_Name"]] = d.get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
    for i, did in enumerate(sorted(rows)):
        d = rows[did]
        ns = d["ns"]
        clk = d.get("GRBM_GUI_ACTIVE", 0.0) / 8 / ns  # GHz: the counter sums the 8 XCDs
        mf = d.get("SQ_VALU_MFMA_BUSY_CYCLES", 0.0) / 1024 / (clk * ns) if clk else 0.0
        src = CLOCK_RUNS[min(i // 6, len(CLOCK_RUNS) - 1)]
        print(f"dispatch {did:5d} {src}: {ns / 1e6:.3f} ms, clock {clk:.2f} GHz, MFMA busy {mf:.1%}, "
              f"SQ_BUSY_CYCLES {d.get('SQ_BUSY_CYCLES', 0):.3g}")


def cmd_ablate(argv):
    torch, _, _, _, K = _env()
    variants = [int(v) for v in argv] or [0, 1, 2, 3, 4, 5]
    for n, d, k in ((20_000_000, 256, 256), (20_000_000, 16, 5), (10_000_000, 128, 64)):
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
                best = torch.empty(n, device="cuda") if -(-kp // ap.kc) > 1 else None
                for xx, tag in ((x, "full"), (torch.as_strided(x, (n, dp), (0, 1)), "ldx0")):
                    if tag == "ldx0" and kk != k:
                        continue

                    def run():
                        K.assign_bf16(xx, n, dp, cb, cn, ap, lab, best, cost, xnorm=xn)
                    run()
                    t = min(event_ms(run))
                    print(f"n={n} d={d} k={kk} v{v} grid={ap.grid}x{ap.nwaves}w {tag:5s}: {t:.3f} ms "
                          f"{n * dp * 2 / t / 1e9:.2f} TB/s {2 * n * dp * kp / t / 1e9:.0f} TF/s", flush=True)
        K.set_assign_variant(0)
        del x, xn
        torch.cuda.empty_cache()


def cmd_sched(argv):
    torch, _, _, KM, K = _env()
    n = _arg(argv, 0, 20_000_000)
    scheds = [int(v) for v in argv[1].split(",")] if len(argv) > 1 else [0, 1, 18, 34, 66, 35, 0]
    eng, x0 = engine(n, 256, 256)
    eng.step()
    for sc in scheds:
        K.set_assign_sched(sc)
        assign(eng, eng.x)
        torch.cuda.synchronize()
        ts = sorted(event_ms(lambda: assign(eng, eng.x), 7))
        t = ts[3]
        print(f"sched {sc:3d}: median {t:.3f} ms (min {ts[0]:.3f}) -> {2 * n * 256 * 256 / t / 1e9:.0f} TF/s, "
              f"{n * 512 / t / 1e9:.2f} TB/s", flush=True)
    K.set_assign_sched(0)
    t = sorted(event_ms(lambda: assign(eng, x0), 7))[3]
    print(f"compute-only (ldx=0): median {t:.3f} ms -> {2 * n * 256 * 256 / t / 1e9:.0f} TF/s", flush=True)
    e32 = KM.LloydEngine(eng.x[:, :256], 256, 32, use_graph=False)
    e32.set_centers(eng.x[:32, :256].to(torch.float32).double().cpu().numpy())
    e32.step()

    def run32():
        K.assign_bf16(e32.x, n, e32.dp, e32.cb, e32.cnorm, e32.aplan, e32.labels, None, e32.cost_part, None, None,
                      xnorm=e32.xnorm)
    run32()
    t = sum(event_ms(run32)) / 5
    print(f"k=32 (memory-bound): {t:.3f} ms -> {n * 512 / t / 1e9:.2f} TB/s", flush=True)


COMMANDS = {"rr": cmd_rr, "dbg": cmd_dbg, "modes": cmd_modes, "pmc": cmd_pmc, "pmc-mode": cmd_pmc_mode,
            "clock": cmd_clock, "clock-show": cmd_clock_show, "ablate": cmd_ablate, "sched": cmd_sched}

if __name__ == "__main__":
    if len(sys.argv) < 2 or sys.argv[1] not in COMMANDS:
        print(__doc__)
        sys.exit(2)
    COMMANDS[sys.argv[1]](sys.argv[2:])
