#!/usr/bin/env python3
"""Headline benchmark: KMeans fit samples/sec (whole job), BASELINE.json config
"KMeans k=256 on 100M×256, DP across MI355X with RCCL all-reduce of centroid sums".

The timed region is ONE WHOLE ``KMeans(k=256, maxIter=steps, tol=0, seed=42).fit(df)`` through the
public pyspark.ml-compatible Estimator API (ml/clustering.py; the reference's ``lr.fit(train_data)``
contract, ref.py:147) on a frame of this rank's HBM-resident shard (``createDataFrameFromTensors``) —
the metric SURVEY.md §6 / BASELINE.md define (samples/s = N_rows x Lloyd iterations / fit wall time):
engine construction (device layout + row norms), k-means|| initialisation (initSteps=2, as Spark's
KMeans.fit runs it), ``steps`` Lloyd iterations and the model + summary (trainingCost; clusterSizes is
lazy, as Spark's). A step = one distributed Lloyd iteration: exact bound-pruned K9r MFMA assign, K10
incremental f64 sums, RCCL all-reduce of the [k·D sums | k counts | cost] message, K11 update.
--warmup runs an untimed warm-up fit of that many iterations first. The same fit driven on the
LloydEngine directly, the steady-state step and a forced full step are reported in extra (not the
headline), and with --data blobs (the headline) also a fit on overlapping blobs (extra.overlap), where
the bounds prune little. The dataset is ONE fixed table (100M rows total) sharded over the N ranks in
row order, so scaling is *strong*: every value is generated from its global row index (utils/synth.py),
and the fit is partition-invariant, so N = 1, 2, 4, 8 fit the same problem and report the same
trainingCost bits and cluster sizes (extra.training_cost_hex / cluster_sizes_digest). Data: synthetic
Gaussian blobs generated on the GPU, bf16 features (no network).

Usage (driver contract):
    python bench.py --gpus 1 --steps 20 --warmup 3
    python -m torch.distributed.run --nnodes=1 --nproc-per-node N --master-addr 127.0.0.1 \
        --master-port P bench.py --gpus N --steps K --warmup W
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import torch

from clustermachinelearningforhospitalnetworks_apache_spark_amd.models.kmeans import LloydEngine
from clustermachinelearningforhospitalnetworks_apache_spark_amd.parallel.comm import Communicator
from clustermachinelearningforhospitalnetworks_apache_spark_amd.utils.synth import shard_range

METRIC = "KMeans fit samples/sec (whole node), 100M×256 k=256 at 1/2/4/8 MI355X"
BASELINE_VALUE = None  # the reference publishes no number

# --data: centre spread of the Gaussian blobs (unit noise); "uniform" has no cluster structure
_DATA = {"blobs": 4.0, "overlap": 0.5, "uniform": None}


def make_blobs(n: int, d: int, k_true: int, seed: int, device, dtype=torch.bfloat16, spread=4.0, row0: int = 0):
    """Rows row0 .. row0 + n - 1 of ONE fixed table of k_true Gaussian blobs (centres N(0, spread²), unit noise;
    U(-2, 2) rows when spread is None). Every value is a pure function of (seed, global row, column)
    (utils/synth.py, synth.hip), so rank r of W generating its shard writes exactly those rows of the W = 1
    table: the 1/2/4/8-GPU runs fit the same 100M rows."""
    from clustermachinelearningforhospitalnetworks_apache_spark_amd.utils import synth
    centers = None
    if spread is not None:  # rows 0 .. k_true - 1 of the centre table: identical on every rank
        centers = synth.synth_rows(0, k_true, d, seed=1234, stream=1, device=device) * spread
    gdt = dtype if dtype in (torch.bfloat16, torch.float32) or not torch.device(device).type == "cuda" else torch.float32
    x = synth.synth_rows(row0, n, d, seed=seed, stream=0, centres=centers,
                         mode="uniform" if spread is None else "normal", dtype=gdt, device=device)
    return x if x.dtype == dtype else x.to(dtype)


def _col_dot(z: torch.Tensor, w: torch.Tensor) -> torch.Tensor:
    """z @ w in f64, accumulated column by column (elementwise ops: each row's bits do not depend on how many
    rows the chunk holds, unlike a GEMV whose reduction tiling follows the shape)."""
    acc = torch.zeros(z.shape[0], dtype=torch.float64, device=z.device)
    for j, wj in enumerate(w.to(torch.float64).cpu().tolist()):
        acc.add_(z[:, j].to(torch.float64), alpha=wj)
    return acc


_T0 = time.time()
try:  # the phase log counts from the process start (import torch included)
    import psutil
    _T0 = psutil.Process().create_time()
except Exception:  # noqa: BLE001
    pass


def _digest(sizes) -> str:
    """Short digest of a cluster-size list (the labels histogram; equal across rank counts for one problem)."""
    import hashlib
    return hashlib.sha256(",".join(str(int(v)) for v in sizes).encode()).hexdigest()[:16]


def _phase(comm, what: str) -> None:
    """Timestamped phase line on rank 0's stderr (where a run's wall time goes: VERDICT r5 weak 9)."""
    if comm is None or comm.rank == 0:
        print(f"[bench +{time.time() - _T0:7.2f}s] {what}", file=sys.stderr, flush=True)


def _drop_norm_cache(x: torch.Tensor) -> None:
    """The engine caches ||x||² on the feature tensor (Spark's VectorWithNorm); a timed fit must
    compute them itself, so the cache of an earlier fit on the same tensor is dropped."""
    if hasattr(x, "_cml_xnorm"):
        del x._cml_xnorm


def kmeans_fit(x, args, comm, seed: int = 42, iters: int = 20, breakdown: bool = False):
    """One whole KMeans fit on the LloydEngine directly (what ``KMeans.fit`` drives): engine
    construction (device layout, row norms), k-means|| init (initSteps=2) and ``iters`` Lloyd
    iterations. Returns (engine, init seconds, per-iteration seconds or None)."""
    gpu = x.is_cuda
    eng = LloydEngine(x, args.dim, args.k, comm, row_chunks=args.chunks,
                      incremental=not args.full_accumulate, prune=args.prune, precision=args.precision)
    eng.track_prune = breakdown
    init = (eng.init_kmeans_parallel(seed=seed, as_device=True) if args.init == "k-means||"
            else eng.init_random(seed=seed))
    eng.set_centers(init)
    if gpu and breakdown:
        torch.cuda.synchronize()
    t_init = time.perf_counter()
    per = [] if breakdown else None
    for _ in range(iters):
        t = time.perf_counter()
        eng.step()
        if breakdown:
            if gpu:
                torch.cuda.synchronize()
            per.append(time.perf_counter() - t)
    return eng, t_init, per


def api_fit(df, args, seed: int, iters: int):
    """The public Estimator fit: ``KMeans(k, maxIter=iters, tol, seed).fit(df)``."""
    from clustermachinelearningforhospitalnetworks_apache_spark_amd.ml.clustering import KMeans
    km = KMeans(k=args.k, maxIter=iters, tol=args.tol, seed=seed, initMode=args.init,
                featuresCol="features")
    return km.fit(df)


def _timed(comm, gpu, fn):
    """Run fn bracketed by barrier + device sync on both sides; (result, max seconds over ranks)."""
    comm.barrier()
    if gpu:
        torch.cuda.synchronize()
    t0 = time.perf_counter()
    out = fn()
    if gpu:
        torch.cuda.synchronize()
    comm.barrier()
    return out, comm.max_scalar(time.perf_counter() - t0)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20, help="Lloyd iterations of the timed fit (maxIter)")
    ap.add_argument("--warmup", type=int, default=3, help="Lloyd iterations of the untimed warm-up fit")
    ap.add_argument("--rows", type=int, default=100_000_000, help="total rows (strong scaling)")
    ap.add_argument("--dim", type=int, default=256)
    ap.add_argument("--k", type=int, default=256)
    ap.add_argument("--tol", type=float, default=0.0, help="KMeans tol of the timed fit (headline: 0)")
    ap.add_argument("--data", default="blobs", choices=sorted(_DATA),
                    help="blobs = the headline data (separated blobs); overlap = blob centres 8x closer; "
                         "uniform = no cluster structure")
    ap.add_argument("--no-overlap", action="store_true", help="skip the extra overlap-data fit")
    ap.add_argument("--dtype", default="bf16", choices=["bf16", "f32", "f64"],
                    help="feature dtype of the frame (f32/f64: the reference's Double/Integer columns, fitted at "
                         "source precision by default)")
    ap.add_argument("--precision", default=None, choices=["auto", "bf16", "exact", "screen"],
                    help="cml.ml.kmeans.precision of the session (default: auto)")
    ap.add_argument("--init", default="k-means||", choices=["k-means||", "random"])
    ap.add_argument("--chunks", type=int, default=None, help="row chunks per rank (comm/compute overlap)")
    ap.add_argument("--prune", default=None, choices=["on", "off"],
                    help="engine measurements: force the exact bound-pruned Lloyd step on or off")
    ap.add_argument("--full-accumulate", action="store_true",
                    help="engine measurements: re-accumulate every row each step instead of the exact incremental sums")
    ap.add_argument("--breakdown", action="store_true",
                    help="also run one engine fit with a device sync after every iteration and report per-iteration "
                         "times (extra.breakdown); the headline fit is never synchronised inside")
    ap.add_argument("--workload", default="kmeans", choices=["kmeans", "logreg", "pipeline", "csv", "kmeans_ooc"],
                    help="kmeans = the BASELINE headline; logreg = BASELINE config 4 (StandardScaler + "
                         "LogisticRegression, 100M x 256), one step = one distributed gradient pass + L-BFGS update; "
                         "pipeline = BASELINE config 5 (VectorAssembler -> StandardScaler(fp8) -> KMeans -> "
                         "LogisticRegression, 125M x 512 per GPU = 1B x 512 at 8 GPUs), one step = one Pipeline.fit; "
                         "csv = BASELINE config 1 (1k x 16 synthetic CSV -> VectorAssembler -> KMeans k=5 on local[2] "
                         "CPU, plumbing), one step = read + assemble + fit")
    ap.add_argument("--rows-per-gpu", type=int, default=125_000_000, help="pipeline workload (weak scaling)")
    ap.add_argument("--ooc-rows", type=int, default=250_000_000,
                    help="kmeans_ooc workload: fp8 rows (x 512) kept in pinned host memory")
    ap.add_argument("--solver", default="lbfgs", choices=["lbfgs", "sgd"],
                    help="logreg workload: Spark's L-BFGS (full-batch passes) or data-parallel mini-batch SGD")
    ap.add_argument("--batch", type=int, default=1 << 20, help="logreg SGD rows per rank per step")
    args = ap.parse_args()
    args.prune = None if args.prune is None else args.prune == "on"
    if args.workload == "logreg":
        return bench_logreg(args)
    if args.workload == "pipeline":
        return bench_pipeline(args)
    if args.workload == "csv":
        return bench_csv(args)
    if args.workload == "kmeans_ooc":
        return bench_kmeans_ooc(args)

    from clustermachinelearningforhospitalnetworks_apache_spark_amd.sql import SparkSession
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if world != args.gpus and world != 1:
        print(f"warning: --gpus {args.gpus} but WORLD_SIZE={world}", file=sys.stderr)
    gpu = torch.cuda.is_available()
    if not gpu:
        # CPU plumbing run only (no MI355X here): shrink so it finishes.
        args.rows, args.dim, args.k = min(args.rows, 200_000), min(args.dim, 32), min(args.k, 16)
    spark = (SparkSession.builder.appName("bench-kmeans").master("mi355x" if gpu else "local[1]")
             .config("cml.ml.features.dtype", "bf16" if gpu else "float64").getOrCreate())
    if args.precision:
        spark.conf.set("cml.ml.kmeans.precision", args.precision)
    fdt = {"bf16": torch.bfloat16, "f32": torch.float32, "f64": torch.float64}[args.dtype] if gpu else torch.float64
    comm = spark._comm
    rank, W = comm.rank, comm.world_size
    dev = comm.device

    # this rank's rows of the ONE fixed table: [r0, r1) of args.rows, generated by global row index, so every N
    # fits the same problem (strong scaling; the fit is partition-invariant bit for bit: tests/test_bench_invariance)
    r0, r1 = shard_range(args.rows, rank, W)
    n_local = r1 - r0
    _phase(comm, f"session up (rank 0 of {W}); generating rows [{r0}, {r1})")
    t0 = time.perf_counter()
    x = make_blobs(n_local, args.dim, args.k, seed=1000, device=dev, dtype=fdt, spread=_DATA[args.data], row0=r0)
    if gpu:
        torch.cuda.synchronize()
    gen_s = time.perf_counter() - t0
    df = spark.createDataFrameFromTensors({"features": x})

    # untimed warm-up fit: code objects, allocator pools, RCCL channels (its results are discarded)
    _phase(comm, f"data ready ({gen_s:.2f} s); warm-up fit")
    if args.warmup > 0:
        api_fit(df, args, seed=7, iters=args.warmup)
        _drop_norm_cache(x)

    # the timed region: one whole public-API fit from scratch, bracketed by barrier + device sync
    _phase(comm, "timed fit")
    model, elapsed = _timed(comm, gpu, lambda: api_fit(df, args, seed=42, iters=args.steps))
    _phase(comm, f"timed fit done ({1000 * elapsed:.1f} ms); engine / step measurements")
    summ = model.summary
    sizes = summ.clusterSizes
    acc = {"api": f"KMeans(k={args.k}, maxIter={args.steps}, tol={args.tol:g}, seed=42).fit(df)",
           "iterations": summ.numIter, "training_cost": summ.trainingCost,
           "training_cost_hex": float(summ.trainingCost).hex(), "cluster_sizes_digest": _digest(sizes),
           "cluster_sizes_minmax": [min(sizes), max(sizes)]}
    del model, summ
    _drop_norm_cache(x)

    # the same fit on the engine directly (no Estimator layer), then its steady-state and full steps
    (eng, t_init), eng_s = _timed(comm, gpu, lambda: kmeans_fit(x, args, comm, seed=42, iters=args.steps)[:2])
    acc["engine_fit_ms"] = round(1000.0 * eng_s, 3)
    acc["api_over_engine"] = round(elapsed / eng_s, 4) if eng_s > 0 else None
    acc["accumulate"] = "incremental (exact)" if eng.delta is not None else "full"
    acc["assign"] = "pruned (exact bounds)" if eng.prune else "full (every row x every centre)"
    if eng.prune:
        acc["last_step_prune_rank0"] = eng.prune_stats()
    acc["precision"] = eng.precision
    if gpu and eng.gpu:
        acc.update(_step_rates(eng, comm))
    del eng
    _drop_norm_cache(x)
    if args.breakdown:
        comm.barrier()
        tb = time.perf_counter()
        eng, tbi, per_it = kmeans_fit(x, args, comm, seed=42, iters=args.steps, breakdown=True)
        acc["breakdown"] = {"init_ms": round(1000.0 * (tbi - tb), 3),
                            "iteration_ms": [round(1000.0 * t, 3) for t in per_it]}
        if eng.prune:
            acc["breakdown"]["prune_history_rank0"] = eng.prune_history()
        if getattr(eng, "_scr", None) is not None:  # precision "screen": screened rows re-checked in f64,
            # then per certified step (rows the bounds no longer proved, rows re-assigned exactly, moves)
            acc["breakdown"]["screen_rechecked_rank0"] = list(eng._scr.rechecked)
            cert = getattr(eng._scr, "cert", None)
            acc["breakdown"]["certified_steps_rank0"] = list(cert.history) if cert is not None else None
        # pruned k-means|| rounds: (rows, rows with a few relevant candidates, rows sent to the K9r pass)
        acc["breakdown"]["init_pruned_rounds_rank0"] = getattr(eng, "_init_prune_history", None)
        del eng
        _drop_norm_cache(x)

    if gpu and args.data == "blobs" and args.dtype == "bf16" and not args.no_overlap:
        # the same public-API fit on overlapping blobs (centres 8x closer), where the exact bounds prune
        # little: the robustness of the headline. Same shape, separate data.
        del df
        _phase(comm, "overlap-data fits")
        x2 = make_blobs(n_local, args.dim, args.k, seed=2000, device=dev, spread=_DATA["overlap"], row0=r0)
        df2 = spark.createDataFrameFromTensors({"features": x2})
        api_fit(df2, args, seed=7, iters=max(1, args.warmup))
        _drop_norm_cache(x2)
        m2, el2 = _timed(comm, gpu, lambda: api_fit(df2, args, seed=42, iters=args.steps))
        ov = {"fit_ms": round(1000.0 * el2, 3), "samples_per_s": args.rows * args.steps / el2,
              "iterations": m2.summary.numIter, "training_cost_hex": float(m2.summary.trainingCost).hex(),
              "cluster_sizes_digest": _digest(m2.summary.clusterSizes)}
        del m2
        _drop_norm_cache(x2)
        e2, _, _ = kmeans_fit(x2, args, comm, seed=42, iters=args.steps)
        ov.update(_step_rates(e2, comm))
        del e2, df2, x2
        acc["overlap"] = ov

    total_rows = args.rows
    value = total_rows * args.steps / elapsed
    headline = (args.rows, args.dim, args.k, args.data, args.dtype) == (100_000_000, 256, 256, "blobs", "bf16")
    metric = METRIC if headline else (f"KMeans fit samples/sec (whole node), {args.rows / 1e6:g}M×{args.dim} "
                                      f"k={args.k}" + ("" if args.data == "blobs" else f", {args.data} data") +
                                      ("" if args.dtype == "bf16" else f", {args.dtype} rows"))
    if rank == 0:
        out = {
            "metric": metric,
            "value": value,
            "unit": "samples/s",
            "n_gpus": W if gpu else 0,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": 1000.0 * elapsed / args.steps,
            "higher_is_better": True,
            "scaling": "strong",
            "vs_baseline": (value / BASELINE_VALUE) if BASELINE_VALUE else None,
            "dtype": (args.dtype if args.dtype != "f32" else "fp32") if gpu else "fp64",
            "data": f"synthetic ({args.data}: generated on device; centres from k-means|| init inside the timed fit)",
            "config": {
                "model": f"KMeans k={args.k}, {args.rows}x{args.dim}",
                "global_batch": total_rows,
                "seq_len": None,
                "parallelism": f"dp{W}",
                "k": args.k, "rows": total_rows, "dim": args.dim,
                "timed": f"whole public-API fit: KMeans(k={args.k}, maxIter={args.steps}, tol={args.tol:g}).fit(df) "
                         "= engine + norms, k-means|| init, Lloyd iterations, model + summary",
            },
            "extra": {"fit_s": round(elapsed, 4), "datagen_s": round(gen_s, 3),
                      "device": torch.cuda.get_device_name(dev) if gpu else "cpu", **acc},
        }
        print(json.dumps(out), flush=True)
    _phase(comm, "done")
    spark.stop()


def _step_rates(eng, comm) -> dict:
    """Steady-state step time of a fitted engine (5 more pruned steps), a forced full-assign step (bounds
    invalid: K9r over every row with top-2 bounds; the sums move by the changed rows as in every step
    whose labels barely move — what a fit on data the bounds cannot prune runs each iteration), and a
    forced from-scratch step (also the full counting-sort f64 accumulate: a fit's first step)."""
    out = {}
    comm.barrier()
    torch.cuda.synchronize()
    ts = time.perf_counter()
    for _ in range(5):
        eng.step()
    torch.cuda.synchronize()
    comm.barrier()
    out["steady_state_ms_per_step"] = 1000.0 * comm.max_scalar(time.perf_counter() - ts) / 5
    if eng._pdev:
        comm.barrier()
        torch.cuda.synchronize()
        ts = time.perf_counter()
        for _ in range(3):
            eng._pst.force.fill_(1)
            eng.step()
        torch.cuda.synchronize()
        comm.barrier()
        out["full_step_ms"] = 1000.0 * comm.max_scalar(time.perf_counter() - ts) / 3
        comm.barrier()
        torch.cuda.synchronize()
        ts = time.perf_counter()
        for _ in range(3):
            eng._pst.force.fill_(1)
            eng.delta.invalidate()
            eng.step()
        torch.cuda.synchronize()
        comm.barrier()
        out["full_step_from_scratch_ms"] = 1000.0 * comm.max_scalar(time.perf_counter() - ts) / 3
    if eng.delta is not None and not eng.prune:
        out["last_step_changed_rows_rank0"] = eng.delta.changed_rows()
        comm.barrier()
        torch.cuda.synchronize()
        ts = time.perf_counter()
        for _ in range(3):
            eng.delta.invalidate()
            eng.step()
        torch.cuda.synchronize()
        comm.barrier()
        out["full_accumulate_ms_per_step"] = 1000.0 * comm.max_scalar(time.perf_counter() - ts) / 3
    return out


def bench_logreg(args):
    """BASELINE.json config 4: standardized binomial LogisticRegression on 100M x 256 bf16.

    Untimed: data generation, the StandardScaler moments pass (K7 + all-reduce). Timed: `steps`
    L-BFGS iterations of the Spark objective (standardization inside the gradient, as Spark
    does), each = >= 1 full K13 gradient pass over every row + RCCL all-reduce + host update.
    Reported value = rows x gradient passes / s.
    """
    import numpy as np
    from clustermachinelearningforhospitalnetworks_apache_spark_amd.models.optim import lbfgs
    from clustermachinelearningforhospitalnetworks_apache_spark_amd.ops import glm_ops
    gpu = torch.cuda.is_available()
    if not gpu:
        args.rows, args.dim = min(args.rows, 200_000), min(args.dim, 32)
    comm = Communicator.from_env(want_gpu=gpu)
    rank, W = comm.rank, comm.world_size
    dev = comm.device
    # this rank's rows [r0, r1) of one fixed 100M-row table, generated by global row index (utils/synth.py)
    r0, r1 = shard_range(args.rows, rank, W)
    n = r1 - r0
    d = args.dim
    t0 = time.perf_counter()
    from clustermachinelearningforhospitalnetworks_apache_spark_amd.utils import synth
    gp = synth.synth_rows(0, 2, d, seed=99, stream=1, device=dev, mode="uniform")  # global parameters
    w_true = gp[0] * (0.5 * 3 ** 0.5 / d ** 0.5)  # U(-2, 2)·sqrt(3)/2: unit variance, / sqrt(d)
    scale = (gp[1] + 2.0) * 0.75 + 0.5  # U(0.5, 3.5)
    dt = torch.bfloat16 if gpu else torch.float64
    x = torch.empty((n, d), dtype=dt, device=dev)
    y = torch.empty(n, dtype=torch.float64, device=dev)
    for s0 in range(0, n, 1 << 22):
        m = min(1 << 22, n - s0)
        z = synth.synth_rows(r0 + s0, m, d, seed=2000, stream=0, device=dev)
        e = synth.synth_rows(r0 + s0, m, 1, seed=2000, stream=2, device=dev)[:, 0]
        x[s0:s0 + m] = (z * scale).to(dt)
        logit = _col_dot(z, w_true) + 0.3 * e.to(torch.float64)
        y[s0:s0 + m] = (logit > 0).to(torch.float64)
        del z, e
    if gpu:
        torch.cuda.synchronize()
    gen_s = time.perf_counter() - t0
    t0 = time.perf_counter()
    cnt, s1, s2, shift = glm_ops.moments(x, d)
    msg = torch.cat([torch.tensor([float(cnt)], dtype=torch.float64, device=dev), s1 + cnt * shift,
                     s2 + 2 * shift * s1 + cnt * shift * shift])
    comm.allreduce_(msg)
    N = msg[0].item()
    mean = msg[1:1 + d] / N
    std = torch.sqrt(torch.clamp((msg[1 + d:] - N * mean * mean) / max(N - 1, 1), min=0)).cpu().numpy()
    sd = np.where(std > 0, std, 1.0)
    scaler_s = time.perf_counter() - t0
    evals = [0]

    def fg(p):
        coef = np.r_[p[:d] / sd, p[d]]
        out = glm_ops.logreg_grad(x, d, y, torch.as_tensor(coef, device=dev))
        comm.allreduce_(out)
        o = out.cpu().numpy()
        evals[0] += 1
        ws = max(o[d + 2], 1e-300)
        grad = np.r_[o[:d] / sd, o[d]] / ws
        return o[d + 1] / ws, grad

    if args.solver == "sgd":
        # data-parallel mini-batch SGD with momentum: per step one K13 pass over `batch` rows per
        # rank, one RCCL all-reduce of the [d+3] gradient message, device-side update (no host sync)
        from clustermachinelearningforhospitalnetworks_apache_spark_amd.models.sgd import LogisticSGD
        bs = min(args.batch, n)
        opt = LogisticSGD(x, d, y, None, comm, bs, lr=0.5, momentum=0.9,
                          scale=torch.as_tensor(1.0 / sd, device=dev))

        def sgd_step(i):
            opt.step()
            return opt.loss_acc

        for i in range(args.warmup):
            sgd_step(i)
        comm.barrier()
        if gpu:
            torch.cuda.synchronize()
        t0 = time.perf_counter()
        for i in range(args.steps):
            loss = sgd_step(args.warmup + i)
        if gpu:
            torch.cuda.synchronize()
        comm.barrier()
        elapsed = comm.max_scalar(time.perf_counter() - t0)
        if rank == 0:
            rows = bs * W * args.steps
            print(json.dumps({
                "metric": f"LogisticRegression mini-batch SGD rows/sec (whole node), StandardScaler-standardized "
                          f"{args.rows}x{d}",
                "value": rows / elapsed, "unit": "rows/s", "n_gpus": W if gpu else 0, "steps": args.steps,
                "warmup": args.warmup, "ms_per_step": 1000.0 * elapsed / args.steps, "higher_is_better": True,
                "scaling": "strong", "vs_baseline": None, "dtype": "bf16" if gpu else "fp64",
                "data": "synthetic (Gaussian features, logistic labels)",
                "config": {"model": f"LogisticRegression d={d} SGD(momentum 0.9)", "global_batch": bs * W,
                           "seq_len": None, "parallelism": f"dp{W}"},
                "extra": {"mean_loss": float(loss.item()) / max(opt.steps, 1), "hip_graph": opt.use_graph}}),
                flush=True)
        comm.shutdown()
        return
    p0 = np.zeros(d + 1)
    if args.warmup:
        p0, _, _ = lbfgs(fg, p0, args.warmup, 0.0)
    comm.barrier()
    if gpu:
        torch.cuda.synchronize()
    evals[0] = 0
    t0 = time.perf_counter()
    p, hist, iters = lbfgs(fg, p0, args.steps, 0.0)
    if gpu:
        torch.cuda.synchronize()
    comm.barrier()
    elapsed = comm.max_scalar(time.perf_counter() - t0)
    passes = evals[0]
    value = args.rows * passes / elapsed
    if rank == 0:
        print(json.dumps({
            "metric": "LogisticRegression fit rows/sec per gradient pass (whole node), StandardScaler-standardized "
                      f"{args.rows}x{d}",
            "value": value, "unit": "rows/s", "n_gpus": W if gpu else 0, "steps": iters, "warmup": args.warmup,
            "ms_per_step": 1000.0 * elapsed / max(iters, 1), "ms_per_gradient_pass": 1000.0 * elapsed / max(passes, 1),
            "gradient_passes": passes, "higher_is_better": True, "scaling": "strong", "vs_baseline": None,
            "dtype": (args.dtype if args.dtype != "f32" else "fp32") if gpu else "fp64", "data": "synthetic (Gaussian features, logistic labels)",
            "config": {"model": f"LogisticRegression d={d}", "global_batch": args.rows, "seq_len": None,
                       "parallelism": f"dp{W}"},
            "extra": {"datagen_s": round(gen_s, 3), "scaler_s": round(scaler_s, 3), "final_loss": hist[-1] if hist
                      else None}}), flush=True)
    comm.shutdown()


def bench_kmeans_ooc(args):
    """Out-of-core KMeans (SURVEY §5.7, config 5's row scale on ONE GPU): 250M x 512 e4m3 rows = 128 GB
    live in pinned host memory (more than the HBM budget the pipeline leaves) and every pass over X
    streams them through two device buffers (utils/hoststream.py). Timed: one whole fit (k-means|| init,
    ``--steps`` Lloyd iterations, k = 128, tol = 0). Reports rows·iterations/s like the headline, the
    streamed bytes, and the copy engine's H2D rate of one pass with no kernels attached."""
    gpu = torch.cuda.is_available()
    n, d, k = args.ooc_rows, 512, 128
    if not gpu:
        n = min(n, 50_000)
    dev = torch.device("cuda", 0) if gpu else torch.device("cpu")
    t0 = time.perf_counter()
    xh = torch.empty((n, d), dtype=torch.uint8, pin_memory=gpu)
    g = torch.Generator(device=dev)
    g.manual_seed(7)
    cen = torch.randn((64, d), generator=g, device=dev) * 3
    step = 1 << 22
    for s0 in range(0, n, step):
        m = min(step, n - s0)
        z = cen[torch.randint(0, 64, (m,), generator=g, device=dev)] + torch.randn((m, d), generator=g, device=dev)
        xh[s0:s0 + m].copy_(z.clamp_(-440.0, 440.0).to(torch.float8_e4m3fn).view(torch.uint8))
        del z
    x8 = xh.view(torch.float8_e4m3fn)
    gen_s = time.perf_counter() - t0
    if not gpu:
        x8 = x8.to(torch.float32)
    mk = (lambda rows: LloydEngine(rows, d, k, device=dev)) if gpu else (lambda rows: LloydEngine(rows, d, k))
    # untimed warm-up on a slice (code objects, pinned staging buffers)
    w = mk(x8[: min(n, 1 << 20)])
    w.set_centers(w.init_kmeans_parallel(seed=3))
    w.step()
    del w
    if gpu:
        torch.cuda.synchronize()
    t0 = time.perf_counter()
    eng = mk(x8)
    eng.set_centers(eng.init_kmeans_parallel(seed=42))
    t_init = time.perf_counter()
    for _ in range(args.steps):
        eng.step()
    if gpu:
        torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    extra = {"fit_s": round(elapsed, 3), "init_s": round(t_init - t0, 3), "datagen_s": round(gen_s, 2),
             "training_cost": eng.training_cost(), "host_bytes": n * d}
    if gpu and eng._hs is not None:
        hs = eng._hs
        extra["streamed_GB"] = round(hs.bytes / 1e9, 2)
        extra["passes_over_x"] = hs.passes
        extra["streamed_GB_per_s_in_fit"] = round(hs.bytes / 1e9 / elapsed, 2)
        for _ in hs.chunks(eng.bounds, timed=True):
            pass
        extra["h2d_GB_per_s_copy_only"] = round(hs.last_h2d_gbps() or 0.0, 2)
        extra["chunk_rows"] = hs.chunk_rows
    print(json.dumps({
        "metric": f"Out-of-core KMeans fit samples/sec, {n / 1e6:g}M x {d} fp8 in pinned host memory, k={k}",
        "value": n * args.steps / elapsed, "unit": "samples/s", "n_gpus": 1 if gpu else 0, "steps": args.steps,
        "warmup": 1, "ms_per_step": 1000.0 * elapsed / args.steps, "higher_is_better": True, "scaling": "weak",
        "vs_baseline": None, "dtype": _fp8_dtype("fp8 rows (e4m3fn)"), "data": "synthetic Gaussian blobs",
        "config": {"model": f"KMeans k={k}", "global_batch": n, "seq_len": None, "parallelism": "dp1 (streamed)",
                   "rows": n, "dim": d}, "extra": extra}), flush=True)


def _fp8_dtype(what: str) -> str:
    """dtype field of the fp8 workloads: the MFMA the KMeans passes ran (kmeans_ops.set_fp8_mx)."""
    from clustermachinelearningforhospitalnetworks_apache_spark_amd.ops import kmeans_ops as K
    return f"{what}, " + ("MX-scaled fp8 MFMA in the KMeans assign" if K.fp8_mx_on() else "bf16 MFMA")


def bench_pipeline(args):
    """BASELINE.json config 5 through the public API: a sharded frame of HBM-resident bf16 raw
    features -> Pipeline(VectorAssembler, StandardScaler(withMean, outputDtype=fp8),
    KMeans(k=128, 10 Lloyd iterations after k-means||), LogisticRegression(10 L-BFGS iterations)).
    Timed: whole Pipeline.fit calls (every stage's fit and the intermediate transforms)."""
    from clustermachinelearningforhospitalnetworks_apache_spark_amd.ml.classification import LogisticRegression
    from clustermachinelearningforhospitalnetworks_apache_spark_amd.ml.clustering import KMeans
    from clustermachinelearningforhospitalnetworks_apache_spark_amd.ml.feature import StandardScaler, VectorAssembler
    from clustermachinelearningforhospitalnetworks_apache_spark_amd.ml.pipeline import Pipeline
    from clustermachinelearningforhospitalnetworks_apache_spark_amd.sql import SparkSession
    gpu = torch.cuda.is_available()
    n, d = args.rows_per_gpu, (args.dim if args.dim != 256 else 512)
    if not gpu:
        n, d = min(n, 100_000), min(d, 64)
    spark = (SparkSession.builder.appName("bench-pipeline").master("mi355x" if gpu else "local[4]")
             .config("cml.ml.features.dtype", "bf16" if gpu else "float64").getOrCreate())
    comm = spark._comm
    rank, W = comm.rank, comm.world_size
    dev = spark._device
    t0 = time.perf_counter()
    # weak scaling: rank r holds global rows [r·n, (r + 1)·n) of one table generated by global row index
    # (utils/synth.py): the rows of the N-GPU run are the first N·n rows of one fixed dataset
    from clustermachinelearningforhospitalnetworks_apache_spark_amd.utils import synth
    centers = synth.synth_rows(0, 32, d, seed=7, stream=1, device=dev) * 3
    gp = synth.synth_rows(0, 3, d, seed=7, stream=2, device=dev)
    spread = (synth.synth_rows(3, 1, d, seed=7, stream=2, device=dev, mode="uniform")[0] + 2.0) + 0.25  # U(.25, 4.25)
    offset = gp[0] * 10
    w_true = gp[1] / d ** 0.5
    raw = torch.empty((n, d), dtype=torch.bfloat16 if gpu else torch.float64, device=dev)
    y = torch.empty(n, dtype=torch.float64, device=dev)
    for s0 in range(0, n, 1 << 22):
        m = min(1 << 22, n - s0)
        z = synth.synth_rows(rank * n + s0, m, d, seed=5000, stream=0, centres=centers, device=dev)
        raw[s0:s0 + m] = (z * spread + offset).to(raw.dtype)
        y[s0:s0 + m] = (_col_dot(z, w_true) > 0).to(torch.float64)
        del z
    df = spark.createDataFrameFromTensors({"raw": raw, "label": y})
    del raw, y
    if gpu:
        torch.cuda.synchronize()
    gen_s = time.perf_counter() - t0
    pipe = Pipeline(stages=[
        VectorAssembler(inputCols=["raw"], outputCol="assembled"),
        StandardScaler(inputCol="assembled", outputCol="features", withMean=True,
                       outputDtype="fp8" if gpu else "float64"),
        KMeans(k=128, maxIter=10, tol=0.0, seed=11, predictionCol="cluster"),
        LogisticRegression(maxIter=10, tol=0.0),
    ])
    for _ in range(args.warmup):
        pipe.fit(df)
    comm.barrier()
    if gpu:
        torch.cuda.synchronize()
    from clustermachinelearningforhospitalnetworks_apache_spark_amd.utils.trace import TRACER
    TRACER.reset()  # the CML_TRACE report covers the timed fits only
    t0 = time.perf_counter()
    model = None
    for _ in range(args.steps):
        model = None  # release the previous fit's transformed columns (its summaries hold them) first
        model = pipe.fit(df)
    if gpu:
        torch.cuda.synchronize()
    comm.barrier()
    elapsed = comm.max_scalar(time.perf_counter() - t0)
    total = n * W
    if rank == 0:
        km, lr = model.stages[2], model.stages[3]
        print(json.dumps({
            "metric": f"Pipeline fit rows/sec (whole node), VectorAssembler->StandardScaler(fp8)->KMeans->LogReg, "
                      f"{total / 1e9:g}B x {d}",
            "value": total * args.steps / elapsed, "unit": "rows/s", "n_gpus": W if gpu else 0, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": 1000.0 * elapsed / args.steps, "higher_is_better": True,
            "scaling": "weak", "vs_baseline": None, "dtype": _fp8_dtype("fp8 features (e4m3fn)") if gpu else "fp64",
            "data": "synthetic (Gaussian blobs, logistic labels), generated on device",
            "config": {"model": "Pipeline[VectorAssembler, StandardScaler, KMeans k=128 x10, LogReg x10]",
                       "global_batch": total, "seq_len": None, "parallelism": f"dp{W}", "rows_per_gpu": n, "dim": d},
            "extra": {"datagen_s": round(gen_s, 3), "kmeans_iters": km.summary.numIter,
                      "kmeans_cost": km.summary.trainingCost, "logreg_iters": lr.summary.totalIterations}}),
              flush=True)
        if os.environ.get("CML_TRACE") == "1":
            print(TRACER.report(), file=sys.stderr, flush=True)
    spark.stop()


def bench_csv(args):
    """BASELINE.json config 1 ("KMeans k=5 on 1k x 16 synthetic CSV via local[2] CPU, plumbing"):
    spark.read.csv (native C++ tokenizer/parser, K1) -> VectorAssembler -> KMeans(k=5).fit, on the
    CPU session (no GPU). One step = the whole read + assemble + fit. The fitted centres are checked
    against a numpy Lloyd run from the same initial centres (extra.max_center_err)."""
    import tempfile

    import numpy as np

    from clustermachinelearningforhospitalnetworks_apache_spark_amd.ml.clustering import KMeans
    from clustermachinelearningforhospitalnetworks_apache_spark_amd.ml.feature import VectorAssembler
    from clustermachinelearningforhospitalnetworks_apache_spark_amd.sql import SparkSession
    os.environ["CML_FORCE_CPU"] = "1"
    n, d, k = 1000, 16, 5
    rs = np.random.RandomState(0)
    cent = rs.randn(k, d) * 5
    x = cent[rs.randint(0, k, n)] + rs.randn(n, d)
    tmp = tempfile.mkdtemp(prefix="cml_csv_bench_")
    cols = [f"f{i}" for i in range(d)]
    with open(os.path.join(tmp, "part-0.csv"), "w") as fh:
        fh.write(",".join(cols) + "\n")
        for row in x:
            fh.write(",".join(repr(float(v)) for v in row) + "\n")
    spark = SparkSession.builder.appName("bench-csv").master("local[2]").getOrCreate()

    def one():
        df = spark.read.option("header", True).option("inferSchema", True).csv(tmp)
        feats = VectorAssembler(inputCols=cols, outputCol="features").transform(df)
        return KMeans(k=k, seed=1, maxIter=20, initMode="random").fit(feats)

    for _ in range(args.warmup):
        one()
    t0 = time.perf_counter()
    model = None
    for _ in range(args.steps):
        model = one()
    elapsed = time.perf_counter() - t0
    # numpy Lloyd oracle from the same data: converged centres must agree (same partition)
    got = np.stack(model.clusterCenters())
    c = got.copy()
    for _ in range(50):
        lab = ((x[:, None, :] - c[None]) ** 2).sum(-1).argmin(1)
        c = np.stack([x[lab == j].mean(0) if (lab == j).any() else c[j] for j in range(k)])
    err = float(np.abs(c - got).max())
    print(json.dumps({
        "metric": "KMeans fit samples/sec, 1k x 16 CSV k=5 via local[2] CPU (read + assemble + fit)",
        "value": n * model.summary.numIter * args.steps / elapsed, "unit": "samples/s", "n_gpus": 0,
        "steps": args.steps, "warmup": args.warmup, "ms_per_step": 1000.0 * elapsed / args.steps,
        "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "fp64",
        "data": "synthetic (Gaussian blobs written to CSV)",
        "config": {"model": "KMeans k=5", "global_batch": n, "seq_len": None, "parallelism": "local[2]", "dim": d},
        "extra": {"kmeans_iters": model.summary.numIter, "training_cost": model.summary.trainingCost,
                  "max_center_err_vs_numpy_lloyd": err}}), flush=True)
    spark.stop()
    import shutil
    shutil.rmtree(tmp, ignore_errors=True)


if __name__ == "__main__":
    main()
