"""Device warm-up at GPU session start (session conf ``cml.session.warmup``, default on; ``cml.session.poolBytes``).

The first call of every path pays one-time costs that have nothing to do with its data: the caching
allocator's first hipMalloc of each size class, the first launch of each kernel of the in-tree library
and of torch's, library handles. The reference workflow's per-batch retrain (``ref.py:91-106``: na.drop,
VectorAssembler, LinearRegression per micro-batch) ran 95 ms of na.drop and 20 ms of fit cold against
5 ms and 0.5 ms warm on 4M rows (profiles/r4/per_batch_retrain_4M_rows.log) — a streaming job pays that
on its first batch. The session therefore (1) reserves one allocator segment (freed at once, so the
caching allocator keeps it and splits later requests from it) and (2) runs the frame / GLM / evaluator
kernels a micro-batch runs once on a few rows, so a session's first batch runs at its warm rate. A
Spark executor warms its JVM the same way before the first task.
"""
from __future__ import annotations

import time

import numpy as np
import torch


def warm_device(device: torch.device, pool_bytes: int = 1 << 30) -> float:
    """Warm ``device``; returns the seconds it took (0 on a CPU device)."""
    if device.type != "cuda":
        return 0.0
    t0 = time.perf_counter()
    if pool_bytes > 0:
        blk = torch.empty(int(pool_bytes), dtype=torch.uint8, device=device)
        del blk
    from ..ops import frame_ops, glm_ops
    n, d = 4096, 4
    # host-generated data: a device randn would load torch's distribution kernels (~160 ms on first use)
    # for a warm-up whose jobs draw their random numbers from the in-tree counter-based generator
    x = torch.from_numpy(np.random.default_rng(0).standard_normal((n, d))).to(device)
    xi = (x[:, 0] * 100).to(torch.int32)
    valid = x[:, 1] > -3.0
    y = x @ torch.ones(d, dtype=torch.float64, device=device)
    # na.drop / filter: validity + NaN masks, compaction, row gathers
    good = valid.to(torch.int32) + (~torch.isnan(x[:, 2])).to(torch.int32)
    keep = good == 2
    bool(keep.all())
    idx = frame_ops.compact(keep)
    for t in (x[:, 0], xi, valid, x):
        t[idx]
    # every column dtype a frame holds (numbers, dictionary string codes, masks): its null test, the
    # int32 tally, and the row gather of the compaction
    for dt in (torch.float32, torch.float64, torch.int8, torch.int16, torch.int32, torch.int64, torch.uint8,
               torch.bool, torch.bfloat16):
        t = x[:, 3].to(dt)
        if t.is_floating_point():
            (~torch.isnan(t)).to(torch.int32)
        (t != 0).to(torch.int32)
        t[idx]
        t[keep]
    # VectorAssembler (K2) and the GLM / evaluator kernels of a per-batch fit
    m, bad = frame_ops.assemble([(x[:, j], None) for j in range(d)] + [(xi, valid)], out_dtype=torch.float64)
    bool(bad.any())
    glm_ops.gram(m, d + 1, y, None)
    glm_ops.moments(m, d + 1)
    glm_ops.linear_predict(m, d + 1, torch.zeros(d + 2, dtype=torch.float64, device=device), "identity")
    frame_ops.reg_metric_sums(y, y * 0.5)
    torch.sort(xi, stable=True)
    torch.unique(xi)
    torch.cuda.synchronize(device)
    return time.perf_counter() - t0


def warm_frames(session) -> float:
    """Run the reference micro-batch's frame path once on a tiny frame of every column kind the CSV
    reader produces (dictionary strings with a null, integers with nulls, doubles with NaN, timestamps):
    na.drop, a timestamp BETWEEN filter, VectorAssembler and a LinearRegression fit. The kernels' first
    launches (each loads its code object) then happen here and not inside a stream's first batch
    (na.drop ran 12-23 ms cold vs 2-5 ms warm on 4M rows: profiles/r4/dropna_cold_trace.log).
    Tracing is paused so warm-up ranges never show in a job's report."""
    from ..sql import types as T
    from ..sql.column import ColumnData, DictColumnData
    from ..sql.dataframe import DataFrame
    from .trace import TRACER
    dev = session._device
    if dev.type != "cuda":
        return 0.0
    t0 = time.perf_counter()
    was = TRACER.enabled
    TRACER.disable()
    try:
        n = 64
        ar = torch.arange(n, device=dev)
        schema = T.StructType([T.StructField("h", T.StringType()), T.StructField("t", T.TimestampType()),
                               T.StructField("a", T.IntegerType()), T.StructField("s", T.DoubleType()),
                               T.StructField("y", T.DoubleType())])
        codes = (np.arange(n) % 3).astype(np.int32)
        codes[5] = -1
        valid_a = torch.ones(n, dtype=torch.bool, device=dev)
        valid_a[7] = False
        sv = ar.to(torch.float64) * 0.5
        sv[9] = float("nan")
        cols = {"h": DictColumnData(codes, np.array(["x", "y", "z", None], dtype=object), None, T.StringType()),
                "t": ColumnData(ar.to(torch.int64) * 1_000_000 + 1_700_000_000_000_000, None, T.TimestampType()),
                "a": ColumnData(ar.to(torch.int32), valid_a, T.IntegerType()),
                "s": ColumnData(sv, None, T.DoubleType()),
                "y": ColumnData(ar.to(torch.float64), None, T.DoubleType())}
        df = DataFrame(session, schema, cols, n, ar.to(torch.int64), dev)
        clean = df.na.drop()
        df.filter("t BETWEEN '2023-11-14 22:13:20' AND '2023-11-14 22:14:00'").count()
        from ..ml.feature import VectorAssembler
        from ..ml.regression import LinearRegression
        data = VectorAssembler(inputCols=["a", "s"], outputCol="features").transform(clean)
        LinearRegression(featuresCol="features", labelCol="y").fit(data).summary.rootMeanSquaredError
        torch.cuda.synchronize(dev)
    finally:
        if was:
            TRACER.enable(TRACER.sync)
    return time.perf_counter() - t0
