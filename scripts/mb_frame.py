"""Bandwidth of the frame kernels (K2 assemble, K3 compact, K5 split / counter uniform, K22 Poisson,
K6 binarize, K23 metric sums / confusion, K7 moments, K8 scale, K4 absmax / fp8 quantise) on one
MI355X, against the torch expression of the same op. Bytes are the kernel's compulsory HBM traffic
(inputs read once, outputs written once); the ceiling is ~8 TB/s.

    python scripts/mb_frame.py [--rows 100000000] [--reps 10]
"""
import argparse
import json
import sys

import torch

sys.path.insert(0, ".")
from clustermachinelearningforhospitalnetworks_apache_spark_amd.ops import frame_ops, glm_ops  # noqa: E402


def timed(fn, reps):
    fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(reps):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / reps


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=100_000_000)
    ap.add_argument("--reps", type=int, default=10)
    args = ap.parse_args()
    n, reps = args.rows, args.reps
    dev = torch.device("cuda")
    g = torch.Generator(device=dev).manual_seed(0)
    out = []

    def rec(name, ms, nbytes, torch_ms=None):
        r = {"kernel": name, "ms": round(ms, 4), "GB": round(nbytes / 1e9, 3), "TB_s": round(nbytes / ms / 1e9, 3)}
        if torch_ms is not None:
            r["torch_ms"] = round(torch_ms, 4)
            r["speedup_vs_torch"] = round(torch_ms / ms, 2)
        out.append(r)
        print(json.dumps(r), flush=True)

    # K2 assemble: the reference's 4 feature columns (3 int32 + 1 float64) -> [n, 4] float64
    c1 = torch.randint(0, 100, (n,), device=dev, dtype=torch.int32, generator=g)
    c2 = torch.randint(0, 500, (n,), device=dev, dtype=torch.int32, generator=g)
    c3 = torch.randint(0, 50, (n,), device=dev, dtype=torch.int32, generator=g)
    c4 = torch.rand(n, device=dev, dtype=torch.float64, generator=g)
    parts = [(c1, None), (c2, None), (c3, None), (c4, None)]
    ms = timed(lambda: frame_ops.assemble(parts), reps)
    tms = timed(lambda: torch.stack([c1.double(), c2.double(), c3.double(), c4], 1), reps)
    rec("K2 assemble 3xi32+f64 -> [n,4] f64", ms, n * (12 + 8 + 32 + 1), tms)
    del c1, c2, c3

    # K3 compact (half the rows kept)
    mask = torch.rand(n, device=dev, generator=g) < 0.5
    kept = int(mask.sum())
    ms = timed(lambda: frame_ops.compact(mask), reps)
    tms = timed(lambda: torch.nonzero(mask).flatten(), reps)
    rec("K3 compact 50% of n", ms, n + 8 * kept, tms)
    del mask

    # K5 counter-based uniform / split buckets, K22 Poisson(1) weights
    rows = torch.arange(n, device=dev, dtype=torch.int64)
    ms = timed(lambda: frame_ops.counter_uniform(rows, 12345), reps)
    rec("K5 counter_uniform", ms, n * 16)
    ms = timed(lambda: frame_ops.split_buckets(rows, 12345, [0.0, 0.7, 1.0]), reps)
    rec("K5 split_buckets 70/30", ms, n * 9)
    ms = timed(lambda: frame_ops.poisson1(rows, 12345, [0.36787944117144233, 0.7357588823428847,
                                                          0.9196986029286058, 0.9810118431238462], torch.int32), reps)
    rec("K22 poisson1 -> int32", ms, n * 12)
    del rows

    # K6 binarize, K23 metric sums
    ms = timed(lambda: frame_ops.binarize(c4, 0.5), reps)
    tms = timed(lambda: (c4 > 0.5).to(torch.float64), reps)
    rec("K6 binarize f64", ms, n * 16, tms)
    p = torch.rand(n, device=dev, dtype=torch.float64, generator=g)
    ms = timed(lambda: frame_ops.reg_metric_sums(c4, p), reps)
    tms = timed(lambda: torch.stack([((c4 - p) ** 2).sum(), (c4 - p).abs().sum(), c4.sum(), (c4 * c4).sum(),
                                     p.sum(), (p * p).sum()]), reps)
    rec("K23 reg_metric_sums", ms, n * 16, tms)
    yl = (c4 > 0.5).to(torch.int64)
    pl = (p > 0.5).to(torch.int64)
    ms = timed(lambda: frame_ops.confusion(yl, pl, 2), reps)
    rec("K23 confusion 2x2 (int64 labels)", ms, n * 16)
    del p, yl, pl, c4

    # K7 moments, K8 scale, K4 absmax / fp8 quantise on [m, 256] bf16
    m = n // 4
    X = torch.randn((m, 256), device=dev, dtype=torch.bfloat16, generator=g)
    ms = timed(lambda: glm_ops.moments(X, 256), reps)
    tms = timed(lambda: (X.float().mean(0), X.float().var(0)), reps)
    rec(f"K7 moments [{m},256] bf16", ms, m * 512, tms)
    mean = torch.zeros(256, device=dev, dtype=torch.float64)
    inv = torch.ones(256, device=dev, dtype=torch.float64)
    ms = timed(lambda: glm_ops.scale_apply(X, 256, mean, inv, True, out_dtype=torch.bfloat16), reps)
    rec(f"K8 scale_apply [{m},256] bf16 -> bf16", ms, m * 1024)
    ms = timed(lambda: frame_ops.col_absmax(X, 256), reps)
    tms = timed(lambda: X.abs().amax(0), reps)
    rec(f"K4 col_absmax [{m},256] bf16", ms, m * 512, tms)
    sc = torch.ones(256, device=dev, dtype=torch.float32)
    ms = timed(lambda: frame_ops.quant_fp8(X, 256, sc), reps)
    tms = timed(lambda: (X.float() * sc).to(torch.float8_e4m3fn), reps)
    rec(f"K4 quant_fp8 [{m},256] bf16 -> e4m3", ms, m * 768, tms)
    print(json.dumps({"rows": n, "results": out}))


if __name__ == "__main__":
    main()
