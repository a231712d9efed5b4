"""CPU comparison point named by BASELINE.md ("a CPU numpy implementation of the same algorithm on
the same data"): one Lloyd iteration (f32 distance GEMM via BLAS + argmin + per-cluster sums) on
a row subset, reported as samples/s (per-row cost is independent of the row count)."""
import json
import os
import sys
import time

import numpy as np


def lloyd_step(x, c):
    xn = np.einsum("ij,ij->i", x, x)
    cn = np.einsum("ij,ij->i", c, c)
    best = np.full(x.shape[0], np.inf, dtype=np.float32)
    lab = np.zeros(x.shape[0], dtype=np.int64)
    for s in range(0, x.shape[0], 65536):
        d = xn[s:s + 65536, None] - 2.0 * (x[s:s + 65536] @ c.T) + cn[None, :]
        lab[s:s + 65536] = d.argmin(1)
        best[s:s + 65536] = d.min(1)
    sums = np.zeros((c.shape[0], x.shape[1]), dtype=np.float64)
    np.add.at(sums, lab, x.astype(np.float64))
    counts = np.bincount(lab, minlength=c.shape[0])
    return sums, counts, float(best.sum())


def main():
    n, d, k = (int(a) for a in (sys.argv[1:4] if len(sys.argv) >= 4 else (1_000_000, 256, 256)))
    rs = np.random.RandomState(0)
    cen = rs.randn(k, d).astype(np.float32) * 4
    x = (cen[rs.randint(0, k, n)] + rs.randn(n, d).astype(np.float32)).astype(np.float32)
    c = x[:k].copy()
    lloyd_step(x[:100000], c)
    t0 = time.perf_counter()
    reps = 3
    for _ in range(reps):
        lloyd_step(x, c)
    dt = (time.perf_counter() - t0) / reps
    print(json.dumps({"metric": "CPU numpy Lloyd iteration samples/s", "value": n / dt, "rows": n, "dim": d, "k": k,
                      "ms_per_step": dt * 1e3, "cpus": os.cpu_count(), "dtype": "fp32 (numpy/BLAS)",
                      "extrapolated_100M_step_s": dt * 100_000_000 / n}))


if __name__ == "__main__":
    main()
