"""Counter-based random numbers keyed by (seed, stream, global row id).

Spark draws per-partition XORShift sequences, so a row's random value depends on
how the data is partitioned (``ref.py:139``).  Here every random
decision about a row is a pure hash of (seed, stream, row id): results are
identical on 1, 2, 4 or 8 GPUs and on the CPU (the same int64 torch ops run on
both devices, wrap-around multiplication included).
"""
from __future__ import annotations

import torch

_M31 = (1 << 31) - 1
_M53 = (1 << 53) - 1


def _s64(c: int) -> int:
    c &= (1 << 64) - 1
    return c - (1 << 64) if c >= (1 << 63) else c


_C1 = _s64(0xBF58476D1CE4E5B9)
_C2 = _s64(0x94D049BB133111EB)
_GOLD = _s64(0x9E3779B97F4A7C15)


def _lsr(x: torch.Tensor, s: int) -> torch.Tensor:
    """Logical shift right of int64 (torch's >> is arithmetic)."""
    return (x >> s) & ((1 << (64 - s)) - 1)


def splitmix64(x: torch.Tensor) -> torch.Tensor:
    x = x + _GOLD
    x = (x ^ _lsr(x, 30)) * _C1
    x = (x ^ _lsr(x, 27)) * _C2
    return x ^ _lsr(x, 31)


def _splitmix64_int(x: int) -> int:
    """splitmix64 of one value in Python integers (mod 2^64): the bits of ``splitmix64`` without torch ops
    (a key is derived on every launch path; the tensor form cost ~8 host ops per key)."""
    m = (1 << 64) - 1
    x = (x + 0x9E3779B97F4A7C15) & m
    x = ((x ^ (x >> 30)) * 0xBF58476D1CE4E5B9) & m
    x = ((x ^ (x >> 27)) * 0x94D049BB133111EB) & m
    return _s64(x ^ (x >> 31))


def key(seed: int, stream: int = 0) -> int:
    return _splitmix64_int(_s64(seed * 0x100000001B3 + stream * 0xC2B2AE3D27D4EB4F) & ((1 << 64) - 1))


def uniform(row_ids: torch.Tensor, seed: int, stream: int = 0) -> torch.Tensor:
    """u in [0, 1) (float64) for every row id (device tensors: one fused HIP kernel, K5)."""
    if row_ids.is_cuda:
        from ..ops import frame_ops
        return frame_ops.counter_uniform(row_ids, key(seed, stream))
    h = splitmix64(row_ids.to(torch.int64) ^ key(seed, stream))
    return _lsr(h, 11).to(torch.float64) * (1.0 / (1 << 53))


def poisson_thresholds(max_k: int = 16) -> list:
    """CDF of Poisson(1) at 0..max_k-1, accumulated in float64 in a fixed order (shared by the
    CPU path and the K22 kernel, so both invert the same thresholds)."""
    p = torch.exp(torch.tensor(-1.0, dtype=torch.float64)).item()
    cdf = p
    out = []
    for kk in range(1, max_k + 1):
        out.append(cdf)
        p = p / kk
        cdf += p
    return out


def poisson1(row_ids: torch.Tensor, seed: int, stream: int = 0, max_k: int = 16,
             dtype: torch.dtype = torch.int32) -> torch.Tensor:
    """Poisson(λ=1) counts per row by CDF inversion of one counter-based uniform."""
    th = poisson_thresholds(max_k)
    if row_ids.is_cuda:
        from ..ops import frame_ops
        return frame_ops.poisson1(row_ids, key(seed, stream), th, out_dtype=dtype)
    u = uniform(row_ids, seed, stream)
    out = torch.zeros_like(u, dtype=torch.int32)
    for t in th:
        out += (u >= t).to(torch.int32)
    return out.to(dtype)
