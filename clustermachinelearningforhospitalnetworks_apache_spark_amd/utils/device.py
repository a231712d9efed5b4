"""Device helpers: gfx950 properties, padding rules, dtype maps, host-latency guards."""
from __future__ import annotations

import contextlib
import functools
import gc
import os

import torch

LDS_BYTES = 160 * 1024          # LDS per CU on MI355X (MI355X_MICROARCH.md "Chip-level parameters")
LDS_BUDGET = 152 * 1024         # what one workgroup may claim, leaving slack for statics
MFMA_K = 16                     # k-step of v_mfma_f32_32x32x16_bf16
MFMA_TILE = 32                  # M/N of the 32x32 MFMA tile


def round_up(x: int, m: int) -> int:
    return (x + m - 1) // m * m


def next_pow2(x: int) -> int:
    p = 1
    while p < x:
        p <<= 1
    return p


def padded_dim(d: int) -> int:
    """Padded feature width used by the MFMA kernels: 16 * 2^j (16, 32, 64, 128, 256, 512)."""
    return max(16, MFMA_K * next_pow2((d + MFMA_K - 1) // MFMA_K))


@functools.lru_cache(None)
def num_cus(device_index: int = 0) -> int:
    if not torch.cuda.is_available():
        return 1
    return int(torch.cuda.get_device_properties(device_index).multi_processor_count)


def is_gpu(t: torch.Tensor) -> bool:
    return t.is_cuda


def gpu_available() -> bool:
    return torch.cuda.is_available() and os.environ.get("CML_FORCE_CPU") != "1"


@contextlib.contextmanager
def gc_paused():
    """Python's cyclic garbage collector off for the duration (Estimator.fit). A fit on a small shard is bound by
    the host's launch latency; a collection pass that lands between two launches idles the GPU for its whole
    duration. Reference counting still frees everything a fit allocates; the collector resumes (and catches
    up) when the fit returns. Nested fits (a Pipeline's stages) see it paused already. CML_GC_PAUSE=0: off."""
    if os.environ.get("CML_GC_PAUSE", "1") == "0" or not gc.isenabled():
        yield
        return
    gc.disable()
    try:
        yield
    finally:
        gc.enable()
