"""Synthetic tables keyed by GLOBAL row index (the benchmarks' data; ``_native/csrc/synth.hip``).

The reference partitions ONE table across its executors (``ref.py:57``, ``ref.py:139``), and the
north star asks for the same metric at 1/2/4/8 GPUs, so a scaling curve must fit the same rows at
every rank count. Every value here is a pure function of (seed, global row, column): rank r of W
generating its row range writes exactly those rows of the one-rank table (on the GPU bit for bit;
the CPU twin below is W-invariant in the same way, with float64 Box-Muller instead of the kernel's
f32 math).
"""
from __future__ import annotations

from typing import Optional, Tuple

import torch

from . import rng


def shard_range(total: int, rank: int, world: int) -> Tuple[int, int]:
    """Rows [r0, r1) of rank ``rank`` when ``total`` rows are split in rank order, the first
    ``total % world`` ranks holding one extra row (the layout every bench and the engine's row ids assume)."""
    per, rem = divmod(int(total), int(world))
    r0 = rank * per + min(rank, rem)
    return r0, r0 + per + (1 if rank < rem else 0)


def _keys(seed: int, stream: int) -> Tuple[int, int]:
    return rng.key(seed, stream), rng.key(seed, stream + 7919)


def synth_rows(row0: int, n: int, d: int, seed: int, stream: int = 0, centres: Optional[torch.Tensor] = None,
               mode: str = "normal", dtype: torch.dtype = torch.float32, device=None, ld: Optional[int] = None,
               with_labels: bool = False, out: Optional[torch.Tensor] = None):
    """Rows row0 .. row0 + n - 1 of the table ``centres[label(row)] + noise(row, j)`` as an [n, ld] tensor
    (columns past d are zero). ``mode`` "normal": N(0, 1) noise; "uniform": U(-2, 2). ``centres``: [kt, d]
    (f32; None: no centre term). Returns the rows, or (rows, int32 labels) with ``with_labels``."""
    device = torch.device(device) if device is not None else (centres.device if centres is not None
                                                              else torch.device("cpu"))
    ld = d if ld is None else int(ld)
    if mode not in ("normal", "uniform"):
        raise ValueError(f"synth_rows: mode 'normal' or 'uniform', got {mode!r}")
    key, key_lab = _keys(seed, stream)
    kt = 0 if centres is None else int(centres.shape[0])
    if centres is not None:
        centres = centres.to(device=device, dtype=torch.float32).contiguous()
        if centres.shape[1] != d:
            raise ValueError(f"synth_rows: centres are [{kt}, {centres.shape[1]}], want [kt, {d}]")
    if out is None:
        out = torch.empty((max(n, 0), ld), dtype=dtype, device=device)
    lab = torch.empty(max(n, 0), dtype=torch.int32, device=device) if with_labels else None
    if with_labels and kt == 0:
        raise ValueError("synth_rows: labels need centres")
    if device.type == "cuda":
        from ..ops import frame_ops
        frame_ops.synth_rows(row0, n, d, ld, centres, kt, key, key_lab, 1 if mode == "uniform" else 0, out, lab)
    elif n > 0:
        _synth_rows_cpu(row0, n, d, ld, centres, kt, key, key_lab, mode, out, lab)
    return (out, lab) if with_labels else out


def _labels_cpu(rows: torch.Tensor, kt: int, key_lab: int) -> torch.Tensor:
    h = rng.splitmix64(rows ^ key_lab)
    return ((rng._lsr(h, 32) * kt) >> 32).to(torch.int64)


def _synth_rows_cpu(row0, n, d, ld, centres, kt, key, key_lab, mode, out, lab, chunk: int = 1 << 16) -> None:
    """Host twin of synth_rows_kernel (same hashes; float64 Box-Muller)."""
    cols = torch.arange(d, dtype=torch.int64)
    for s in range(0, n, chunk):
        m = min(chunk, n - s)
        rows = torch.arange(row0 + s, row0 + s + m, dtype=torch.int64)
        h = rng.splitmix64((rows[:, None] * d + cols[None, :]) ^ key)
        u1 = (rng._lsr(h, 40).to(torch.float64) + 1.0) * (1.0 / 16777216.0)
        u2 = (h & 0xFFFFFF).to(torch.float64) * (1.0 / 16777216.0)
        if mode == "uniform":
            z = 4.0 * u2 - 2.0
        else:
            z = torch.sqrt(-2.0 * torch.log(u1)) * torch.cos(6.283185307179586 * u2)
        if centres is not None or lab is not None:
            lb = _labels_cpu(rows, kt, key_lab)
            if lab is not None:
                lab[s:s + m] = lb.to(torch.int32)
            if centres is not None:
                z = z + centres[lb].to(torch.float64)
        blk = out[s:s + m]
        blk[:, :d] = z.to(out.dtype)
        if ld > d:
            blk[:, d:] = 0
