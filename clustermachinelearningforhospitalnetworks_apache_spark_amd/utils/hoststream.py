"""Out-of-core rows: a feature matrix kept in pinned host memory and streamed to the GPU in fixed-size
row chunks (SURVEY §5.7 — a shard larger than the HBM budget, e.g. config 5's 1B x 512 fp8 on fewer
than 2 GPUs).

Two device buffers alternate: while the kernels of chunk c read buffer c % 2, the copy stream fills
buffer (c + 1) % 2 with the next chunk (hipMemcpyAsync from pinned memory, DMA engines, no CU time).
The copy into a buffer waits for the event the compute stream records after the last kernel that
reads the buffer's previous chunk, and the compute stream waits for the copy's ready event — so one
pass over X costs max(H2D, compute) per chunk, and the H2D link (not HBM) is the bound for the
distance/accumulate passes whose HBM time is ~1/100 of the copy's.

The passes that consume the chunks are the resident ones, unchanged (K12 row pass, K9r assign, K10
sort-regime sums, k-means|| candidate merges): every per-row result is written to the slice r0:r1 of
the device-resident per-row state (norms, labels, costs), and the per-chunk f64 partial sums are exact,
so a streamed fit equals the resident fit bit for bit.

Reference: rows are the reference's scaling axis (``ref.py:75-115`` generates them, ``ref.py:123-128``
assembles and caches them in executor memory; Spark spills cached partitions that do not fit).
"""
from __future__ import annotations

import math
from typing import Iterator, List, Optional, Tuple

import torch


def hbm_budget_bytes(device: torch.device, conf_value=None) -> int:
    """``cml.hbm.budgetBytes`` (session conf or CML_HBM_BUDGET_BYTES), default 85% of the device's
    memory: a feature matrix larger than this stays in host memory and is streamed."""
    import os
    v = conf_value if conf_value is not None else os.environ.get("CML_HBM_BUDGET_BYTES")
    if v is not None and str(v) != "":
        return int(float(v))
    if device.type != "cuda" or not torch.cuda.is_available():
        return 1 << 62
    return int(0.85 * torch.cuda.get_device_properties(device).total_memory)


def pinned_rows(x: torch.Tensor) -> torch.Tensor:
    """``x`` (host) in page-locked memory (copied once unless already pinned)."""
    if x.is_cuda:
        raise ValueError("pinned_rows takes a host tensor")
    if not torch.cuda.is_available() or x.is_pinned():
        return x
    return x.pin_memory()


def cached_stream(xh: torch.Tensor, chunk_rows: int, device: torch.device) -> "HostRowStream":
    """One HostRowStream (two device chunk buffers + copy stream) per pinned matrix, chunk size and
    device, kept on the matrix: repeated fits / transforms of an out-of-core column reuse its buffers
    instead of allocating 2 x ~1 GiB of HBM per call."""
    key = (str(device), int(chunk_rows))
    cache = getattr(xh, "_cml_streams", None)
    if cache is None:
        cache = {}
        try:
            xh._cml_streams = cache
        except (AttributeError, RuntimeError):
            pass
    hs = cache.get(key)
    if hs is None or hs.xh is not xh:
        hs = HostRowStream(xh, chunk_rows, device)
        cache[key] = hs
    return hs


class HostRowStream:
    """Double-buffered H2D streaming of a pinned host matrix [n, dp] in row chunks."""

    def __init__(self, xh: torch.Tensor, chunk_rows: int, device: torch.device):
        if xh.is_cuda or xh.dim() != 2:
            raise ValueError("HostRowStream takes a 2-D host matrix")
        self.xh = xh
        self.n, self.dp = int(xh.shape[0]), int(xh.shape[1])
        self.device = device
        self.chunk_rows = max(1, int(chunk_rows))
        rows = min(self.chunk_rows, max(self.n, 1))
        self.buf = [torch.empty((rows, self.dp), dtype=xh.dtype, device=device) for _ in range(2)]
        self.copy_stream = torch.cuda.Stream(device=device)
        self.ready = [torch.cuda.Event() for _ in range(2)]
        self.free = [torch.cuda.Event() for _ in range(2)]
        self.passes = 0
        self.bytes = 0
        self._t0: Optional[torch.cuda.Event] = None
        self._t1: Optional[torch.cuda.Event] = None
        self.h2d_ms = 0.0  # copy-stream time of the last timed pass (first copy start -> last copy end)

    @staticmethod
    def chunk_bounds(n: int, chunk_rows: int, align: int = 32) -> List[int]:
        """Row boundaries of the chunks: every chunk but the last a multiple of ``align`` rows."""
        step = max(align, (max(1, int(chunk_rows)) // align) * align)
        nch = max(1, math.ceil(n / step))
        return [min(n, i * step) for i in range(nch)] + [n]

    def chunks(self, bounds: List[int], timed: bool = False) -> Iterator[Tuple[int, int, int, torch.Tensor]]:
        """Yield (chunk, r0, r1, device rows) for consecutive chunks; the caller enqueues the chunk's
        kernels on the current stream before asking for the next one."""
        cur = torch.cuda.current_stream(self.device)
        nch = len(bounds) - 1
        if timed:
            self._t0, self._t1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)

        def issue(i: int) -> None:
            b = i % 2
            r0, r1 = bounds[i], bounds[i + 1]
            with torch.cuda.stream(self.copy_stream):
                self.copy_stream.wait_event(self.free[b])  # chunk i - 2's kernels are done with buffer b
                if timed and i == 0:
                    self._t0.record(self.copy_stream)
                if r1 > r0:
                    self.buf[b][: r1 - r0].copy_(self.xh[r0:r1], non_blocking=True)
                    self.bytes += (r1 - r0) * self.dp * self.xh.element_size()
                self.ready[b].record(self.copy_stream)
                if timed and i == nch - 1:
                    self._t1.record(self.copy_stream)

        # every copy is ordered after the work already queued on the compute stream (buffers of a
        # previous pass may still be read by it)
        self.copy_stream.wait_stream(cur)
        issue(0)
        for i in range(nch):
            if i + 1 < nch:
                issue(i + 1)
            b = i % 2
            cur.wait_event(self.ready[b])
            r0, r1 = bounds[i], bounds[i + 1]
            yield i, r0, r1, self.buf[b][: r1 - r0]
            self.free[b].record(cur)
        self.passes += 1

    def last_h2d_gbps(self) -> Optional[float]:
        """GB/s of the last timed pass's copies (synchronises on its last copy)."""
        if self._t0 is None or self._t1 is None:
            return None
        self._t1.synchronize()
        ms = self._t0.elapsed_time(self._t1)
        self.h2d_ms = ms
        nbytes = self.n * self.dp * self.xh.element_size()
        return nbytes / (ms * 1e-3) / 1e9 if ms > 0 else None
