"""Host wrappers of the columnar-frame kernels (``_native/csrc/frame.hip``: K2 assemble, K3 compact,
K5 split buckets, K22 Poisson weights, K6 binarize, K23 metric reductions, K4 fp8 quantisation).

Every function takes device tensors and runs the HIP kernel; the CPU code paths of the frame
and the estimators keep their torch implementations (they are the numerics oracles of the GPU
tests).  Calling one of these on a CPU tensor is a programming error and raises.
"""
from __future__ import annotations

from typing import List, Optional, Sequence, Tuple

import numpy as np
import torch

from .. import _native
from .._native import c_int, c_ll, c_vp

c_double = __import__("ctypes").c_double
c_ull = __import__("ctypes").c_ulonglong

_native.register_kernel_sigs({
    "cml_split_buckets": (c_int, [c_vp, c_ll, c_ull, c_vp, c_int, c_vp, c_vp]),
    "cml_poisson1": (c_int, [c_vp, c_ll, c_ull, c_vp, c_int, c_vp, c_vp, c_vp]),
    "cml_counter_uniform": (c_int, [c_vp, c_ll, c_ull, c_vp, c_vp]),
    "cml_compact_blocks": (c_ll, [c_ll]),
    "cml_compact": (c_int, [c_vp, c_ll, c_vp, c_vp, c_vp, c_vp]),
    "cml_assemble": (c_int, [c_vp, c_int, c_ll, c_vp, c_int, c_ll, c_int, c_vp, c_int, c_int, c_vp]),
    "cml_assemble_col_bytes": (c_int, []),
    "cml_binarize": (c_int, [c_vp, c_int, c_ll, c_double, c_vp, c_vp]),
    "cml_metric_grid": (c_int, [c_ll]),
    "cml_reg_metrics": (c_int, [c_vp, c_vp, c_vp, c_ll, c_vp, c_int, c_vp]),
    "cml_cls_confusion": (c_int, [c_vp, c_vp, c_vp, c_ll, c_int, c_vp, c_int, c_vp]),
    "cml_col_absmax": (c_int, [c_vp, c_int, c_ll, c_int, c_ll, c_int, c_vp, c_vp]),
    "cml_quant_fp8": (c_int, [c_vp, c_int, c_ll, c_int, c_ll, c_vp, c_vp, c_ll, c_vp]),
    "cml_has_nan": (c_int, [c_vp, c_ll, c_int, c_ll, c_int, c_vp, c_vp]),
    "cml_synth_rows": (c_int, [c_ll, c_ll, c_int, c_ll, c_vp, c_int, c_ull, c_ull, c_int, c_vp, c_int, c_vp, c_vp]),
})


def has_nan(x: torch.Tensor, d: Optional[int] = None, stream=None) -> bool:
    """Any NaN in x[:, :d] (one streaming pass; bf16/f32/f64 with 16-B aligned rows)."""
    _dev(x, "has_nan")
    d = x.shape[1] if d is None else d
    if x.dtype not in (torch.bfloat16, torch.float32, torch.float64) or x.stride(1) != 1 \
            or (x.stride(0) * x.element_size()) % 16 or x.data_ptr() % 16:
        return bool(torch.isnan(x[:, :d]).any().item()) if x.is_floating_point() else False
    flag = torch.zeros(1, dtype=torch.int32, device=x.device)
    _native.check(_native.kernels().cml_has_nan(x.data_ptr(), x.shape[0], d, x.stride(0) * x.element_size(),
                                                x.element_size(), flag.data_ptr(), _st(stream)), "has_nan")
    return bool(flag.item())

_SRC_TYPES = {torch.float64: 0, torch.float32: 1, torch.int32: 2, torch.int64: 3, torch.uint8: 4,
              torch.bool: 4, torch.int16: 5, torch.bfloat16: 6, torch.int8: 7}
_OUT_TYPES = {torch.float64: 0, torch.float32: 1, torch.bfloat16: 2}


def _dev(t: torch.Tensor, what: str) -> None:
    if not t.is_cuda:
        raise RuntimeError(f"{what}: frame kernels run on the GPU only (got a {t.device} tensor)")


def _u64(k: int) -> int:
    return k & ((1 << 64) - 1)


def _st(stream) -> int:
    return _native.stream_ptr(stream)


# ------------------------------------------------------------------------------ synthetic rows
def synth_rows(row0: int, n: int, d: int, ld: int, centres: Optional[torch.Tensor], kt: int, key: int, key_lab: int,
               mode: int, out: torch.Tensor, labels: Optional[torch.Tensor] = None, stream=None) -> None:
    """out[i, :d] = centres[label(row0 + i)] + noise(row0 + i, j), zeros past d (synth.hip; utils/synth.py)."""
    _dev(out, "synth_rows")
    if out.dtype not in (torch.bfloat16, torch.float32) or not out.is_contiguous() or out.shape[0] < n \
            or out.shape[1] != ld or out.data_ptr() % 16:
        raise ValueError("synth_rows: a contiguous 16-byte aligned [n, ld] bf16 / f32 output")
    if centres is not None and (centres.dtype != torch.float32 or not centres.is_contiguous()
                                or tuple(centres.shape) != (kt, d)):
        raise ValueError("synth_rows: centres must be contiguous f32 [kt, d]")
    if labels is not None and (labels.dtype != torch.int32 or labels.numel() < n):
        raise ValueError("synth_rows: int32 labels [n]")
    _native.check(_native.kernels().cml_synth_rows(
        int(row0), int(n), int(d), int(ld), _native.ptr(centres), int(kt), _u64(key), _u64(key_lab), int(mode),
        out.data_ptr(), 0 if out.dtype == torch.bfloat16 else 1, _native.ptr(labels), _st(stream)), "synth_rows")


# ------------------------------------------------------------------------------------ K5 / K22
def counter_uniform(rows: torch.Tensor, key: int, stream=None) -> torch.Tensor:
    _dev(rows, "counter_uniform")
    rows = rows.to(torch.int64).contiguous()
    out = torch.empty(rows.numel(), dtype=torch.float64, device=rows.device)
    _native.check(_native.kernels().cml_counter_uniform(rows.data_ptr(), rows.numel(), _u64(key), out.data_ptr(),
                                                        _st(stream)), "counter_uniform")
    return out


def split_buckets(rows: torch.Tensor, key: int, cum: Sequence[float], stream=None) -> torch.Tensor:
    """int8 split index per row: first b with cum[b] <= u < cum[b+1] (-1 if none)."""
    _dev(rows, "split_buckets")
    nb = len(cum) - 1
    if not 1 <= nb <= 16:
        raise ValueError("randomSplit supports 1..16 weights on the GPU")
    rows = rows.to(torch.int64).contiguous()
    out = torch.empty(rows.numel(), dtype=torch.int8, device=rows.device)
    c = np.ascontiguousarray(np.asarray(cum, dtype=np.float64))
    _native.check(_native.kernels().cml_split_buckets(rows.data_ptr(), rows.numel(), _u64(key), c.ctypes.data, nb,
                                                      out.data_ptr(), _st(stream)), "split_buckets")
    return out


def poisson1(rows: torch.Tensor, key: int, thresholds: Sequence[float], out_dtype=torch.int32,
             stream=None) -> torch.Tensor:
    _dev(rows, "poisson1")
    rows = rows.to(torch.int64).contiguous()
    out = torch.empty(rows.numel(), dtype=out_dtype, device=rows.device)
    t = np.ascontiguousarray(np.asarray(thresholds, dtype=np.float64))
    i32 = out.data_ptr() if out_dtype == torch.int32 else 0
    f32 = out.data_ptr() if out_dtype == torch.float32 else 0
    if not (i32 or f32):
        raise ValueError("poisson1 output dtype must be int32 or float32")
    _native.check(_native.kernels().cml_poisson1(rows.data_ptr(), rows.numel(), _u64(key), t.ctypes.data, len(t), i32,
                                                 f32, _st(stream)), "poisson1")
    return out


# --------------------------------------------------------------------------------------------- K3
def compact(mask: torch.Tensor, stream=None) -> torch.Tensor:
    """Ascending int64 indices of the True entries of a bool mask (stream compaction)."""
    _dev(mask, "compact")
    m = mask.contiguous().view(torch.uint8) if mask.dtype == torch.bool else mask.to(torch.uint8).contiguous()
    n = m.numel()
    lib = _native.kernels()
    idx = torch.empty(max(n, 1), dtype=torch.int64, device=m.device)
    blocks = torch.empty(max(int(lib.cml_compact_blocks(n)), 1), dtype=torch.int64, device=m.device)
    cnt = torch.zeros(1, dtype=torch.int64, device=m.device)
    _native.check(lib.cml_compact(m.data_ptr(), n, idx.data_ptr(), blocks.data_ptr(), cnt.data_ptr(), _st(stream)),
                  "compact")
    return idx[: int(cnt.item())]


# --------------------------------------------------------------------------------------------- K2
def assemble(parts: List[Tuple[torch.Tensor, Optional[torch.Tensor]]], out_dtype=torch.float64, ld: int = 0,
             keep_nan: bool = True, stream=None) -> Tuple[torch.Tensor, torch.Tensor]:
    """Row-major [n, ld] matrix from scalar ([n]) and vector ([n, w]) device columns.

    ``parts`` = [(values, valid-or-None)]. Returns (matrix, invalid) where invalid[r] is True
    when any input of row r is null or NaN. Null entries become NaN (``keep_nan``) or 0.
    """
    if not parts:
        raise ValueError("assemble needs at least one column")
    dev = parts[0][0].device
    n = parts[0][0].shape[0]
    rec = np.zeros(len(parts), dtype=np.dtype([("ptr", "<u8"), ("valid", "<u8"), ("ld", "<i8"), ("type", "<i4"),
                                               ("width", "<i4"), ("off", "<i4"), ("pad", "<i4")]))
    keep = []
    off = 0
    for i, (v, valid) in enumerate(parts):
        _dev(v, "assemble")
        if v.shape[0] != n:
            raise ValueError("assemble: column lengths differ")
        if v.dtype not in _SRC_TYPES:
            raise TypeError(f"assemble: unsupported column dtype {v.dtype}")
        if v.dim() == 2 and v.stride(1) != 1:
            v = v.contiguous()
        if v.dim() == 1 and v.stride(0) != 1:
            v = v.contiguous()
        if v.dtype == torch.bool:
            v = v.view(torch.uint8)
        vv = None
        if valid is not None:
            vv = valid.to(device=dev, dtype=torch.bool).contiguous().view(torch.uint8)
            keep.append(vv)
        keep.append(v)
        w = 1 if v.dim() == 1 else int(v.shape[1])
        rec[i] = (v.data_ptr(), 0 if vv is None else vv.data_ptr(), 1 if v.dim() == 1 else v.stride(0),
                  _SRC_TYPES[v.dtype], w, off, 0)
        off += w
    d = off
    ld = max(ld, d)
    lib = _native.kernels()
    assert rec.itemsize == lib.cml_assemble_col_bytes()
    cols = torch.from_numpy(rec.view(np.uint8).copy()).to(dev)
    out = torch.empty((n, ld), dtype=out_dtype, device=dev)
    invalid = torch.empty(n, dtype=torch.uint8, device=dev)
    scalar_only = int(all(int(r["width"]) == 1 for r in rec))
    _native.check(lib.cml_assemble(cols.data_ptr(), len(parts), n, out.data_ptr(), _OUT_TYPES[out_dtype], ld, d,
                                   invalid.data_ptr(), int(keep_nan), scalar_only, _st(stream)), "assemble")
    del keep  # stream-ordered: any reuse of these blocks by the caching allocator runs after the launch
    return out, invalid.view(torch.bool)


# --------------------------------------------------------------------------------------------- K6
def binarize(x: torch.Tensor, threshold: float, stream=None) -> torch.Tensor:
    _dev(x, "binarize")
    if x.dtype not in _SRC_TYPES:
        raise TypeError(f"binarize: unsupported dtype {x.dtype}")
    xc = x.contiguous().reshape(-1)
    if xc.dtype == torch.bool:
        xc = xc.view(torch.uint8)
    out = torch.empty(xc.numel(), dtype=torch.float64, device=x.device)
    _native.check(_native.kernels().cml_binarize(xc.data_ptr(), _SRC_TYPES[xc.dtype], xc.numel(), float(threshold),
                                                 out.data_ptr(), _st(stream)), "binarize")
    return out.reshape(x.shape)


# -------------------------------------------------------------------------------------------- K23
def reg_metric_sums(y: torch.Tensor, p: torch.Tensor, w: Optional[torch.Tensor] = None, stream=None) -> torch.Tensor:
    """[Σw, Σw e², Σw |e|, Σw y, Σw y², Σw p, Σw p²] (float64, on device), e = y - p."""
    _dev(y, "reg_metric_sums")
    y = y.to(torch.float64).contiguous()
    p = p.to(device=y.device, dtype=torch.float64).contiguous()
    wv = None if w is None else w.to(device=y.device, dtype=torch.float64).contiguous()
    n = y.numel()
    lib = _native.kernels()
    grid = int(lib.cml_metric_grid(n))
    part = torch.empty((grid, 7), dtype=torch.float64, device=y.device)
    _native.check(lib.cml_reg_metrics(y.data_ptr(), p.data_ptr(), 0 if wv is None else wv.data_ptr(), n,
                                      part.data_ptr(), grid, _st(stream)), "reg_metrics")
    return part.sum(0)


def confusion(y: torch.Tensor, p: torch.Tensor, num_classes: int, w: Optional[torch.Tensor] = None,
              stream=None) -> torch.Tensor:
    """Weighted confusion matrix [C, C] (rows: label, cols: prediction), float64 on device."""
    _dev(y, "confusion")
    y = y.to(torch.int64).contiguous()
    p = p.to(device=y.device, dtype=torch.int64).contiguous()
    wv = None if w is None else w.to(device=y.device, dtype=torch.float64).contiguous()
    n = y.numel()
    lib = _native.kernels()
    grid = int(lib.cml_metric_grid(n))
    part = torch.empty((grid, num_classes * num_classes), dtype=torch.float64, device=y.device)
    _native.check(lib.cml_cls_confusion(y.data_ptr(), p.data_ptr(), 0 if wv is None else wv.data_ptr(), n,
                                        num_classes, part.data_ptr(), grid, _st(stream)), "cls_confusion")
    return part.sum(0).reshape(num_classes, num_classes)


# --------------------------------------------------------------------------------------------- K4
def col_absmax(x: torch.Tensor, d: int, stream=None) -> torch.Tensor:
    _dev(x, "col_absmax")
    codes = {torch.bfloat16: 0, torch.float32: 1}
    if x.dtype not in codes:
        raise TypeError("col_absmax: bf16 or f32 input")
    n = x.shape[0]
    rpb = 4096
    nb = max(1, (n + rpb - 1) // rpb)
    part = torch.zeros((nb, d), dtype=torch.float32, device=x.device)
    _native.check(_native.kernels().cml_col_absmax(x.data_ptr(), codes[x.dtype], n, d, x.stride(0), rpb,
                                                   part.data_ptr(), _st(stream)), "col_absmax")
    return part.amax(0)


def quant_fp8(x: torch.Tensor, d: int, scale: torch.Tensor, ld: Optional[int] = None, stream=None) -> torch.Tensor:
    """OCP e4m3fn bytes of x[:, :d]·scale (saturating), row-major [n, ld] (padding zero)."""
    _dev(x, "quant_fp8")
    codes = {torch.bfloat16: 0, torch.float32: 1}
    if x.dtype not in codes:
        raise TypeError("quant_fp8: bf16 or f32 input")
    n = x.shape[0]
    ld = d if ld is None else ld
    out = torch.empty((n, ld), dtype=torch.uint8, device=x.device)
    sc = scale.to(device=x.device, dtype=torch.float32).contiguous()
    _native.check(_native.kernels().cml_quant_fp8(x.data_ptr(), codes[x.dtype], n, d, x.stride(0), sc.data_ptr(),
                                                  out.data_ptr(), ld, _st(stream)), "quant_fp8")
    return out.view(torch.float8_e4m3fn)
