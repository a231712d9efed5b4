"""Python bindings of the KMeans kernels (K9–K11, ``_native/csrc/kmeans.hip``).

GPU tensors go to the gfx950 HIP kernels; there is no silent fallback — if the
kernel library is missing on a GPU box, the call raises.  CPU tensors use the
torch reference implementations below (the ``local[n]`` plumbing path and the
numerical oracle of the tests).
"""
from __future__ import annotations

import ctypes
import os
import threading

from dataclasses import dataclass

import torch

from .. import _native
from .._native import c_dbl, c_int, c_ll, c_vp
from ..utils.device import LDS_BUDGET, num_cus, round_up

_native.register_kernel_sigs({
    "cml_kmeans_assign_lds_bytes": (c_ll, [c_int, c_int, c_int]),
    "cml_kmeans_assign_threads": (c_int, [c_int]),
    "cml_kmeans_set_assign_variant": (c_int, [c_int]),
    "cml_kmeans_set_assign_sched": (c_int, [c_int]),
    "cml_kmeans_assign_occupancy": (c_int, [c_int, c_int, c_int, c_int]),
    "cml_kmeans_seg_threads": (c_int, []),
    "cml_kmeans_seg_ints": (c_ll, [c_int]),
    "cml_kmeans_assign_bf16": (c_int, [c_vp, c_ll, c_ll, c_int, c_vp, c_ll, c_int, c_int, c_int, c_vp, c_vp, c_vp,
                                       c_vp, c_int, c_int, c_vp, c_vp, c_vp, c_int, c_int, c_vp, c_vp, c_vp, c_vp,
                                       c_int, c_int, c_vp]),
    "cml_kmeans_assign_rr_plan": (c_int, [c_int, c_int, c_int, c_int, c_vp]),
    "cml_kmeans_set_rr_default": (c_int, [c_int]),
    "cml_kmeans_set_rr_debug": (c_int, [c_int]),
    "cml_kmeans_set_rr_m32": (c_int, [c_int]),
    "cml_kmeans_set_fp8_mx": (c_int, [c_int]),
    "cml_kmeans_set_delta_fused_fixup": (c_int, [c_int]),
    "cml_kmeans_assign_tile_rows": (c_int, [c_int]),
    "cml_row_sqnorm_bf16": (c_int, [c_vp, c_ll, c_ll, c_int, c_vp, c_vp]),
    "cml_row_sqnorm_fp8": (c_int, [c_vp, c_ll, c_ll, c_int, c_vp, c_vp]),
    "cml_kmeans_priv_lds_bytes": (c_ll, [c_int, c_int, c_int]),
    "cml_kmeans_accum_priv": (c_int, [c_vp, c_ll, c_ll, c_vp, c_int, c_int, c_int, c_int, c_vp, c_vp, c_int, c_int,
                                      c_vp]),
    "cml_kmeans_reduce": (c_int, [c_vp, c_vp, c_vp, c_int, c_int, c_int, c_int, c_int, c_vp, c_vp]),
    "cml_kmeans_sort_accum": (c_int, [c_vp, c_ll, c_ll, c_int, c_int, c_vp, c_vp, c_vp, c_int, c_int, c_int, c_int,
                                      c_vp, c_int, c_vp, c_vp, c_vp, c_int, c_int, c_vp, c_vp, c_vp, c_int, c_vp,
                                      ctypes.c_double, c_vp]),
    "cml_kmeans_sort_accum_ub": (c_int, [c_vp, c_ll, c_ll, c_int, c_int, c_vp, c_vp, c_vp, c_int, c_int, c_int,
                                         c_int, c_vp, c_int, c_vp, c_vp, c_vp, c_int, c_int, c_vp, c_vp, c_vp, c_int,
                                         c_vp, c_vp, c_ll, c_vp, ctypes.c_double, c_vp, c_vp]),
    "cml_kmeans_delta_gate": (c_int, [c_vp, c_int, c_int, c_vp, c_vp, c_vp, c_int, c_vp, c_vp]),
    "cml_kmeans_delta_accum": (c_int, [c_vp, c_ll, c_int, c_int, c_vp, c_vp, c_vp, c_vp, c_int, c_int, c_int, c_vp,
                                       c_int, c_vp, c_vp, c_vp, c_vp, c_int, c_int, c_vp, c_vp, c_vp, c_vp, c_vp,
                                       c_int, c_vp, c_int, ctypes.c_double, c_vp]),
    "cml_kmeans_seg_slot_doubles": (c_ll, [c_int, c_int]),
    "cml_kmeans_seg_slot_ints": (c_ll, [c_int]),
    "cml_kmeans_update": (c_int, [c_vp, c_int, c_ll, c_int, c_int, c_vp, c_vp, c_ll, c_int, c_int, c_vp, c_vp,
                                  ctypes.c_double, c_vp]),
    "cml_kmeans_prune_lower": (c_int, [c_vp, c_int, c_vp, c_vp, ctypes.c_float, ctypes.c_float, c_ll, c_vp, c_vp]),
    "cml_kmeans_prune_bounds": (c_int, [c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_int, c_ll, c_vp,
                                        c_vp, c_vp, c_vp, c_vp, c_vp, c_ll, c_vp, c_vp]),
    "cml_kmeans_prune_gate": (c_int, [c_vp, c_ll, c_vp, c_vp, c_vp, c_int, c_vp]),
    "cml_kmeans_converge_latch": (c_int, [c_vp, c_int, ctypes.c_double, c_vp, c_vp]),
    "cml_kmeans_cond_copy": (c_int, [c_vp, c_vp, c_ll, c_vp, c_vp, c_vp]),
    "cml_kmeans_seed_bounds": (c_int, [c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, ctypes.c_float, c_ll,
                                       c_vp, c_vp, c_vp, c_vp]),
    "cml_kmeans_label_hist": (c_int, [c_vp, c_ll, c_int, c_int, c_int, c_vp, c_vp, c_vp, c_int, c_vp]),
    "cml_kmeans_centre_stats": (c_int, [c_vp, c_vp, c_ll, c_int, c_int, c_vp, ctypes.c_float, c_vp, c_vp, c_vp,
                                        c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp]),
    "cml_kmeans_assign_rr_ext": (c_int, [c_int, c_vp, c_ll, c_ll, c_int, c_vp, c_ll, c_int, c_int, c_vp, c_vp,
                                         c_vp, c_vp, c_vp, c_vp, c_int, c_int, c_vp, c_vp, c_vp, c_vp, c_int,
                                         c_int, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, ctypes.c_float, c_vp, c_int,
                                         c_vp, c_vp, c_int, c_vp, c_vp, c_int, c_vp]),
    "cml_kmeans_init_classify": (c_int, [c_vp, c_vp, c_vp, c_vp, c_vp, c_int, ctypes.c_float, c_ll, c_int, c_vp,
                                         c_vp, c_vp, c_vp, c_vp]),
    "cml_kmeans_init_near_list": (c_int, [c_vp, c_ll, c_int, c_int, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_int, c_vp,
                                          c_int, ctypes.c_float, c_vp, c_vp, c_ll, c_vp]),
    "cml_kmeans_init_merge_list": (c_int, [c_vp, c_vp, c_vp, c_vp, c_int, c_vp, c_vp, c_ll, c_vp]),
})


_native.register_kernel_sigs({
    "cml_kmeans_row_pass": (c_int, [c_vp, c_ll, c_ll, c_int, c_int, c_vp, c_vp, ctypes.c_float, c_vp, c_vp, c_vp,
                                    c_vp, c_vp, c_vp, c_vp]),
    "cml_int_hist": (c_int, [c_vp, c_ll, c_int, c_vp, c_vp]),
    "cml_kmeans_cost_combine": (c_int, [c_vp, c_vp, c_int, c_ll, c_int, c_int, c_dbl, c_vp, c_int, c_vp, c_vp, c_vp]),
    "cml_kmeans_init_merge": (c_int, [c_vp, c_vp, c_vp, c_vp, c_int, c_ll, c_vp]),
    "cml_sum_f32_f64_parts": (c_int, []),
    "cml_kmeans_cost_parts": (c_int, []),
    "cml_kmeans_cost_pass": (c_int, [c_vp, c_ll, c_ll, c_int, c_int, c_vp, c_vp, c_ll, c_vp, c_vp, c_vp]),
    "cml_sum_f32_f64": (c_int, [c_vp, c_ll, c_vp, c_vp, c_vp]),
    "cml_fixsum": (c_int, [c_vp, c_int, c_vp, c_ll, c_int, c_vp, ctypes.c_float, c_vp, c_vp]),
    "cml_fixsum_finalize": (c_int, [c_vp, c_int, c_vp, ctypes.c_float, c_vp, c_vp]),
    "cml_kmeans_init_sample": (c_int, [c_vp, c_vp, c_ll, ctypes.c_uint64, ctypes.c_double, c_vp, c_vp, c_ll,
                                       c_vp, c_vp]),
    "cml_local_kpp": (c_int, [c_vp, c_vp, c_int, c_int, c_vp, c_int, ctypes.c_uint64, c_vp, c_vp, c_vp, c_vp,
                              c_vp]),
    "cml_local_assign": (c_int, [c_vp, c_int, c_int, c_vp, c_int, c_vp, c_vp, c_vp, c_vp]),
    "cml_local_update": (c_int, [c_vp, c_int, c_int, c_vp, c_vp, c_int, c_vp, c_vp, c_vp, c_int, c_vp, c_int, c_vp]),
    "cml_local_empty": (c_int, [c_vp, c_int, c_int, c_vp, c_int, ctypes.c_uint64, c_vp, c_vp, c_vp, c_vp, c_vp,
                                c_vp]),
})
_native.register_kernel_sigs({
    "cml_kmeans_exact_assign": (c_int, [c_vp, c_int, c_ll, c_ll, c_int, c_vp, c_int, c_vp, c_vp, c_vp, c_vp, c_vp,
                                        c_vp]),
    "cml_kmeans_exact_dist": (c_int, [c_vp, c_int, c_ll, c_ll, c_int, c_vp, c_int, c_vp, c_ll, c_vp, c_vp]),
    "cml_kmeans_to_bf16_err": (c_int, [c_vp, c_int, c_ll, c_ll, c_int, c_vp, c_ll, c_vp, c_vp]),
    "cml_kmeans_screen_cert": (c_int, [c_vp, c_vp, c_vp, c_vp, c_ll, c_vp, c_vp, c_vp, c_vp, c_vp]),
    "cml_kmeans_exact_chunks": (c_ll, [c_ll]),
    "cml_kmeans_exact_segsum": (c_int, [c_vp, c_int, c_ll, c_int, c_vp, c_vp, c_int, c_ll, c_vp, c_vp, c_vp, c_vp,
                                        c_vp]),
    "cml_kmeans_exact_top2": (c_int, [c_vp, c_int, c_ll, c_ll, c_int, c_vp, c_int, c_vp, c_vp, c_vp, c_vp, c_vp,
                                      c_vp, c_vp, c_vp, c_vp, c_vp, c_vp]),
    "cml_kmeans_to_bf16_split": (c_int, [c_vp, c_int, c_ll, c_ll, c_int, c_int, c_vp, c_ll, c_vp, c_vp, c_vp, c_vp,
                                         c_vp]),
    "cml_kmeans_screen_cert_split": (c_int, [c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_ll, c_vp, c_vp, c_vp, c_vp, c_vp]),
    "cml_kmeans_sum_dd": (c_int, [c_vp, c_ll, c_vp, c_vp, c_vp]),
    "cml_kmeans_init_table": (c_int, [c_vp, c_int, c_vp, c_int, c_int, c_vp, c_vp, c_vp, c_vp]),
    "cml_kmeans_pair_table": (c_int, [c_vp, c_int, c_vp, c_int, c_int, c_vp, c_vp, c_vp, c_vp]),
    "cml_kmeans_prune_bounds_gated": (c_int, [c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_int, c_ll, c_vp, c_vp,
                                              c_vp, c_vp, c_vp, c_vp, c_ll, c_vp, c_vp, c_ll, c_vp, c_int, c_vp,
                                              c_vp, c_vp]),
    "cml_kmeans_update_pdev": (c_int, [c_vp, c_int, c_ll, c_int, c_int, c_vp, c_vp, c_ll, c_int, c_int, c_vp, c_vp,
                                       c_dbl, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp]),
    "cml_kmeans_centre_half_stats": (c_int, [c_vp, c_ll, c_int, c_int, c_vp, c_vp, c_vp, c_vp, ctypes.c_float, c_vp,
                                             c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp]),
    "cml_kmeans_gather_rank_rows": (c_int, [c_vp, c_ll, c_int, c_int, c_vp, c_vp, c_int, c_vp, c_int, c_int, c_vp]),
    "cml_kmeans_gather_rank_max": (c_int, []),
    "cml_kmeans_seed_table": (c_int, [c_vp, c_int, c_int, c_vp, c_ll, c_int, c_vp, c_vp, c_vp, c_vp, c_vp]),
    "cml_kmeans_unique_rows": (c_int, [c_vp, c_int, c_int, c_vp, c_vp, c_vp, c_vp, c_vp]),
    "cml_kmeans_cert_stats": (c_int, [c_vp, c_vp, c_int, c_int, c_vp, c_vp, c_vp, c_vp, c_int, c_vp]),
    "cml_kmeans_cert_bounds": (c_int, [c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_ll, c_vp, c_vp, c_vp]),
    "cml_kmeans_cert_tighten": (c_int, [c_vp, c_int, c_ll, c_ll, c_int, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp,
                                        c_vp, c_vp, c_vp, c_vp, c_vp, c_vp]),
    "cml_kmeans_split_centres": (c_int, [c_vp, c_int, c_int, c_int, c_int, c_vp, c_ll, c_vp, c_vp, c_vp, c_vp]),
    "cml_kmeans_cert_list": (c_int, [c_vp, c_vp, c_ll, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp,
                                     c_vp, c_vp, c_vp, c_vp, c_vp]),
    "cml_kmeans_cert_slices": (c_int, [c_int]),
    "cml_kmeans_cert_moves": (c_int, [c_vp, c_int, c_ll, c_ll, c_int, c_int, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp,
                                      c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp]),
    "cml_mx_probe": (c_int, [c_vp, c_vp, c_vp, c_vp, c_vp, c_vp]),
    "cml_kmeans_centre_decay_stats": (c_int, [c_vp, c_vp, c_vp, c_int, c_vp, ctypes.c_float, c_vp, c_vp, c_vp, c_vp,
                                              c_vp, c_vp, c_vp, c_vp, c_vp]),
    "cml_kmeans_mx_snap": (c_int, [c_vp, c_ll, c_int, c_int, c_vp, c_vp, c_vp, c_vp, c_vp]),
})
_native.register_host_sigs({
    "cml_local_kmeans_host": (c_int, [c_vp, c_int, c_int, c_vp, c_int, ctypes.c_uint64, ctypes.c_uint64, c_int,
                                      c_int, c_vp]),
    "cml_exact_assign_host": (c_int, [c_vp, c_ll, c_ll, c_int, c_vp, c_int, c_vp, c_vp, c_int]),
    "cml_exact_sums_host": (c_int, [c_vp, c_ll, c_ll, c_int, c_vp, c_int, c_vp, c_vp, c_vp]),
})


def _ptr(t) -> int:
    return 0 if t is None else t.data_ptr()


def _u64(v: int) -> int:
    return int(v) & ((1 << 64) - 1)


def row_pass(x: torch.Tensor, n: int, dp: int, xn: torch.Tensor, c0: torch.Tensor | None = None, c0n: float = 0.0,
             cost: torch.Tensor | None = None, near: torch.Tensor | None = None,
             xn_max: torch.Tensor | None = None, erange: torch.Tensor | None = None,
             xn64: torch.Tensor | None = None, c0n_dev: torch.Tensor | None = None, stream=None) -> None:
    """One read of X (``kmeans_init.hip``): ``xn`` = ||x||² (bitwise ``row_sqnorm``), optionally the
    first k-means|| cost against the bf16-rounded centre ``c0`` (f32 [dp], norm ``c0n``) with
    ``near`` = 0, the max ||x||² (``xn_max``: f32 [1], zero-initialised, updated by bit-pattern
    atomicMax), the range of bf16 exponents (``erange``: int32 [2] = {INT_MAX, -1} initialised) and the
    norms summed in f64 (``xn64``: f64 [n], the training cost's per-centre Σ|x|²). ``c0n_dev`` (f32 [1]
    device scalar) replaces ``c0n`` with no host read."""
    if xn64 is not None and (xn64.dtype != torch.float64 or not xn64.is_contiguous() or xn64.numel() < n):
        raise ValueError("row_pass: xn64 must be a contiguous f64 [n] tensor")
    _native.check(_native.kernels().cml_kmeans_row_pass(
        x.data_ptr(), int(n), x.stride(0), int(dp), int(is_fp8(x)), xn.data_ptr(), _ptr(c0), float(c0n), _ptr(cost),
        _ptr(near), _ptr(xn_max), _ptr(erange), _ptr(xn64), _ptr(c0n_dev), _native.stream_ptr(stream)),
        "kmeans_row_pass")


def sum_f64(x: torch.Tensor, n: int, stream=None) -> torch.Tensor:
    """Σ x[:n] of a contiguous f32 device vector as an f64 device scalar (kmeans_init.hip: fixed-order
    block partials, no f64 copy of the input)."""
    if x.dtype != torch.float32 or not x.is_cuda or not x.is_contiguous() or x.data_ptr() % 16:
        raise ValueError("sum_f64: a 16-byte aligned contiguous f32 device vector")
    lib = _native.kernels()
    part = torch.empty(int(lib.cml_sum_f32_f64_parts()), dtype=torch.float64, device=x.device)
    out = torch.empty(1, dtype=torch.float64, device=x.device)
    _native.check(lib.cml_sum_f32_f64(x.data_ptr(), int(n), part.data_ptr(), out.data_ptr(),
                                      _native.stream_ptr(stream)), "sum_f32_f64")
    return out[0]


def cost_pass(x: torch.Tensor, n: int, dp: int, lab: torch.Tensor, cb: torch.Tensor, stream=None) -> torch.Tensor:
    """Σ_i |x_i - cb[lab_i]|² over the first n device rows as an f64 device tensor [1] (``kmeans_init.hip``):
    every difference and square in f64, fixed-order block partials — the exact cost of an assignment
    against the bf16 centres ``cb`` [kp, >= dp] it was made with, with no cancellation for data far from
    the origin (the expanded Σ(Q - 2c·S + n|c|²) form loses ~(|x|²/cost)·2^-24)."""
    if lab.dtype != torch.int32 or not lab.is_contiguous() or cb.dtype != torch.bfloat16 or cb.stride(1) != 1:
        raise ValueError("cost_pass: int32 labels and bf16 centres")
    if lab.numel() < n or cb.shape[1] < dp or x.shape[0] < n:
        raise ValueError("cost_pass: operand shapes")
    lib = _native.kernels()
    part = torch.empty(int(lib.cml_kmeans_cost_parts()), dtype=torch.float64, device=x.device)
    out = torch.empty(1, dtype=torch.float64, device=x.device)
    _native.check(lib.cml_kmeans_cost_pass(x.data_ptr(), int(n), x.stride(0), int(dp), int(is_fp8(x)),
                                           lab.data_ptr(), cb.data_ptr(), cb.stride(0), part.data_ptr(),
                                           out.data_ptr(), _native.stream_ptr(stream)), "kmeans_cost_pass")
    return out


def init_merge(cost: torch.Tensor, near: torch.Tensor, best: torch.Tensor, lab: torch.Tensor, off: int,
               n: int, stream=None) -> None:
    """cost/near <- best/lab+off where best < cost (a k-means|| candidate chunk's assign pass)."""
    _native.check(_native.kernels().cml_kmeans_init_merge(cost.data_ptr(), near.data_ptr(), best.data_ptr(),
                                                          lab.data_ptr(), int(off), int(n),
                                                          _native.stream_ptr(stream)), "kmeans_init_merge")


def init_sample(cost: torch.Tensor, ids: torch.Tensor, n: int, key: int, scale, out: torch.Tensor,
                count: torch.Tensor, stream=None) -> None:
    """Rows with counter-uniform(ids[i]) < scale·cost[i] appended (unordered) to ``out`` (at most
    len(out)); ``count`` (zeroed by the caller) receives their number. ``scale``: a float, or an f64 [2]
    device tensor {Σcost, 2k} whose quotient 2k / Σcost the kernel forms (no host read)."""
    dev_scale = torch.is_tensor(scale)
    if dev_scale and (scale.dtype != torch.float64 or scale.numel() < 2 or not scale.is_contiguous()):
        raise ValueError("init_sample: device scale is an f64 [2] tensor {sum, 2k}")
    _native.check(_native.kernels().cml_kmeans_init_sample(
        cost.data_ptr(), ids.data_ptr(), int(n), _u64(key), 0.0 if dev_scale else float(scale), out.data_ptr(),
        count.data_ptr(), int(out.shape[0]), scale.data_ptr() if dev_scale else 0, _native.stream_ptr(stream)),
        "kmeans_init_sample")


def fixsum(v: torch.Tensor, n: int, bound: torch.Tensor, mul: float = 1.0, lab: torch.Tensor | None = None,
           k: int = 1, limbs: torch.Tensor | None = None, stream=None) -> torch.Tensor:
    """Partition-invariant sum(s) of values 0 <= v <= bound·mul (exactsum.hip): the int64 limbs [2k] of Σ v (per
    label with ``lab``) on the grid of the device f32 ``bound`` — every rank must pass the same bound. The limbs
    add exactly, so they are all-reduced (sum) as is and ``fixsum_finalize`` turns them into f64 sums that are
    the same bits for any split of the rows over ranks."""
    if not v.is_cuda or v.dtype not in (torch.float32, torch.float64) or not v.is_contiguous():
        raise ValueError("fixsum: a contiguous f32 / f64 device vector")
    if bound.dtype != torch.float32 or not bound.is_cuda:
        raise ValueError("fixsum: the bound is a device f32 scalar")
    if lab is not None and (lab.dtype != torch.int32 or not lab.is_contiguous() or lab.numel() < n):
        raise ValueError("fixsum: int32 labels [n]")
    if lab is None and k != 1:
        raise ValueError("fixsum: k > 1 needs labels")
    if limbs is None:
        limbs = torch.zeros(2 * k, dtype=torch.int64, device=v.device)
    _native.check(_native.kernels().cml_fixsum(v.data_ptr(), 1 if v.dtype == torch.float32 else 2, _native.ptr(lab),
                                               int(n), int(k), bound.data_ptr(), float(mul), limbs.data_ptr(),
                                               _native.stream_ptr(stream)), "fixsum")
    return limbs


def fixsum_finalize(limbs: torch.Tensor, k: int, bound: torch.Tensor, mul: float = 1.0,
                    out: torch.Tensor | None = None, stream=None) -> torch.Tensor:
    """f64 [k] sums from (all-reduced) fixsum limbs, in a fixed order (the same bits on every rank)."""
    if out is None:
        out = torch.empty(k, dtype=torch.float64, device=limbs.device)
    _native.check(_native.kernels().cml_fixsum_finalize(limbs.data_ptr(), int(k), bound.data_ptr(), float(mul),
                                                        out.data_ptr(), _native.stream_ptr(stream)), "fixsum_finalize")
    return out


def int_hist(vals: torch.Tensor, n: int, m: int, counts: torch.Tensor, stream=None) -> None:
    """counts[v] += #{i < n: vals[i] = v} for int32 values in [0, m) (int32 counts, exact; device only)."""
    if vals.dtype != torch.int32 or counts.dtype != torch.int32 or counts.numel() < m or not vals.is_contiguous():
        raise ValueError("int_hist: int32 values and counts [m]")
    _native.check(_native.kernels().cml_int_hist(vals.data_ptr(), int(n), int(m), counts.data_ptr(),
                                                 _native.stream_ptr(stream)), "int_hist")


def zeros_block(device, specs) -> list:
    """Zeroed device tensors of the given (numel, dtype) specs as views of ONE allocation (one fill
    instead of one per tensor: each small torch.zeros costs ~10-20 us of host time on the launch path).
    Every view starts on a 512-byte boundary, the caching allocator's granule, so a view keeps the same
    slack past its end that a separate allocation had."""
    offs, o = [], 0
    for numel, dt in specs:
        offs.append(o)
        o += -(-max(int(numel), 1) * torch.empty((), dtype=dt).element_size() // 512) * 512
    blk = torch.zeros(max(o, 512), dtype=torch.uint8, device=device)
    es = [torch.empty((), dtype=dt).element_size() for _, dt in specs]
    return [blk[off: off + int(n) * e].view(dt) for off, (n, dt), e in zip(offs, specs, es)]


def cost_combine(q: torch.Tensor, msgs: torch.Tensor, k: int, d: int, unit: float, cb: torch.Tensor,
                 stream=None) -> torch.Tensor:
    """Σ_j q_j - 2 c_j·(S_j·unit) + n_j |c_j|², clamped at 0 (f64 device scalar): the training cost of an
    assignment from its per-cluster sums (msgs [rows, >= k*d + k]: S then n), the f64 per-cluster Σ||x||²
    ``q`` and the bf16 centres ``cb`` it compared against. Device tensors: a per-centre term launch and a
    fixed-order sum (kmeans_init.hip); host tensors: the same formula in torch."""
    kd = k * d
    if not q.is_cuda or cb.dtype != torch.bfloat16:  # (host engines; centres of another dtype)
        s_ = msgs[:, :kd].sum(0).view(k, d) * unit
        cnt = msgs[:, kd:kd + k].sum(0)
        c = cb[:k, :d].to(torch.float64)
        return (q.sum() - 2.0 * (c * s_).sum() + (cnt * (c * c).sum(1)).sum()).clamp(min=0.0)
    if (q.dtype != torch.float64 or msgs.dtype != torch.float64 or q.numel() < k
            or msgs.dim() != 2 or msgs.shape[1] < kd + k or msgs.stride(1) != 1 or cb.stride(1) != 1
            or cb.shape[0] < k or cb.shape[1] < d or not q.is_contiguous()):
        raise ValueError("cost_combine: f64 q [k], f64 msgs [rows, >= k*d + k], centres [>= k, >= d]")
    buf = torch.empty(k + 1, dtype=torch.float64, device=q.device)  # [k] per-centre terms, then the total
    _native.check(_native.kernels().cml_kmeans_cost_combine(
        q.data_ptr(), msgs.data_ptr(), int(msgs.shape[0]), int(msgs.stride(0)), int(k), int(d), float(unit),
        cb.data_ptr(), int(cb.stride(0)), buf.data_ptr(), buf[k:].data_ptr(), _native.stream_ptr(stream)),
        "kmeans_cost_combine")
    return buf[k]


_STOP = threading.local()  # per-thread pinned stop-flag word of local_kmeans (allocated once)


def local_kmeans(points: torch.Tensor, weights: torch.Tensor, k: int, seed: int, max_iter: int = 30,
                 spherical: bool = False, counts: bool = False) -> torch.Tensor:
    """Weighted k-means++ seeding + weighted Lloyd on a small candidate set (Spark
    LocalKMeans.kMeansPlusPlus), f64 [k, d]. GPU tensors run the ``kmeans_init.hip`` kernels (no host
    read: convergence is latched on the device); CPU tensors the host twin
    (``host/kmeans_local.cpp``), which performs the same rounded operations in the same order: both
    return the same bits. Draws: counter uniforms under (seed, 200) for the picks and (seed, 201) for
    empty-cluster reseeds. ``counts``: the caller guarantees non-negative weights with a positive sum
    (row counts of a non-empty dataset), so the clamp and the all-zero fallback are skipped."""
    from ..utils import rng
    pts = points.to(torch.float64).contiguous()
    m, d = pts.shape
    w = weights.to(device=pts.device, dtype=torch.float64)
    if not counts:
        # all-zero weights -> uniform, decided on the device (no host read before the seeding kernels)
        w = w.clamp(min=0)
        w = torch.where(w.sum() > 0, w, torch.ones_like(w))
    w = w.contiguous()
    key_pp, key_e = rng.key(seed, 200), rng.key(seed, 201)
    lds_update = ((m * 4 + 15) & ~15) + d * 8
    if pts.is_cuda and d * 8 <= 64 * 1024 and lds_update <= 150 * 1024:
        lib = _native.kernels()
        st = _native.stream_ptr(None)
        dev = pts.device
        C = torch.empty((k, d), dtype=torch.float64, device=dev)
        CT = torch.empty((d, k), dtype=torch.float64, device=dev)
        d2 = torch.empty(m, dtype=torch.float64, device=dev)
        lab = torch.full((m,), -1, dtype=torch.int32, device=dev)
        # cnt (f64 [k]), ctr (i64), flags (i32 [3] + pad) and picks (i32 [2k]): views of one zeroed block
        zb = torch.zeros(16 * k + 24, dtype=torch.uint8, device=dev)
        cnt = zb[: 8 * k].view(torch.float64)
        ctr = zb[8 * k: 8 * k + 8].view(torch.int64)
        flags = zb[8 * k + 8: 8 * k + 20].view(torch.int32)
        picks = zb[8 * k + 24:].view(torch.int32)
        PT = pts.t().contiguous()
        # pairwise candidate distances up front (one parallel pass) when they fit 1 GiB: each pick is
        # then a row read instead of m dimension folds on the one seeding workgroup
        D = torch.empty((m, m), dtype=torch.float64, device=dev) if m * m * 8 <= (1 << 30) else None
        _native.check(lib.cml_local_kpp(pts.data_ptr(), PT.data_ptr(), m, d, w.data_ptr(), int(k), _u64(key_pp),
                                        C.data_ptr(), CT.data_ptr(), d2.data_ptr(), _ptr(D), st), "local_kpp")
        del D
        # Lloyd without host reads: flags = {stop, moved[2]}; the update kernel latches stop once an
        # iteration's assign moved no label (the host loop's break), after which every queued launch
        # returns at once — max_iter iterations are enqueued back to back, the same bits as the host
        # twin's loop (a few no-op launches instead of one host round trip per iteration)
        fp = flags.data_ptr()
        # the stop flag is read back every 8 iterations (one small copy): converged local fits (a few
        # iterations) then launch 8 instead of max_iter x 3 no-op kernels (k-means|| finish on the shard)
        stop_h = getattr(_STOP, "h", None)
        if stop_h is None:
            stop_h = _STOP.h = torch.zeros(1, dtype=torch.int32, pin_memory=True)
        for it in range(max_iter):
            if it and it % 8 == 0:
                stop_h.copy_(flags[0:1], non_blocking=True)
                torch.cuda.current_stream(dev).synchronize()
                if int(stop_h[0]):
                    break
            slot = it & 1
            _native.check(lib.cml_local_assign(pts.data_ptr(), m, d, CT.data_ptr(), int(k), lab.data_ptr(),
                                               fp + 4 * (1 + slot), fp, st), "local_assign")
            _native.check(lib.cml_local_update(pts.data_ptr(), m, d, w.data_ptr(), lab.data_ptr(), int(k),
                                               C.data_ptr(), CT.data_ptr(), cnt.data_ptr(), int(bool(spherical)), fp,
                                               slot, st), "local_update")
            _native.check(lib.cml_local_empty(pts.data_ptr(), m, d, cnt.data_ptr(), int(k), _u64(key_e),
                                              ctr.data_ptr(), C.data_ptr(), CT.data_ptr(), picks.data_ptr(), fp, st),
                          "local_empty")
        return C
    P = pts.cpu().contiguous()
    W = w.cpu().contiguous()
    C = torch.empty((k, d), dtype=torch.float64)
    r = _native.host().cml_local_kmeans_host(P.data_ptr(), m, d, W.data_ptr(), int(k), _u64(key_pp), _u64(key_e),
                                             int(max_iter), int(bool(spherical)), C.data_ptr())
    if r < 0:
        raise ValueError("local k-means: empty candidate set")
    return C.to(pts.device)


@dataclass
class AssignPlan:
    n: int
    dp: int
    kp: int
    kc: int            # centres per launch (multiple of 32)
    grid: int
    nwaves: int
    round_rows: int = 0  # rows a workgroup ranks per round (sort-regime scatter geometry)
    rr_ct: int = 0       # > 0: K9r (register-resident centres, LDS-DMA X ring), centre tiles per wave


@dataclass
class AccumPlan:
    """Race-free accumulation regime (kmeans.hip K10).

    ``priv``: per-(wave,row-group) private LDS copies (small k·dw) — slabs + reduce.
    ``sort``: counting sort by label + segmented f64 accumulation (large k·D, skew-proof).
    """
    mode: str
    dw: int = 0
    cpl: int = 2
    rpw: int = 0
    nsl: int = 1
    gx: int = 1
    seg_grid: int = 1

    @property
    def dsl(self) -> int:
        return self.dw


FP8 = torch.float8_e4m3fn


def is_fp8(x: torch.Tensor) -> bool:
    return x.dtype == FP8


_ENV_APPLIED = False


def _apply_env_knobs(lib) -> None:
    """CML_KMEANS_ASSIGN_VARIANT / CML_KMEANS_RR (0/1) set the K9 launch knobs once per process."""
    global _ENV_APPLIED
    if _ENV_APPLIED:
        return
    _ENV_APPLIED = True
    v = os.environ.get("CML_KMEANS_ASSIGN_VARIANT")
    if v:
        _native.check(lib.cml_kmeans_set_assign_variant(int(v)), "set_assign_variant")
    rr = os.environ.get("CML_KMEANS_RR")
    if rr:
        _native.check(lib.cml_kmeans_set_rr_default(int(rr)), "set_rr_default")
    m32 = os.environ.get("CML_KMEANS_RR_M32")
    if m32:
        _native.check(lib.cml_kmeans_set_rr_m32(int(m32)), "set_rr_m32")
    if os.environ.get("CML_KMEANS_FP8_MX") == "0":
        lib.cml_kmeans_set_fp8_mx(0)
    fx = os.environ.get("CML_DELTA_FUSED_FIXUP")
    if fx:  # incremental sums: cross-slice partials added by the apply instead of a fixup launch (A/B)
        lib.cml_kmeans_set_delta_fused_fixup(int(fx))


def plan_assign(n: int, dp: int, k: int, device_index: int = 0, fp8: bool = False) -> AssignPlan:
    lib = _native.kernels()
    _apply_env_knobs(lib)
    kp = round_up(max(k, 1), 32)
    out = (ctypes.c_longlong * 3)()
    ct = lib.cml_kmeans_assign_rr_plan(dp, kp, kp, int(fp8), ctypes.addressof(out))
    if ct > 0:  # K9r: one 512-thread workgroup per CU, TR-row tiles dealt round-robin
        tr = int(out[1])
        grid = max(1, min((n + tr - 1) // tr, num_cus(device_index)))
        return AssignPlan(n=n, dp=dp, kp=kp, kc=kp, grid=grid, nwaves=1, round_rows=tr, rr_ct=int(ct))
    kc = kp
    while kc > 32 and lib.cml_kmeans_assign_lds_bytes(kc, kp, dp) > LDS_BUDGET:
        kc -= 32
    lds = lib.cml_kmeans_assign_lds_bytes(kc, kp, dp)
    if lds > LDS_BUDGET:
        raise ValueError(f"feature width {dp} / k={k} too large for the LDS-resident centroid tile")
    waves = lib.cml_kmeans_assign_threads(dp) // 64
    per_cu = max(1, min(4, (160 * 1024) // max(lds, 1)))
    if torch.cuda.is_available():
        occ = lib.cml_kmeans_assign_occupancy(dp, kc, kp, int(fp8))
        if occ > 0:  # persistent grid: never more workgroups than can be resident at once
            per_cu = max(1, min(per_cu, occ))
    ntiles = (n + 31) // 32
    grid = max(1, min((ntiles + waves - 1) // waves, num_cus(device_index) * per_cu))
    return AssignPlan(n=n, dp=dp, kp=kp, kc=kc, grid=grid, nwaves=waves,
                      round_rows=waves * lib.cml_kmeans_assign_tile_rows(dp))


def set_assign_variant(v: int) -> None:
    """Tuning knob for the K9 launch shape (0 auto, 1 one wave/SIMD, 2 two waves/SIMD, ..., 6 default shape with
    per-sub-tile accumulator seeding, 7 PACK4 keys, 8 K9r register-resident centres + LDS-DMA X ring).
    Plans made before a change keep the kernel they were made for."""
    _native.check(_native.kernels().cml_kmeans_set_assign_variant(int(v)), "set_assign_variant")


def set_rr_default(on: bool) -> None:
    """Whether variant 0 (auto) picks K9r wherever it applies."""
    _native.check(_native.kernels().cml_kmeans_set_rr_default(int(bool(on))), "set_rr_default")


def set_rr_m32(on: bool) -> None:
    """K9r compute waves on 32x32x16 MFMA tiles (even centre-tile counts; CML_KMEANS_RR_M32=1) or the
    16x16x32 form (default, faster on MI355X). Both give the same labels up to the distance rounding."""
    _native.check(_native.kernels().cml_kmeans_set_rr_m32(int(bool(on))), "set_rr_m32")


def set_assign_sched(v: int) -> None:
    """Tuning knob: partner-wave desynchronisation of K9 (bit 0 priority, bit 1 + v>>2 stagger)."""
    _native.check(_native.kernels().cml_kmeans_set_assign_sched(int(v)), "set_assign_sched")


def plan_accum(n: int, dp: int, k: int, device_index: int = 0, force: str | None = None,
               fp8: bool = False) -> AccumPlan:
    lib = _native.kernels()
    ncu = num_cus(device_index)
    if fp8:  # e4m3 rows: sort regime, CPL bytes per lane (dp >= 256)
        if force == "priv" or dp < 256 or dp > 1024:
            raise ValueError("fp8 features accumulate in the sort regime with 256 <= Dp <= 1024")
        return AccumPlan(mode="sort", cpl=dp // 64, seg_grid=max(1, min((n + 255) // 256, ncu * 4)), dw=dp)
    dw = min(dp, 256)
    cpl = 4 if dw > 128 else 2
    # Default: the sort regime whenever it applies. Its f64 segmented sums of bf16 rows are exact, so
    # results do not depend on how rows are split over workgroups or GPUs, and it carries the
    # incremental-sums step. The private-copy regime (f32 LDS partials) stays for Dp > 512 and on request.
    if force is None and dp <= 512:
        force = "sort"
    if force != "sort":
        r = max(1, min(16, (cpl * 64) // dw))
        while r >= 1:
            lds = lib.cml_kmeans_priv_lds_bytes(k, dw, r)
            if lds <= LDS_BUDGET:
                nsl = (dp + dw - 1) // dw
                per_cu = max(1, min(2, (160 * 1024) // max(lds, 1)))
                want = max(1, (n + 8191) // 8192)
                gx = max(1, min(want, (ncu * per_cu + nsl - 1) // nsl))
                return AccumPlan(mode="priv", dw=dw, cpl=cpl, rpw=r, nsl=nsl, gx=gx)
            r //= 2
    if force == "priv":
        raise ValueError("private-copy accumulation does not fit LDS")
    if dp > 512:
        raise ValueError("sort-regime accumulation supports Dp <= 512")
    scpl = 2 if dp <= 128 else (4 if dp <= 256 else 8)
    seg_grid = max(1, min((n + 255) // 256, ncu * 4))
    return AccumPlan(mode="sort", cpl=scpl, seg_grid=seg_grid, dw=dp)


def assign_bf16(x: torch.Tensor, n: int, dp: int, cb: torch.Tensor, cnorm: torch.Tensor, plan: AssignPlan,
                labels: torch.Tensor, best: torch.Tensor | None, cost_part: torch.Tensor | None,
                hist: torch.Tensor | None = None, rank: torch.Tensor | None = None, stream=None,
                xnorm: torch.Tensor | None = None, delta: "DeltaState | None" = None) -> None:
    """K9: labels/best[i] = argmin/min_j ||x_i - c_j||² over all kp (padded) centres.

    With ``hist``/``rank`` also emits the per-workgroup label histogram and per-row rank
    (first pass of the counting sort used by the sort accumulation regime). ``xnorm`` are the
    cached ||x_i||² (row_sqnorm; Spark's KMeans caches point norms the same way,
    mllib/clustering/KMeans.scala ``VectorWithNorm``); ``best`` may be None when the centres fit
    one LDS chunk and the distances themselves are not wanted. With ``delta`` (single-launch plans
    only) rows whose label changes are logged for the incremental sums.
    """
    lib = _native.kernels()
    st = _native.stream_ptr(stream)
    nch = (plan.kp + plan.kc - 1) // plan.kc
    if xnorm is None:
        xnorm = row_sqnorm(x, n, dp, stream=stream)
    if best is None and nch > 1:
        raise ValueError("multi-chunk assignment needs the `best` scratch buffer")
    if delta is not None and nch > 1:
        raise ValueError("label-change logging needs a single-launch assign")
    for ci in range(nch):
        c0 = ci * plan.kc
        kc = min(plan.kc, plan.kp - c0)
        last = ci == nch - 1
        status = lib.cml_kmeans_assign_bf16(
            x.data_ptr(), n, x.stride(0), dp,
            cb.data_ptr() + c0 * cb.stride(0) * 2, cb.stride(0), kc, plan.kp, c0,
            cnorm.data_ptr() + c0 * 4, xnorm.data_ptr(),
            labels.data_ptr(), best.data_ptr() if best is not None else 0,
            int(ci == 0), int(last),
            cost_part.data_ptr() if (cost_part is not None and last) else 0,
            hist.data_ptr() if (hist is not None and last) else 0,
            rank.data_ptr() if (rank is not None and last) else 0,
            plan.grid, int(is_fp8(x)),
            delta.rows.data_ptr() if delta is not None else 0, delta.old.data_ptr() if delta is not None else 0,
            delta.wg_count.data_ptr() if delta is not None else 0,
            delta.overflow.data_ptr() if delta is not None else 0, delta.pcap if delta is not None else 0,
            plan.rr_ct, st)
        _native.check(status, "kmeans_assign_bf16")


def row_sqnorm(x: torch.Tensor, n: int, dp: int, out: torch.Tensor | None = None, stream=None) -> torch.Tensor:
    """||x_i||² (f32) of the padded bf16 device matrix, computed once per fit."""
    if out is None:
        out = torch.empty(max(n, 1), dtype=torch.float32, device=x.device)
    if n > 0:
        fn = _native.kernels().cml_row_sqnorm_fp8 if is_fp8(x) else _native.kernels().cml_row_sqnorm_bf16
        _native.check(fn(x.data_ptr(), n, x.stride(0), dp, out.data_ptr(), _native.stream_ptr(stream)), "row_sqnorm")
    return out


def accumulate_priv(x: torch.Tensor, n: int, labels: torch.Tensor, k: int, plan: AccumPlan,
                    slab: torch.Tensor, cslab: torch.Tensor, stream=None) -> None:
    """K10 regime A: slab[sl][g][c][d] = Σ_{rows of WG g, label c} x[row, sl*dw + d]."""
    lib = _native.kernels()
    status = lib.cml_kmeans_accum_priv(x.data_ptr(), n, x.stride(0), labels.data_ptr(), k, plan.dw, plan.cpl,
                                       plan.rpw, slab.data_ptr(), cslab.data_ptr(), plan.gx, plan.nsl,
                                       _native.stream_ptr(stream))
    _native.check(status, "kmeans_accum_priv")


def reduce_slabs(slab, cslab, cost_part, ncost: int, k: int, d: int, plan: AccumPlan, out: torch.Tensor,
                 stream=None) -> None:
    """K10b: out = [Σx per (c,d) | count per c | cost] in f64, fixed summation order."""
    lib = _native.kernels()
    status = lib.cml_kmeans_reduce(slab.data_ptr(), cslab.data_ptr(), cost_part.data_ptr(), plan.gx, ncost, k,
                                   d, plan.dsl, out.data_ptr(), _native.stream_ptr(stream))
    _native.check(status, "kmeans_reduce")


def seg_slots(plan: AccumPlan, d: int, device) -> tuple:
    """Scratch of the deterministic segmented sum: per-slice head/tail partials + their cluster ids."""
    lib = _native.kernels()
    sl = torch.empty(max(int(lib.cml_kmeans_seg_slot_doubles(plan.seg_grid, d)), 1), dtype=torch.float64,
                     device=device)
    sc = torch.empty(max(int(lib.cml_kmeans_seg_slot_ints(plan.seg_grid)), 1), dtype=torch.int32, device=device)
    return sl, sc


def accumulate_sort(x: torch.Tensor, n: int, dp: int, d: int, labels: torch.Tensor, rank: torch.Tensor,
                    hist: torch.Tensor, aplan: AssignPlan, k: int, cost_part: torch.Tensor, off: torch.Tensor,
                    seg: torch.Tensor, perm: torch.Tensor, plan: AccumPlan, msg: torch.Tensor,
                    slots: tuple, stream=None, gate: torch.Tensor | None = None,
                    ub_centres: torch.Tensor | None = None, ub: torch.Tensor | None = None,
                    qscale: float = 0.0, cum: torch.Tensor | None = None) -> None:
    """K10 regime B: counting sort by label, then segmented f64 sums -> msg (deterministic).
    With ``gate`` (DeltaState.mode) the launches only run on steps the gate marks as full. With
    ``ub_centres`` (bf16 [kp, dp]) and ``ub`` (f32 [n]) the segmented pass also writes every row's upper
    bound of |x - c_label| (the exact-pruning bound) as the rows stream through. ``qscale`` (a power of
    two, 0 = off) sums the rows on the grid 1/qscale: every value is scaled and rounded to an integer,
    so the f64 sums are exact integers (LloydEngine._sum_grid) and K11 scales them back. ``cum``
    (f32 [2k], the offset-form bounds' cumulative drifts) stores ub - cum[label] instead of ub."""
    lib = _native.kernels()
    args = (x.data_ptr(), n, x.stride(0), dp, d, labels.data_ptr(), rank.data_ptr(), hist.data_ptr(), aplan.grid,
            aplan.round_rows, k, aplan.kp, cost_part.data_ptr(), aplan.grid, off.data_ptr(), seg.data_ptr(),
            perm.data_ptr(), plan.cpl, plan.seg_grid, msg.data_ptr(), slots[0].data_ptr(), slots[1].data_ptr(),
            int(is_fp8(x)), gate.data_ptr() if gate is not None else 0)
    if ub is not None:
        if ub_centres is None or ub_centres.dtype != torch.bfloat16 or ub.dtype != torch.float32 or ub.numel() < n:
            raise ValueError("accumulate_sort: ub needs bf16 centres and an f32 [n] output")
        status = lib.cml_kmeans_sort_accum_ub(*args, ub_centres.data_ptr(), ub_centres.stride(0), ub.data_ptr(),
                                              float(qscale), _ptr(cum), _native.stream_ptr(stream))
    else:
        status = lib.cml_kmeans_sort_accum(*args, float(qscale), _native.stream_ptr(stream))
    _native.check(status, "kmeans_sort_accum")


class DeltaState:
    """Device state of the incremental-sums Lloyd step (kmeans.hip ``kmeans_delta_gate``).

    ``acc`` rows hold, per row chunk, [k·D sums | k counts | cost] of the chunk's CURRENT labels;
    a step whose label changes exceed ``cap`` rows (or that is forced: the first one) re-accumulates
    ``acc`` in full, every other step applies only the changed rows. ``force`` is set on creation and
    by ``invalidate()``."""

    def __init__(self, n: int, k: int, d: int, dp: int, chunks: int, msg_len: int, device, nblk: int,
                 fp8: bool = False, cap_fraction: float | None = None, cap: int | None = None,
                 pcap: int | None = None, lean: bool = False):
        self.k, self.d, self.nblk = k, d, int(nblk)
        if cap_fraction is None:  # steps with more label changes than this re-accumulate in full
            cap_fraction = float(os.environ.get("CML_KMEANS_DELTA_CAP", 0.25))
        self.cap = max(1024, int(n * cap_fraction)) if cap is None else int(cap)
        # change lists are per assign workgroup: nblk lists of pcap entries (slack for uneven churn)
        self.pcap = max(64, -(-2 * self.cap // self.nblk)) if pcap is None else int(pcap)
        # lean: the lists hold every row of their workgroup (pcap >= its rows), so the delta path can take any
        # number of changes and a step whose sums are valid never needs the full re-accumulation — the caller
        # then enqueues only the delta launches (gate(lean=True)); the full path runs on forced steps only
        self.lean = bool(lean)
        self.host_forced = True  # the device force flag is set (creation / invalidate): next gate is not lean
        self.entries = self.nblk * self.pcap if self.lean else self.cap
        i32, f64, lists = torch.int32, torch.float64, self.nblk * self.pcap
        (self.rows, self.old, self.wg_count, self.overflow, mode, self.dh, self.dseg, self.cursor, self.dperm,
         self.dsum, acc) = zeros_block(device, [(lists, i32), (lists, i32), (self.nblk, i32), (1, i32),
                                                (2 * chunks, i32), (2 * k, i32), (2 * k + 2, i32), (2 * k, i32),
                                                (2 * self.entries, i32), (2 * k * d, f64), (chunks * msg_len, f64)])
        self.mode, self.acc = mode.view(chunks, 2), acc.view(chunks, msg_len)
        self.force = torch.ones(chunks, dtype=torch.int32, device=device)
        ncu = num_cus(device.index or 0)
        self.plan = AccumPlan(mode="sort", cpl=(dp // 64 if fp8 else (2 if dp <= 128 else (4 if dp <= 256 else 8))),
                              seg_grid=max(1, min((2 * self.entries + 255) // 256, ncu * 4)), dw=dp)
        self.slots = seg_slots(self.plan, d, device)

    def invalidate(self) -> None:
        """Next step re-accumulates in full (labels or acc no longer describe each other)."""
        self.force.fill_(1)
        self.host_forced = True

    def lean_step(self) -> bool:
        """Whether the next step may skip the full-accumulate launches (lean lists, no force pending)."""
        return self.lean and not self.host_forced

    def gate(self, chunk: int, stream=None, lean: bool = False) -> None:
        """Full re-accumulation or delta for this step, decided on the device. ``lean``: the step enqueues no
        full path (lean_step()), so only a forced step may pick it — the change count never does."""
        if lean and not self.lean_step():
            raise RuntimeError("lean delta gate on a forced step or without lean change lists")
        _native.check(_native.kernels().cml_kmeans_delta_gate(
            self.wg_count.data_ptr(), self.nblk, (1 << 30) if lean else self.cap, self.overflow.data_ptr(),
            self.force[chunk:].data_ptr(), self.mode[chunk].data_ptr(), self.k, self.dh.data_ptr(),
            _native.stream_ptr(stream)), "kmeans_delta_gate")
        if chunk == self.force.shape[0] - 1:
            self.host_forced = False  # the gate consumed the device flag (every chunk's gate ran)

    def accumulate(self, x: torch.Tensor, dp: int, labels: torch.Tensor, chunk: int, cost_part: torch.Tensor,
                   ncost: int, msg: torch.Tensor, stream=None, qscale: float = 0.0) -> None:
        _native.check(_native.kernels().cml_kmeans_delta_accum(
            x.data_ptr(), x.stride(0), dp, self.d, labels.data_ptr(), self.rows.data_ptr(), self.old.data_ptr(),
            self.wg_count.data_ptr(), self.nblk, self.pcap, self.entries, self.mode[chunk].data_ptr(), self.k,
            self.dh.data_ptr(), self.dseg.data_ptr(),
            self.cursor.data_ptr(), self.dperm.data_ptr(), self.plan.cpl, self.plan.seg_grid, self.dsum.data_ptr(),
            self.slots[0].data_ptr(), self.slots[1].data_ptr(), self.acc[chunk].data_ptr(), cost_part.data_ptr(),
            ncost, msg.data_ptr(), int(is_fp8(x)), float(qscale), _native.stream_ptr(stream)), "kmeans_delta_accum")

    def changed_rows(self, chunk: int = 0) -> int:
        """Label changes of the last step (0 on a full step). Synchronises."""
        return int(self.mode[chunk, 1].item())

    def was_full(self, chunk: int = 0) -> bool:
        return bool(self.mode[chunk, 0].item())


def prune_bounds(labels: torch.Tensor, ub: torch.Tensor, lb: torch.Tensor, drift: torch.Tensor,
                 dmax: torch.Tensor, thr: torch.Tensor, c2, k: int, cand: torch.Tensor,
                 count: torch.Tensor, stream=None, xn: torch.Tensor | None = None,
                 cand_lab: torch.Tensor | None = None, cand_xn: torch.Tensor | None = None,
                 skip: torch.Tensor | None = None, zero_count: bool = True, cum: torch.Tensor | None = None) -> None:
    """K9p (``kmeans_prune.hip``): moves the per-row distance bounds by the centre drifts
    (ub += drift[label], lb -= largest drift of another centre) and appends to ``cand`` the rows whose
    bounds no longer prove the label (neither ub <= thr[label] nor ub <= lb - c2 / lb); ``count[0]`` =
    their number (on the GPU at most ``len(cand)`` of them are written). ``dmax`` = [largest drift, second largest, index of the largest]. GPU: ``c2`` is a
    device scalar; with ``cand_lab``/``cand_xn`` the candidates' labels and norms are written compacted
    beside ``cand`` (the K9r candidate pass reads them); ``skip`` (device flag) turns the launch into a
    no-op; ``zero_count=False`` leaves the zeroing of ``count`` to the caller (the centre-stats pass);
    ``cum`` (f32 [2k] cumulative drifts) selects the offset-form bounds: ``ub``/``lb`` hold ub - cu[label]
    and lb + cl[label], the drifts are already in ``cum``, and the pass only reads them (no bound writes).
    CPU tensors: the same pass in torch (f64 bounds), candidates in row order."""
    n = int(labels.shape[0])
    if labels.is_cuda:
        if zero_count:
            count.zero_()
        if not torch.is_tensor(c2):
            c2 = torch.tensor([float(c2)], dtype=torch.float32, device=labels.device)
        _native.check(_native.kernels().cml_kmeans_prune_bounds(
            labels.data_ptr(), ub.data_ptr(), lb.data_ptr(), drift.data_ptr(), dmax.data_ptr(), thr.data_ptr(),
            c2.data_ptr(), int(k), n, cand.data_ptr(), count.data_ptr(), _ptr(xn), _ptr(cand_lab), _ptr(cand_xn),
            _ptr(skip), int(cand.shape[0]), _ptr(cum), _native.stream_ptr(stream)), "kmeans_prune_bounds")
        return
    c2 = float(c2)
    lab = labels[:n].long()
    ub[:n] += drift[lab]
    other = torch.where(lab == int(dmax[2]), dmax[1], dmax[0])
    lb[:n] = (lb[:n] - other).clamp_(min=0.0)
    w = lb[:n]
    lt = torch.where(w > 0, w - c2 / w.clamp(min=1e-300), torch.full_like(w, -1.0))
    keep = (ub[:n] <= thr[lab]) | (ub[:n] <= lt)
    idx = torch.nonzero(~keep).flatten()
    cand[: idx.numel()] = idx.to(cand.dtype)
    count[0] = idx.numel()


def seed_bounds(nearest: torch.Tensor, cost: torch.Tensor, xn: torch.Tensor, qmap: torch.Tensor, a: torch.Tensor,
                d1: torch.Tensor, d2: torch.Tensor, pn: torch.Tensor, tau: float, n: int, labels: torch.Tensor,
                ub: torch.Tensor, lb: torch.Tensor, stream=None) -> None:
    """Labels and exact-pruning bounds of every row from the k-means|| init (kmeans_prune.hip): nearest
    candidate (int32 index into qmap), its squared distance (f32) and the candidate -> (centre a, d1, d2,
    |p|²) tables (int32 / f32). Device only."""
    for t, dt in ((nearest, torch.int32), (cost, torch.float32), (xn, torch.float32), (qmap, torch.int32),
                  (a, torch.int32), (d1, torch.float32), (d2, torch.float32), (pn, torch.float32),
                  (labels, torch.int32), (ub, torch.float32), (lb, torch.float32)):
        if t.dtype != dt or not t.is_contiguous():
            raise ValueError("seed_bounds: operand dtype/layout")
    _native.check(_native.kernels().cml_kmeans_seed_bounds(
        nearest.data_ptr(), cost.data_ptr(), xn.data_ptr(), qmap.data_ptr(), a.data_ptr(), d1.data_ptr(),
        d2.data_ptr(), pn.data_ptr(), float(tau), int(n), labels.data_ptr(), ub.data_ptr(), lb.data_ptr(),
        _native.stream_ptr(stream)), "kmeans_seed_bounds")


def label_hist(labels: torch.Tensor, n: int, plan: "AssignPlan", hist: torch.Tensor, rank: torch.Tensor,
               stream=None, gate: torch.Tensor | None = None, want: int = 0) -> None:
    """Counting-sort ranks of the current labels in the K9r workgroup geometry (what a full K9r pass
    leaves in hist/rank for the sort-regime accumulate). ``gate``/``want``: run only when gate[0] ==
    want (device flag). Device only."""
    if labels.dtype != torch.int32 or hist.numel() < plan.grid * plan.kp or rank.numel() < n:
        raise ValueError("label_hist: operand shapes")
    _native.check(_native.kernels().cml_kmeans_label_hist(labels.data_ptr(), int(n), int(plan.round_rows),
                                                          int(plan.grid), int(plan.kp), hist.data_ptr(),
                                                          rank.data_ptr(), _ptr(gate), int(want),
                                                          _native.stream_ptr(stream)),
                  "kmeans_label_hist")


def prune_bounds_gated(labels, ub, lb, drift, dmax, thr, c2, k: int, cand, count, xn, cand_lab, cand_xn, flags,
                       cum, mode, gate_cap: int, backoff, nback: int, done, stream=None, mode_host=None) -> None:
    """K9p with the step gate folded in (kmeans_prune.hip): the bounds pass (skipped when flags[0] / flags[1]
    are set) and, in the workgroup that finishes last, kmeans_prune_gate's decision into ``mode``; ``done``
    (int32 [1], zero) is the completion counter. Device only; count is zeroed by the centre statistics.
    ``mode_host`` (pinned int32 [1], optional): the gate also stores its full-pass flag there, for the host to
    read without synchronising (a lagged hint)."""
    n = int(labels.shape[0])
    _native.check(_native.kernels().cml_kmeans_prune_bounds_gated(
        labels.data_ptr(), ub.data_ptr(), lb.data_ptr(), drift.data_ptr(), dmax.data_ptr(), thr.data_ptr(),
        c2.data_ptr(), int(k), n, cand.data_ptr(), count.data_ptr(), _ptr(xn), _ptr(cand_lab), _ptr(cand_xn),
        flags.data_ptr(), int(cand.shape[0]), _ptr(cum), mode.data_ptr(), int(gate_cap), _ptr(backoff), int(nback),
        done.data_ptr(), _ptr(mode_host), _native.stream_ptr(stream)), "kmeans_prune_bounds_gated")


def update_pdev(msgs: torch.Tensor, k: int, d: int, cent: torch.Tensor, cb: torch.Tensor, dp: int, kp: int,
                cnorm: torch.Tensor, shift2: torch.Tensor, unit: float, cb_old: torch.Tensor, cb_cost: torch.Tensor,
                flags: torch.Tensor, cn64: torch.Tensor, drift: torch.Tensor, stream=None, snap: bool = False) -> None:
    """K11 of the device pruned step with its bookkeeping in the same launch (kmeans_prune.hip
    kmeans_update_pdev_kernel): cb_old <- old cb, cb_cost <- old cb unless frozen (flags[1]), the new centres,
    their bf16 copy and norms (f32 cnorm, f64 cn64), the shift and the bf16 drift rounded up. ``snap``: the
    bf16 centres then go onto the MX grid, norms and drifts recomputed (mx_snap)."""
    _native.check(_native.kernels().cml_kmeans_update_pdev(
        msgs.data_ptr(), msgs.shape[0], msgs.stride(0), int(k), int(d), cent.data_ptr(), cb.data_ptr(), cb.stride(0),
        int(dp), int(kp), cnorm.data_ptr(), shift2.data_ptr(), float(unit), cb_old.data_ptr(), cb_cost.data_ptr(),
        flags.data_ptr(), cn64.data_ptr(), drift.data_ptr(), _native.stream_ptr(stream)), "kmeans_update_pdev")
    if snap:
        mx_snap(cb, k, dp, cnorm, cn64=cn64, cb_old=cb_old, drift=drift, stream=stream)


def centre_decay_stats(k: int, cn: torch.Tensor, half: torch.Tensor, drift: torch.Tensor, mx: torch.Tensor,
                       tau: float, thr, dmax, mc, c2, count, force, cum, backoff, stream=None) -> None:
    """The pruned step's centre statistics without the nearest-centre pass (kmeans_centre_decay_stats_kernel):
    half_j lowered by the step's drifts (half_j - (drift_j + max_{i!=j} drift_i) / 2, still a lower bound of
    half the nearest-centre distance), then thr, dmax, mc, c2, the cumulative drifts and the resets of
    centre_half_stats. One workgroup."""
    _native.check(_native.kernels().cml_kmeans_centre_decay_stats(
        cn.data_ptr(), half.data_ptr(), drift.data_ptr(), int(k), mx.data_ptr(), float(tau), thr.data_ptr(),
        dmax.data_ptr(), mc.data_ptr(), c2.data_ptr(), count.data_ptr(), force.data_ptr(), _ptr(cum), _ptr(backoff),
        _native.stream_ptr(stream)), "kmeans_centre_decay_stats")


def centre_half_stats(cb: torch.Tensor, k: int, d: int, cn: torch.Tensor, half: torch.Tensor, drift: torch.Tensor,
                      mx: torch.Tensor, tau: float, thr, dmax, mc, c2, count, force, cum, backoff, done,
                      stream=None) -> None:
    """The pruned step's centre statistics in one launch (kmeans_centre_half_stats_kernel): half nearest-centre
    distances, then — in the workgroup that finishes last — thr, dmax, mc, c2, the cumulative drifts and the
    count / force / backoff resets (norms and drifts come from update_pdev). ``done``: int32 [1], zero."""
    _native.check(_native.kernels().cml_kmeans_centre_half_stats(
        cb.data_ptr(), cb.stride(0), int(k), int(d), cn.data_ptr(), half.data_ptr(), drift.data_ptr(), mx.data_ptr(),
        float(tau), thr.data_ptr(), dmax.data_ptr(), mc.data_ptr(), c2.data_ptr(), count.data_ptr(),
        force.data_ptr(), _ptr(cum), _ptr(backoff), done.data_ptr(), _native.stream_ptr(stream)),
        "kmeans_centre_half_stats")


def prune_gate(count: torch.Tensor, cap: int, flags: torch.Tensor, mode: torch.Tensor, stream=None,
               backoff: torch.Tensor | None = None, nback: int = 2) -> None:
    """mode[0] = 1 (full pass) when flags[0] (force) or count[0] > cap, else 0 (candidate pass); with
    flags[1] (done: the fit converged) a frozen step — candidate pass over 0 rows (count zeroed).
    ``backoff`` (int32 [1]): a step over the cap sets it to ``nback`` and centre_stats then forces that
    many steps full (no bounds pass). ``flags``: int32 [2] device tensor. Device only."""
    if flags.dtype != torch.int32 or flags.numel() < 2:
        raise ValueError("prune_gate: flags must be int32 [force, done]")
    _native.check(_native.kernels().cml_kmeans_prune_gate(count.data_ptr(), int(cap), flags.data_ptr(),
                                                          mode.data_ptr(), _ptr(backoff), int(nback),
                                                          _native.stream_ptr(stream)), "kmeans_prune_gate")


def converge_latch(shift2: torch.Tensor, k: int, lim: float, flags: torch.Tensor, stream=None) -> None:
    """flags[1] = 1 once every shift2[j] (f64 squared centre moves) is <= lim (latched). Device only."""
    _native.check(_native.kernels().cml_kmeans_converge_latch(shift2.data_ptr(), int(k), float(lim),
                                                              flags.data_ptr(), _native.stream_ptr(stream)),
                  "kmeans_converge_latch")


def cond_copy(dst: torch.Tensor, src: torch.Tensor, flags: torch.Tensor, stream=None,
              dst_always: torch.Tensor | None = None) -> None:
    """dst <- src (same size, contiguous) unless flags[1] is set; ``dst_always`` <- src in the same launch.
    Device only."""
    nb = src.numel() * src.element_size()
    for t in (dst, dst_always):
        if t is not None and (t.numel() * t.element_size() != nb or not t.is_contiguous()):
            raise ValueError("cond_copy: contiguous tensors of the same size")
    if not src.is_contiguous():
        raise ValueError("cond_copy: contiguous source")
    _native.check(_native.kernels().cml_kmeans_cond_copy(dst.data_ptr(), src.data_ptr(), nb, flags.data_ptr(),
                                                         _ptr(dst_always), _native.stream_ptr(stream)),
                  "kmeans_cond_copy")


def centre_stats(cb: torch.Tensor, cb_old: torch.Tensor | None, k: int, d: int, mx: torch.Tensor, tau: float,
                 cn: torch.Tensor, half: torch.Tensor, drift: torch.Tensor, thr: torch.Tensor, dmax: torch.Tensor,
                 mc: torch.Tensor, c2: torch.Tensor, count: torch.Tensor, force: torch.Tensor, stream=None,
                 cum: torch.Tensor | None = None, backoff: torch.Tensor | None = None) -> None:
    """Centre statistics of the device pruned step (``kmeans_prune.hip``) over the bf16 centres: norms,
    drifts against ``cb_old`` (None: no drift), half nearest-centre distances -> thr, dmax, mc, c2;
    resets ``count`` and ``force``. No host synchronisation."""
    _native.check(_native.kernels().cml_kmeans_centre_stats(
        cb.data_ptr(), _ptr(cb_old), cb.stride(0), int(k), int(d), mx.data_ptr(), float(tau), cn.data_ptr(),
        half.data_ptr(), drift.data_ptr(), thr.data_ptr(), dmax.data_ptr(), mc.data_ptr(), c2.data_ptr(),
        count.data_ptr(), force.data_ptr(), _ptr(cum), _ptr(backoff), _native.stream_ptr(stream)),
        "kmeans_centre_stats")


def mx_probe(a: torch.Tensor, b: torch.Tensor, sa: torch.Tensor, sb: torch.Tensor) -> torch.Tensor:
    """One v_mfma_scale_f32_16x16x128_f8f6f4 (kmeans_mx.hip, a layout/precision probe for tests):
    out[i, j] = sum_k a[i, k]·b[j, k] with the E8M0 scale of lane l (row l % 16, k block l // 16) from
    ``sa``/``sb`` (int32 [64]). a, b: uint8 e4m3fn bytes [16, 128]."""
    if a.shape != (16, 128) or b.shape != (16, 128) or sa.numel() != 64 or sb.numel() != 64:
        raise ValueError("mx_probe: a, b [16, 128] e4m3 bytes, sa, sb [64] int32")
    out = torch.empty((16, 16), dtype=torch.float32, device=a.device)
    _native.check(_native.kernels().cml_mx_probe(a.contiguous().data_ptr(), b.contiguous().data_ptr(),
                                                 sa.to(torch.int32).contiguous().data_ptr(),
                                                 sb.to(torch.int32).contiguous().data_ptr(), out.data_ptr(),
                                                 _native.stream_ptr(None)), "mx_probe")
    return out


def mx_snap(cb: torch.Tensor, kc: int, dp: int, cnorm: torch.Tensor, cn64: torch.Tensor | None = None,
            cb_old: torch.Tensor | None = None, drift: torch.Tensor | None = None, stream=None) -> None:
    """Centres of an fp8 engine onto the MX grid, in place (kmeans_mx.hip kmeans_mx_snap_kernel): each
    32-element block of a bf16 row becomes its exact two-term e4m3 split (the MX assign's operand), with
    cnorm (and cn64, drift against cb_old when given) recomputed from the snapped rows."""
    _native.check(_native.kernels().cml_kmeans_mx_snap(cb.data_ptr(), cb.stride(0), int(kc), int(dp),
                                                      cnorm.data_ptr(), _ptr(cn64), _ptr(cb_old), _ptr(drift),
                                                      _native.stream_ptr(stream)), "kmeans_mx_snap")


def set_fp8_mx(on: bool) -> bool:
    """MX-scaled fp8 MFMA arithmetic for the fp8 K9r passes (default on; CML_KMEANS_FP8_MX=0: the bf16
    widening pass). Returns the previous setting. Engines created while it is on keep their centres on the
    MX grid (mx_snap)."""
    return bool(_native.kernels().cml_kmeans_set_fp8_mx(int(bool(on))))


def fp8_mx_on() -> bool:
    lib = _native.kernels()
    _apply_env_knobs(lib)
    return bool(lib.cml_kmeans_set_fp8_mx(-1))


def mx_applies(x: torch.Tensor) -> bool:
    """Whether the fp8 assign passes on ``x`` run MX arithmetic (fp8 rows on the GPU, toggle on)."""
    return x.is_cuda and is_fp8(x) and fp8_mx_on()


def assign_rr_ext(mode: int, x: torch.Tensor, n: int, dp: int, cb: torch.Tensor, cnorm: torch.Tensor,
                  plan: AssignPlan, xnorm: torch.Tensor, labels: torch.Tensor, cost_part: torch.Tensor | None,
                  ub: torch.Tensor, lb: torch.Tensor, mc: torch.Tensor, tau: float,
                  hist: torch.Tensor | None = None, rank: torch.Tensor | None = None,
                  delta: "DeltaState | None" = None, idx: torch.Tensor | None = None,
                  n_dev: torch.Tensor | None = None, lab_in: torch.Tensor | None = None,
                  gate: torch.Tensor | None = None, want: int = 0, stream=None,
                  best: torch.Tensor | None = None, cum: torch.Tensor | None = None,
                  merge_cost: torch.Tensor | None = None, merge_near: torch.Tensor | None = None,
                  merge_off: int = 0) -> None:
    """K9r with the pruned-step extensions (``kmeans_rr.h``): ``mode`` 1 assigns every row and writes
    the top-2 bounds ``ub``/``lb``; ``mode`` 2 assigns the candidate positions (rows ``idx``, count
    ``n_dev`` on the device; ``xnorm``/``lab_in`` compacted) — labels and bounds land at the real
    rows. ``delta`` logs label changes; ``gate``/``want`` make the launch conditional on a device flag;
    ``best`` (f32, real rows) receives the squared distance to the new label; ``merge_cost``/``merge_near``
    (mode 2, f32/int32 per real row) take the k-means|| merge: strictly nearer rows get (distance, label +
    ``merge_off``)."""
    if plan.rr_ct <= 0 or plan.kc != plan.kp:
        raise ValueError("the pruned-step assign needs the K9r plan (Dp in {128, 256, 512}, k <= 256)")
    _native.check(_native.kernels().cml_kmeans_assign_rr_ext(
        int(mode), x.data_ptr(), int(n), x.stride(0), int(dp), cb.data_ptr(), cb.stride(0), plan.kc, plan.kp,
        cnorm.data_ptr(), xnorm.data_ptr(), labels.data_ptr(), _ptr(cost_part), _ptr(hist), _ptr(rank),
        plan.grid, int(is_fp8(x)),
        _ptr(delta.rows if delta is not None else None), _ptr(delta.old if delta is not None else None),
        _ptr(delta.wg_count if delta is not None else None), _ptr(delta.overflow if delta is not None else None),
        delta.pcap if delta is not None else 0, plan.rr_ct, _ptr(idx), _ptr(n_dev), _ptr(lab_in), ub.data_ptr(),
        lb.data_ptr(), mc.data_ptr(), float(tau), _ptr(gate), int(want), _ptr(best), _ptr(cum),
        int(cum.shape[0] // 2) if cum is not None else 0, _ptr(merge_cost), _ptr(merge_near), int(merge_off),
        _native.stream_ptr(stream)),
        f"kmeans_assign_rr_ext(mode={mode})")


def init_classify(cost: torch.Tensor, near: torch.Tensor, xn: torch.Tensor, pn: torch.Tensor, tab_v: torch.Tensor,
                  tau: float, n: int, lmax: int, list_a: torch.Tensor, cnt_a: torch.Tensor, list_b: torch.Tensor,
                  cnt_b: torch.Tensor, stream=None) -> None:
    """Pruned k-means|| pass, step 1 (kmeans.hip init_classify_kernel): rows with no relevant new
    candidate are dropped, rows with at most ``lmax`` go to ``list_a`` as int32 [n, 4] entries (row,
    nearest candidate, reach and cost as f32 bits), the others to ``list_b`` (row ids; counters zeroed
    by the caller, lists of capacity n)."""
    if list_a.dtype != torch.int32 or list_a.numel() < 4 * n:
        raise ValueError("list_a: int32 [n, 4] entries")
    m = int(tab_v.shape[1])
    _native.check(_native.kernels().cml_kmeans_init_classify(
        cost.data_ptr(), near.data_ptr(), xn.data_ptr(), pn.data_ptr(), tab_v.data_ptr(), m, float(tau), int(n),
        int(lmax), list_a.data_ptr(), cnt_a.data_ptr(), list_b.data_ptr(), cnt_b.data_ptr(),
        _native.stream_ptr(stream)), "kmeans_init_classify")


def unique_rows(P: torch.Tensor):
    """``torch.unique(P, dim=0, return_inverse=True)`` for a device f64 [m, d] matrix in two launches
    (kmeans_init_table.hip: pairwise row comparisons, one block per row) and one host read of the distinct
    count. Same sorted order and inverse as torch's; host tensors, and more than 8192 rows (the pairwise
    passes are O(m²)), fall back to torch."""
    if not P.is_cuda or P.dim() != 2 or P.shape[0] == 0 or P.shape[0] > 8192:
        return torch.unique(P, dim=0, return_inverse=True)
    P = P.to(torch.float64).contiguous()
    m, d = int(P.shape[0]), int(P.shape[1])
    dup = torch.empty(m, dtype=torch.int32, device=P.device)
    inv = torch.empty(m, dtype=torch.int64, device=P.device)
    uniq = torch.empty((m, d), dtype=torch.float64, device=P.device)
    count = torch.zeros(1, dtype=torch.int32, device=P.device)
    _native.check(_native.kernels().cml_kmeans_unique_rows(P.data_ptr(), m, d, dup.data_ptr(), inv.data_ptr(),
                                                           uniq.data_ptr(), count.data_ptr(), _native.stream_ptr()),
                  "kmeans_unique_rows")
    return uniq[: int(count.item())], inv


def init_table(P: torch.Tensor, Y: torch.Tensor, stream=None):
    """The pruned k-means|| pass's table in one launch (kmeans_init_table.hip): (f32 [mp, m] distances from
    every existing candidate to the new ones, rounded down and sorted ascending; int32 [mp, m] their
    indices; f32 [mp] squared norms rounded up). None when m exceeds the kernel's 1024."""
    mp, d = int(P.shape[0]), int(P.shape[1])
    m = int(Y.shape[0])
    if m > 1024 or not P.is_cuda:
        return None
    P = P.to(torch.float64).contiguous()
    Y = Y.to(torch.float64).contiguous()
    tab_v = torch.empty((mp, m), dtype=torch.float32, device=P.device)
    tab_j = torch.empty((mp, m), dtype=torch.int32, device=P.device)
    pn32 = torch.empty(mp, dtype=torch.float32, device=P.device)
    lib = _native.kernels()
    # the coalesced two-rows-per-workgroup form (kmeans_init_fast.hip) where its LDS fits, else the first one
    if d <= 2048:  # the transposed, coalesced form (kmeans_init_fast.hip) where its LDS fits
        YT = Y.t().contiguous()
        _native.check(lib.cml_kmeans_pair_table(P.data_ptr(), mp, YT.data_ptr(), m, d, tab_v.data_ptr(),
                                                tab_j.data_ptr(), pn32.data_ptr(), _native.stream_ptr(stream)),
                      "kmeans_pair_table")
    else:
        _native.check(lib.cml_kmeans_init_table(P.data_ptr(), mp, Y.data_ptr(), m, d, tab_v.data_ptr(),
                                                tab_j.data_ptr(), pn32.data_ptr(), _native.stream_ptr(stream)),
                      "kmeans_init_table")
    return tab_v, tab_j, pn32


def gather_rank_rows(x: torch.Tensor, ids: torch.Tensor, cnt: torch.Tensor, cap: int, d: int, dest: torch.Tensor,
                     pad_rows: int = 0, stream=None) -> bool:
    """dest[rank(i)] = f64(x[ids[i], :d]) for the first min(cnt, cap) sampled ids (distinct; rank = position
    in ascending id order): a k-means|| round's candidate rows in row order, widened, without a sort pass
    or a host read of the count (kmeans_init_fast.hip). Rows [count, pad_rows) are zeroed. False (nothing
    launched) when cap exceeds the kernel's LDS list; the caller then sorts and gathers itself."""
    lib = _native.kernels()
    if cap > int(lib.cml_kmeans_gather_rank_max()) or dest.dtype != torch.float64 or dest.stride(1) != 1 \
            or dest.stride(0) != d or ids.dtype != torch.int32:
        return False
    ldx = x.stride(0) * x.element_size()
    grid = max(1, min(1024, -(-max(cap, pad_rows, 1) // 4)))
    _native.check(lib.cml_kmeans_gather_rank_rows(x.data_ptr(), int(ldx), int(is_fp8(x)), int(d), ids.data_ptr(),
                                                  cnt.data_ptr(), int(cap), dest.data_ptr(), int(pad_rows), grid,
                                                  _native.stream_ptr(stream)), "kmeans_gather_rank_rows")
    return True


def seed_table(U: torch.Tensor, cb: torch.Tensor, k: int, stream=None):
    """(a int32, d1 f32, d2 f32, pn f32) per distinct init candidate (rows of U, f64): its nearest centre of
    the bf16 centres ``cb`` (ties: lowest index), the distances to it and to the second nearest by direct
    differences in f64 rounded up / down, and ||U_i||² rounded up — the first Lloyd step's seed tables
    (kmeans_init_fast.hip seed_table_kernel)."""
    m, d = int(U.shape[0]), int(U.shape[1])
    U = U.to(torch.float64).contiguous()
    dev = U.device
    a = torch.empty(max(m, 1), dtype=torch.int32, device=dev)
    d1 = torch.empty(max(m, 1), dtype=torch.float32, device=dev)
    d2 = torch.empty(max(m, 1), dtype=torch.float32, device=dev)
    pn = torch.empty(max(m, 1), dtype=torch.float32, device=dev)
    _native.check(_native.kernels().cml_kmeans_seed_table(U.data_ptr(), m, d, cb.data_ptr(), cb.stride(0), int(k),
                                                          a.data_ptr(), d1.data_ptr(), d2.data_ptr(), pn.data_ptr(),
                                                          _native.stream_ptr(stream)), "kmeans_seed_table")
    return a, d1, d2, pn


def init_near_list(x: torch.Tensor, dp: int, cost: torch.Tensor, near: torch.Tensor, xn: torch.Tensor,
                   pn: torch.Tensor, tab_v: torch.Tensor, tab_j: torch.Tensor, y: torch.Tensor, off: int, tau: float,
                   lst: torch.Tensor, cnt: torch.Tensor, n_cap: int, stream=None) -> None:
    """Pruned k-means|| pass, step 2: the relevant new candidates of every ``lst`` row (y: bf16 [m, dp])."""
    m = int(tab_v.shape[1])
    _native.check(_native.kernels().cml_kmeans_init_near_list(
        x.data_ptr(), x.stride(0), int(dp), int(is_fp8(x)), cost.data_ptr(), near.data_ptr(), xn.data_ptr(),
        pn.data_ptr(), tab_v.data_ptr(), tab_j.data_ptr(), m, y.data_ptr(), int(off), float(tau), lst.data_ptr(),
        cnt.data_ptr(), int(n_cap), _native.stream_ptr(stream)), "kmeans_init_near_list")


def init_merge_list(cost: torch.Tensor, near: torch.Tensor, best: torch.Tensor, lab: torch.Tensor, off: int,
                    lst: torch.Tensor, cnt: torch.Tensor, n_cap: int, stream=None) -> None:
    """cost/near of the ``lst`` rows <- best/lab+off where best < cost."""
    _native.check(_native.kernels().cml_kmeans_init_merge_list(
        cost.data_ptr(), near.data_ptr(), best.data_ptr(), lab.data_ptr(), int(off), lst.data_ptr(), cnt.data_ptr(),
        int(n_cap), _native.stream_ptr(stream)), "kmeans_init_merge_list")


def prune_lower(dist: torch.Tensor, lab: torch.Tensor, xn: torch.Tensor, mc: float, tau: float,
                out: torch.Tensor, stream=None) -> None:
    """K9p lower bounds (``kmeans_prune.hip``) from a [m, k] f32 block of |c_j|² - 2 x·c_j:
    out = sqrt(max(min_{j != lab} dist + xn - tau·(xn + mc), 0)), rounded down."""
    m, k = dist.shape
    _native.check(_native.kernels().cml_kmeans_prune_lower(
        dist.data_ptr(), int(k), lab.data_ptr(), xn.data_ptr(), float(mc), float(tau), int(m), out.data_ptr(),
        _native.stream_ptr(stream)), "kmeans_prune_lower")


def seg_buffer_ints(k: int) -> int:
    return int(_native.kernels().cml_kmeans_seg_ints(k))


def update_centers(msgs: torch.Tensor | None, k: int, d: int, cent: torch.Tensor, cb: torch.Tensor, dp: int,
                   kp: int, cnorm: torch.Tensor, shift2: torch.Tensor | None, stream=None, unit: float = 1.0,
                   snap: bool = False) -> None:
    """K11: cent <- Σx·unit/count (empty clusters keep their centre), cb <- bf16(cent), cnorm <- ||cb||²;
    ``unit`` is the sum grid step (accumulate_sort ``qscale`` = 1/unit), 1 for plain sums. ``snap``: cb
    then goes onto the MX grid (mx_snap; the fp8 engines)."""
    lib = _native.kernels()
    if msgs is not None:
        nbuf, bstride, mp = msgs.shape[0], msgs.stride(0), msgs.data_ptr()
    else:
        nbuf, bstride, mp = 0, 0, 0
    status = lib.cml_kmeans_update(mp, nbuf, bstride, k, d, cent.data_ptr(), cb.data_ptr(), cb.stride(0), dp, kp,
                                   cnorm.data_ptr(), shift2.data_ptr() if shift2 is not None else 0, float(unit),
                                   _native.stream_ptr(stream))
    _native.check(status, "kmeans_update")
    if snap:
        mx_snap(cb, k, dp, cnorm, stream=stream)


# ----------------------------------------------------------------------------------------------
# CPU reference implementations (torch, float64) — identical semantics, used by local[n] mode.
# ----------------------------------------------------------------------------------------------

def exact_assign(x: torch.Tensor, centers: torch.Tensor, labels: torch.Tensor | None = None,
                 changed: torch.Tensor | None = None, stream=None, idx: torch.Tensor | None = None,
                 n_dev: torch.Tensor | None = None, best: torch.Tensor | None = None):
    """(labels int32, squared distance f64) of device f32/f64 rows against f64 centres in f64
    (``kmeans_exact.hip``): the source-precision assignment (ties: lowest centre index). With ``idx`` /
    ``n_dev`` (int32 row list, device count) only the listed rows are assigned, into ``labels`` /
    ``best`` at their real positions."""
    n, d = int(x.shape[0]), int(centers.shape[1])
    if x.dtype not in (torch.float32, torch.float64):
        x = x.to(torch.float64)
    if x.stride(-1) != 1:
        x = x.contiguous()
    c = centers.to(device=x.device, dtype=torch.float64).contiguous()
    lab = labels if labels is not None else torch.zeros(max(n, 1), dtype=torch.int32, device=x.device)
    if best is None:
        best = torch.empty(max(n, 1), dtype=torch.float64, device=x.device)
    _native.check(_native.kernels().cml_kmeans_exact_assign(
        x.data_ptr(), int(x.dtype == torch.float64), n, x.stride(0), d, c.data_ptr(), int(c.shape[0]),
        lab.data_ptr(), best.data_ptr(), _ptr(changed), _ptr(idx), _ptr(n_dev), _native.stream_ptr(stream)),
        "kmeans_exact_assign")
    return lab[:n], best[:n]


def exact_dist(x: torch.Tensor, centers: torch.Tensor, labels: torch.Tensor, best: torch.Tensor, lab_off: int = 0,
               stream=None) -> None:
    """best[r] = f64 Σ_t (x_t - c_{labels[r] - lab_off, t})² with exact_assign's fold (same bits)."""
    n, d = int(x.shape[0]), int(centers.shape[1])
    c = centers.to(device=x.device, dtype=torch.float64).contiguous()
    if labels.dtype != torch.int32 or best.dtype != torch.float64:
        raise ValueError("exact_dist: int32 labels, f64 best")
    _native.check(_native.kernels().cml_kmeans_exact_dist(
        x.data_ptr(), int(x.dtype == torch.float64), n, x.stride(0), d, c.data_ptr(), int(c.shape[0]),
        labels.data_ptr(), int(lab_off), best.data_ptr(), _native.stream_ptr(stream)), "kmeans_exact_dist")


def to_bf16_err(x: torch.Tensor, d: int, ldo: int, stream=None):
    """(bf16 [n, ldo] zero-padded copy, f32 [n] upper bounds of ||x_r - bf16(x_r)||) of device f32/f64 rows."""
    n = int(x.shape[0])
    out = torch.empty((max(n, 1), ldo), dtype=torch.bfloat16, device=x.device)
    err = torch.empty(max(n, 1), dtype=torch.float32, device=x.device)
    _native.check(_native.kernels().cml_kmeans_to_bf16_err(
        x.data_ptr(), int(x.dtype == torch.float64), n, x.stride(0), int(d), out.data_ptr(), int(ldo), err.data_ptr(),
        _native.stream_ptr(stream)), "kmeans_to_bf16_err")
    return out[:n] if n else out[:0], err


def screen_cert(ub: torch.Tensor, lb: torch.Tensor, err: torch.Tensor, ecmax: torch.Tensor, n: int,
                lst: torch.Tensor, count: torch.Tensor, stream=None, u_out: torch.Tensor | None = None,
                l_out: torch.Tensor | None = None) -> None:
    """Append to ``lst`` the rows whose bf16-screen label is not certified (lb - ub <= 2·(err + ecmax));
    ``count`` (int32 [1], zeroed by the caller) receives their number. ``u_out`` / ``l_out`` (f32, may
    be ``ub`` / ``lb``): bounds of the real distance to the label / every other centre (ub + err + ecmax,
    lb - err - ecmax, rounded outward)."""
    if ecmax.dtype != torch.float64 or lst.dtype != torch.int32 or lst.numel() < n:
        raise ValueError("screen_cert: f64 ecmax, int32 list of n entries")
    _native.check(_native.kernels().cml_kmeans_screen_cert(
        ub.data_ptr(), lb.data_ptr(), err.data_ptr(), ecmax.data_ptr(), int(n), lst.data_ptr(), count.data_ptr(),
        _ptr(u_out), _ptr(l_out), _native.stream_ptr(stream)), "kmeans_screen_cert")


def to_bf16_split(x: torch.Tensor, d: int, ds: int, ldo: int, stream=None):
    """Split-screen copy of device f32/f64 rows: bf16 [n, ldo] = [hi | lo | hi] in ds-wide segments, and
    f32 [n] ||lo||, ||x - hi - lo||, ||x|| (rounded up) and ||x||² (the K9r row norm)."""
    n = int(x.shape[0])
    out = torch.empty((max(n, 1), ldo), dtype=torch.bfloat16, device=x.device)
    ea, eb, en, xn = (torch.empty(max(n, 1), dtype=torch.float32, device=x.device) for _ in range(4))
    _native.check(_native.kernels().cml_kmeans_to_bf16_split(
        x.data_ptr(), int(x.dtype == torch.float64), n, x.stride(0), int(d), int(ds), out.data_ptr(), int(ldo),
        ea.data_ptr(), eb.data_ptr(), en.data_ptr(), xn.data_ptr(), _native.stream_ptr(stream)), "kmeans_to_bf16_split")
    return (out[:n] if n else out[:0]), ea, eb, en, xn


def split_centres(C: torch.Tensor, ds: int, cb: torch.Tensor, cn: torch.Tensor) -> torch.Tensor:
    """Centres (f64 [k, d]) in the split screen's layout: cb[:k] = [c_hi | c_hi | c_lo] (bf16), cn[:k] =
    ||c||² (f32), the padding rows zero with an infinite norm; returns f64 [3] = {max ||c_lo||, max ||c||, max ||c - c_hi - c_lo||} (device)."""
    k, d = int(C.shape[0]), int(C.shape[1])
    ch = C.to(torch.bfloat16)
    r = C - ch.to(torch.float64)
    cl = r.to(torch.bfloat16)
    rc = r - cl.to(torch.float64)
    cb.zero_()
    cb[:k, :d] = ch
    cb[:k, ds:ds + d] = ch
    cb[:k, 2 * ds:2 * ds + d] = cl
    cn.fill_(float("inf"))  # padding centres never win (K11's convention)
    cn[:k] = (C * C).sum(1).to(torch.float32)
    return torch.stack([cl.to(torch.float64).norm(dim=1).max(), C.norm(dim=1).max(), rc.norm(dim=1).max()]) * (1 + 1e-9)


def screen_cert_split(ub, lb, ea, eb, en, cst, n: int, lst, count, u_out, l_out, stream=None) -> None:
    """The split screen's certificate (kmeans_exact.hip screen_cert_split_kernel)."""
    _native.check(_native.kernels().cml_kmeans_screen_cert_split(
        ub.data_ptr(), lb.data_ptr(), ea.data_ptr(), eb.data_ptr(), en.data_ptr(), cst.data_ptr(), int(n),
        lst.data_ptr(), count.data_ptr(), u_out.data_ptr(), l_out.data_ptr(), _native.stream_ptr(stream)),
        "kmeans_screen_cert_split")


def exact_sums(x: torch.Tensor, labels: torch.Tensor, k: int, d: int | None = None, stream=None,
               with_lo: bool = False, counts_int: bool = False):
    """Per-cluster sums [k, d] and counts [k] of device f32/f64 rows, correctly rounded: double-double
    accumulation over a stable label sort (fixed chunks, no atomics), so the result is the rounded exact
    sum — the host twin's bits whatever the order. ``with_lo`` also returns the remainders S_lo (S +
    S_lo = the exact sum; the rank fold adds them); ``counts_int`` returns int32 counts."""
    n = int(labels.shape[0])
    d = int(x.shape[1]) if d is None else d
    if x.dtype not in (torch.float32, torch.float64):
        x = x.to(torch.float64)
    lab = labels[:n]
    lab = lab if lab.dtype == torch.int32 and lab.is_contiguous() else lab.to(torch.int32).contiguous()
    counts = torch.zeros(k, dtype=torch.int32, device=x.device)
    seg = torch.zeros(k + 1, dtype=torch.int32, device=x.device)
    if k == 1:  # one cluster (sum_exact): the rows in order, no histogram or sort
        counts.fill_(n)
        seg[1] = n
        perm = torch.arange(max(n, 1), dtype=torch.int32, device=x.device)
    else:
        if n:
            int_hist(lab, n, k, counts)  # exact int32 counts, no host read (bincount syncs)
        seg[1:] = torch.cumsum(counts, 0, dtype=torch.int32)
        # stable sort of the int32 labels (fixed chunks of the sorted order)
        perm = torch.sort(lab, stable=True).indices.to(torch.int32) if n else torch.zeros(1, dtype=torch.int32,
                                                                                            device=x.device)
    lib = _native.kernels()
    nch = max(1, int(lib.cml_kmeans_exact_chunks(n)))
    slots = torch.empty(4 * nch * d, dtype=torch.float64, device=x.device)
    slot_c = torch.full((2 * nch,), -1, dtype=torch.int32, device=x.device)
    S = torch.zeros((k, d), dtype=torch.float64, device=x.device)
    S_lo = torch.zeros((k, d), dtype=torch.float64, device=x.device)
    _native.check(lib.cml_kmeans_exact_segsum(x.data_ptr(), int(x.dtype == torch.float64), x.stride(0), d,
                                              perm.data_ptr(), seg.data_ptr(), int(k), n, S.data_ptr(),
                                              S_lo.data_ptr(), slots.data_ptr(), slot_c.data_ptr(),
                                              _native.stream_ptr(stream)), "kmeans_exact_segsum")
    cnt = counts if counts_int else counts.to(torch.float64)
    return (S, cnt, S_lo) if with_lo else (S, cnt)


def exact_top2(x: torch.Tensor, centers: torch.Tensor, labels: torch.Tensor, ub: torch.Tensor, lb: torch.Tensor,
               idx: torch.Tensor | None = None, n_dev: torch.Tensor | None = None, best: torch.Tensor | None = None,
               moves: tuple | None = None, stream=None) -> None:
    """The exact fold assignment (exact_assign's bits) of every row, or of idx[0 .. n_dev), writing
    ``labels``, optional ``best`` and the f32 bounds ``ub`` / ``lb`` of the real distance to the label /
    to every other centre; ``moves`` = (rows, old, new, count) int32 lists receiving the label changes."""
    n, d = int(x.shape[0]), int(centers.shape[1])
    if n == 0:
        return
    c = centers.to(device=x.device, dtype=torch.float64).contiguous()
    if labels.dtype != torch.int32 or ub.dtype != torch.float32 or lb.dtype != torch.float32:
        raise ValueError("exact_top2: int32 labels, f32 bounds")
    if idx is not None and (idx.numel() < n or n_dev is None):
        raise ValueError("exact_top2: idx needs n entries and a device count")
    mr, mo, mn, mc = moves if moves is not None else (None, None, None, None)
    _native.check(_native.kernels().cml_kmeans_exact_top2(
        x.data_ptr(), int(x.dtype == torch.float64), n, x.stride(0), d, c.data_ptr(), int(c.shape[0]),
        labels.data_ptr(), _ptr(best), _ptr(idx), _ptr(n_dev), ub.data_ptr(), lb.data_ptr(), _ptr(mr), _ptr(mo),
        _ptr(mn), _ptr(mc), _native.stream_ptr(stream)), "kmeans_exact_top2")


def cert_stats(C: torch.Tensor, Cold: torch.Tensor, s: torch.Tensor, drift: torch.Tensor, dtop: torch.Tensor,
               zero: torch.Tensor | None = None, stream=None) -> None:
    """Half-separations ``s`` of the centres C, drifts ``drift`` = ||C - Cold|| and their top two
    (kmeans_cert.hip); zeroes the int32 ``zero`` buffer (the step's counters)."""
    k, d = int(C.shape[0]), int(C.shape[1])
    _native.check(_native.kernels().cml_kmeans_cert_stats(
        C.data_ptr(), Cold.data_ptr(), k, d, s.data_ptr(), drift.data_ptr(), dtop.data_ptr(), _ptr(zero),
        int(zero.numel()) if zero is not None else 0, _native.stream_ptr(stream)), "kmeans_cert_stats")


def cert_bounds(lab, u, l, drift, dtop, s, n: int, lst, count, stream=None) -> None:
    _native.check(_native.kernels().cml_kmeans_cert_bounds(
        lab.data_ptr(), u.data_ptr(), l.data_ptr(), drift.data_ptr(), dtop.data_ptr(), s.data_ptr(), int(n),
        lst.data_ptr(), count.data_ptr(), _native.stream_ptr(stream)), "kmeans_cert_bounds")


def cert_tighten(x: torch.Tensor, C: torch.Tensor, lab, u, l, s, la, na, lbst, nbst, stream=None,
                 xn: torch.Tensor | None = None, bxn: torch.Tensor | None = None,
                 blab: torch.Tensor | None = None) -> None:
    """List A -> tightened upper bounds; still unproven rows to list B (with ``xn``: their K9r norms and
    current labels compacted into ``bxn`` / ``blab`` beside it)."""
    n = int(x.shape[0])
    _native.check(_native.kernels().cml_kmeans_cert_tighten(
        x.data_ptr(), int(x.dtype == torch.float64), n, x.stride(0), int(C.shape[1]), C.data_ptr(), lab.data_ptr(),
        u.data_ptr(), l.data_ptr(), s.data_ptr(), la.data_ptr(), na.data_ptr(), lbst.data_ptr(), nbst.data_ptr(),
        _ptr(xn), _ptr(bxn), _ptr(blab), _native.stream_ptr(stream)), "kmeans_cert_tighten")


def split_centres_dev(C: torch.Tensor, ds: int, cb: torch.Tensor, cn: torch.Tensor, cst: torch.Tensor,
                      mc: torch.Tensor | None = None, stream=None) -> None:
    """split_centres in one kernel launch (cb [kp, ldc] bf16, cn [kp] f32, cst f64 [3]; mc f32 [1] = the
    largest centre norm)."""
    k, d = int(C.shape[0]), int(C.shape[1])
    _native.check(_native.kernels().cml_kmeans_split_centres(
        C.data_ptr(), k, int(cb.shape[0]), d, int(ds), cb.data_ptr(), cb.stride(0), cn.data_ptr(), cst.data_ptr(),
        _ptr(mc), _native.stream_ptr(stream)), "kmeans_split_centres")


def cert_list(lst, cnt, cap: int, blab, lab, u, l, ea, eb, en, cst, lc, nc, moves, stream=None) -> None:
    """List B after the split K9r candidate pass: certified rows keep their screened labels (moves logged),
    the rest go to list C with their old labels restored."""
    mr, mo, mn, mc = moves
    _native.check(_native.kernels().cml_kmeans_cert_list(
        lst.data_ptr(), cnt.data_ptr(), int(cap), blab.data_ptr(), lab.data_ptr(), u.data_ptr(), l.data_ptr(),
        ea.data_ptr(), eb.data_ptr(), en.data_ptr(), cst.data_ptr(), lc.data_ptr(), nc.data_ptr(), mr.data_ptr(),
        mo.data_ptr(), mn.data_ptr(), mc.data_ptr(), _native.stream_ptr(stream)), "kmeans_cert_list")


def cert_slices(k: int) -> int:
    return int(_native.kernels().cml_kmeans_cert_slices(int(k)))


def cert_moves(x: torch.Tensor, k: int, mv_row, mv_old, mv_new, m_dev, hist, seg, cursor, perm, P_hi, P_lo,
               S_hi, S_lo, cnt, stream=None, C_cur: torch.Tensor | None = None,
               C_next: torch.Tensor | None = None) -> None:
    """Apply the label moves to the double-double cluster sums S_hi / S_lo and the int32 counts; with
    ``C_next`` (one rank) also the centre update C_next = S_hi / count (an empty cluster keeps C_cur)."""
    n, d = int(x.shape[0]), int(S_hi.shape[1])
    _native.check(_native.kernels().cml_kmeans_cert_moves(
        x.data_ptr(), int(x.dtype == torch.float64), n, x.stride(0), d, int(k), mv_row.data_ptr(), mv_old.data_ptr(),
        mv_new.data_ptr(), m_dev.data_ptr(), hist.data_ptr(), seg.data_ptr(), cursor.data_ptr(), perm.data_ptr(),
        P_hi.data_ptr(), P_lo.data_ptr(), S_hi.data_ptr(), S_lo.data_ptr(), cnt.data_ptr(), _ptr(C_cur),
        _ptr(C_next), 0, _native.stream_ptr(stream)), "kmeans_cert_moves")


def sum_exact(v: torch.Tensor) -> torch.Tensor:
    """Correctly rounded sum of an f64 vector (double-double accumulation; a 0-d tensor on v's device): the
    same bits on the host and the device, whatever the order — the exact path's trainingCost."""
    v = v.reshape(-1).to(torch.float64).contiguous()
    n = int(v.shape[0])
    if n == 0:
        return torch.zeros((), dtype=torch.float64, device=v.device)
    if v.is_cuda:  # two launches (block partials in double-double, folded in block order)
        out = torch.empty(1, dtype=torch.float64, device=v.device)
        part = torch.empty(2 * 1024, dtype=torch.float64, device=v.device)
        _native.check(_native.kernels().cml_kmeans_sum_dd(v.data_ptr(), n, out.data_ptr(), part.data_ptr(),
                                                          _native.stream_ptr(None)), "kmeans_sum_dd")
        return out.reshape(())
    lab = torch.zeros(n, dtype=torch.int64, device=v.device)
    S, _ = sums_reference(v.reshape(n, 1), lab, 1)
    return S.reshape(())


def dd_fold(hi: torch.Tensor, lo: torch.Tensor) -> torch.Tensor:
    """Rounded sum over the leading (rank) axis of double-double values [W, ...], in rank order (TwoSum
    per step, exact while the values' exponents span < ~2^80): the same bits as one rank's sums."""
    h, l = hi[0].clone(), lo[0].clone()
    for w in range(1, int(hi.shape[0])):
        v = hi[w]
        s = h + v
        bb = s - h
        l = l + ((h - (s - bb)) + (v - bb))
        l = l + lo[w]
        h = s
    return h + l


def assign_reference(x: torch.Tensor, centers: torch.Tensor, chunk: int = 1 << 16):
    """Return (labels int64, min squared distance f64) with first-index tie breaking. Device f32/f64
    rows run the f64 kernel (exact_assign); host rows the torch f64 form."""
    if x.is_cuda:
        lab, best = exact_assign(x, centers)
        return lab.long(), best
    # host twin of the device kernel (same fold, same ties): CPU and GPU sessions label rows alike
    x = x.to(torch.float64)
    if x.stride(-1) != 1:
        x = x.contiguous()
    c = centers.to(torch.float64).contiguous()
    n = int(x.shape[0])
    labels = torch.empty(n, dtype=torch.int64)
    best = torch.empty(n, dtype=torch.float64)
    if n:
        r = _native.host().cml_exact_assign_host(x.data_ptr(), n, x.stride(0), int(c.shape[1]), c.data_ptr(),
                                                 int(c.shape[0]), labels.data_ptr(), best.data_ptr(),
                                                 max(1, torch.get_num_threads()))
        if r != 0:
            raise ValueError("assign_reference: invalid shapes")
    return labels, best


def _assign_reference_blas(x: torch.Tensor, centers: torch.Tensor, chunk: int = 1 << 16):
    """The BLAS (expansion) form of the f64 assignment, kept as a cross-check of the fold kernels."""
    x = x.to(torch.float64)
    c = centers.to(torch.float64)
    cn = (c * c).sum(1)
    labels = torch.empty(x.shape[0], dtype=torch.int64, device=x.device)
    best = torch.empty(x.shape[0], dtype=torch.float64, device=x.device)
    for s in range(0, x.shape[0], chunk):
        xb = x[s:s + chunk]
        sc = cn[None, :] - 2.0 * xb @ c.T
        m, i = sc.min(1)
        labels[s:s + chunk] = i
        best[s:s + chunk] = torch.clamp((xb * xb).sum(1) + m, min=0.0)
    return labels, best


def sums_reference(x: torch.Tensor, labels: torch.Tensor, k: int, with_lo: bool = False):
    """Correctly rounded per-cluster sums and counts (f64); ``with_lo`` adds the double-double remainders."""
    if x.is_cuda:
        return exact_sums(x, labels, k, with_lo=with_lo)
    x = x.to(torch.float64)
    if x.stride(-1) != 1:
        x = x.contiguous()
    n, d = int(x.shape[0]), int(x.shape[1])
    lab = labels.to(torch.int64).contiguous()
    S = torch.empty((k, d), dtype=torch.float64)
    S_lo = torch.empty((k, d), dtype=torch.float64)
    cnt = torch.empty(k, dtype=torch.float64)
    r = _native.host().cml_exact_sums_host(x.data_ptr(), n, x.stride(0), d, lab.data_ptr(), int(k), S.data_ptr(),
                                           cnt.data_ptr(), S_lo.data_ptr() if with_lo else 0)
    if r != 0:
        raise ValueError("sums_reference: labels outside [0, k)")
    return (S, cnt, S_lo) if with_lo else (S, cnt)


def _sums_reference_torch(x: torch.Tensor, labels: torch.Tensor, k: int):
    x = x.to(torch.float64)
    sums = torch.zeros(k, x.shape[1], dtype=torch.float64, device=x.device)
    sums.index_add_(0, labels, x)
    counts = torch.bincount(labels, minlength=k).to(torch.float64)
    return sums, counts
