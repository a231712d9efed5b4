"""Bindings of the GLM / feature-statistics kernels (K7, K8, K13, K15, K24 in glm.hip).

GPU tensors run the gfx950 kernels (no fallback); CPU tensors run torch float64
reference code with identical semantics.  All functions work on a rank-local
shard and return *partial* statistics; callers all-reduce them.
"""
from __future__ import annotations

import functools
from typing import Optional, Tuple

import torch

from .. import _native
from .._native import c_dbl, c_int, c_ll, c_vp
from ..utils.device import num_cus

_native.register_kernel_sigs({
    "cml_glm_grid": (c_int, [c_ll, c_int, c_int, c_int, c_int]),
    "cml_glm_set_logreg_unroll": (c_int, [c_int]),
    "cml_glm_set_moments_unroll": (c_int, [c_int]),
    "cml_glm_set_fp8_nch": (c_int, [c_int]),
    "cml_col_moments": (c_int, [c_vp, c_ll, c_ll, c_int, c_int, c_vp, c_vp, c_int, c_vp]),
    "cml_scale_apply": (c_int, [c_vp, c_ll, c_ll, c_int, c_int, c_vp, c_vp, c_int, c_vp, c_ll, c_int, c_int, c_vp]),
    "cml_logreg_grad": (c_int, [c_vp, c_ll, c_ll, c_int, c_int, c_vp, c_vp, c_vp, c_vp, c_int, c_vp, c_vp]),
    "cml_linear_predict": (c_int, [c_vp, c_ll, c_ll, c_int, c_int, c_vp, c_int, c_vp, c_int, c_vp]),
    "cml_gram": (c_int, [c_vp, c_ll, c_ll, c_int, c_int, c_vp, c_vp, c_vp, c_int, c_vp]),
    "cml_partial_colsum": (c_int, [c_vp, c_int, c_int, c_vp, c_vp]),
    "cml_multinomial_mfma_supported": (c_int, [c_int, c_int, c_int]),
    "cml_multinomial_mfma_grid": (c_int, [c_ll, c_int]),
    "cml_multinomial_mfma_dpad": (c_int, [c_int, c_int]),
    "cml_multinomial_mfma_set_mode": (c_int, [c_int]),
    "cml_multinomial_predict_lds": (c_ll, [c_int, c_int, c_int]),
    "cml_multinomial_predict": (c_int, [c_vp, c_ll, c_ll, c_int, c_int, c_int, c_vp, c_vp, c_vp, c_int, c_vp]),
    "cml_multinomial_mfma_grad": (c_int, [c_vp, c_ll, c_ll, c_int, c_int, c_int, c_vp, c_vp, c_vp, c_vp, c_int,
                                          c_vp]),
    "cml_glm_loss_grad": (c_int, [c_vp, c_ll, c_ll, c_int, c_int, c_vp, c_vp, c_vp, c_vp, c_int, c_int, c_vp]),
    "cml_sgd_update": (c_int, [c_vp, c_int, c_vp, c_vp, c_vp, c_vp, c_dbl, c_dbl, c_int, c_vp, c_vp, c_vp,
                               c_vp, c_ll, c_ll, c_vp]),
    "cml_multinomial_supported": (c_int, [c_int, c_int, c_int]),
    "cml_multinomial_grid": (c_int, [c_ll, c_int, c_int, c_int, c_int]),
    "cml_multinomial_grad": (c_int, [c_vp, c_ll, c_ll, c_int, c_int, c_int, c_vp, c_vp, c_vp, c_vp, c_int, c_vp]),
})

_CODE = {torch.bfloat16: 0, torch.float32: 1, torch.float64: 2, torch.float8_e4m3fn: 3}


def _prep(x: torch.Tensor) -> torch.Tensor:
    """Row-major with a 16-byte multiple row pitch (vector loads), supported dtype."""
    if x.dtype not in _CODE:
        x = x.to(torch.float64)
    if x.dim() == 1:
        x = x[:, None]
    if x.stride(1) != 1 or (x.stride(0) * x.element_size()) % 16 != 0 or x.data_ptr() % 16 != 0:
        per = 16 // x.element_size()
        ld = (x.shape[1] + per - 1) // per * per
        buf = torch.zeros((x.shape[0], ld), dtype=x.dtype, device=x.device)
        buf[:, : x.shape[1]] = x
        x = buf
    return x


_KIND = {"moments": 0, "logreg": 1, "predict": 2}


_UNROLL = [0]


def _grid(n: int, d: int, code: int, dev, kind: str) -> int:
    return _grid_cached(n, d, code, dev.index or 0, kind, _UNROLL[0])


@functools.lru_cache(maxsize=256)
def _grid_cached(n: int, d: int, code: int, dev_index: int, kind: str, unroll: int) -> int:
    g = _native.kernels().cml_glm_grid(n, d, code, num_cus(dev_index), _KIND[kind])
    if g < 0:
        raise ValueError(f"feature width {d} too large for the GLM kernels")
    return g


def moments(x: torch.Tensor, d: Optional[int] = None) -> Tuple[int, torch.Tensor, torch.Tensor]:
    """Local (count, shifted Σ, shifted Σ², shift) with shift = first row — merge with all-reduce."""
    d = x.shape[1] if d is None else d
    n = x.shape[0]
    if n == 0:
        z = torch.zeros(d, dtype=torch.float64, device=x.device)
        return 0, z, z.clone(), z.clone()
    shift = x[0, :d].to(torch.float64).contiguous()
    if not x.is_cuda:
        xs = x[:, :d].to(torch.float64) - shift
        return n, xs.sum(0), (xs * xs).sum(0), shift
    if x.dtype == torch.float8_e4m3fn and d > 512:  # exact bf16 copies of row chunks (e4m3 ⊂ bf16)
        s1 = torch.zeros(d, dtype=torch.float64, device=x.device)
        s2 = torch.zeros_like(s1)
        for r0 in range(0, n, 1 << 22):
            _, a, b, _ = _moments_kernel(x[r0:r0 + (1 << 22), :d].to(torch.bfloat16), d, shift)
            s1 += a
            s2 += b
        return n, s1, s2, shift
    _, s1, s2, _ = _moments_kernel(x, d, shift)
    return n, s1, s2, shift


def _moments_kernel(x: torch.Tensor, d: int, shift: torch.Tensor):
    n = x.shape[0]
    xx = _prep(x)
    code = _CODE[xx.dtype]
    g = _grid(n, d, code, xx.device, "moments")
    out = torch.empty((g, 2, d), dtype=torch.float64, device=xx.device)
    st = _native.kernels().cml_col_moments(xx.data_ptr(), n, xx.stride(0), d, code, shift.data_ptr(), out.data_ptr(),
                                           g, _native.stream_ptr())
    _native.check(st, "col_moments")
    s = out.sum(0)
    return n, s[0], s[1], shift


def scale_apply(x: torch.Tensor, d: int, mean: torch.Tensor, inv_std: torch.Tensor, with_mean: bool,
                out_dtype=torch.float64, out_width: Optional[int] = None) -> torch.Tensor:
    n = x.shape[0]
    width = d if out_width is None else out_width
    if not x.is_cuda:
        y = x[:, :d].to(torch.float64)
        if with_mean:
            y = y - mean
        y = y * inv_std
        if width > d:
            y = torch.nn.functional.pad(y, (0, width - d))
        if out_dtype == torch.float8_e4m3fn:
            y = y.clamp(-448.0, 448.0)
        return y.to(out_dtype)
    xx = _prep(x)
    out = torch.empty((n, width), dtype=out_dtype, device=x.device)
    if n == 0:
        return out
    st = _native.kernels().cml_scale_apply(xx.data_ptr(), n, xx.stride(0), d, _CODE[xx.dtype],
                                           mean.to(torch.float64).contiguous().data_ptr(),
                                           inv_std.to(torch.float64).contiguous().data_ptr(), int(with_mean),
                                           out.data_ptr(), out.stride(0), width, _CODE[out_dtype],
                                           _native.stream_ptr())
    _native.check(st, "scale_apply")
    return out


def logreg_grad(x: torch.Tensor, d: int, y: torch.Tensor, coef: torch.Tensor,
                weight: Optional[torch.Tensor] = None, batch: Optional[int] = None,
                row_base: Optional[torch.Tensor] = None):
    """Binomial logistic loss + gradient over the local shard.

    coef = [w (d) | b] in the ORIGINAL feature space.  Returns a float64 tensor
    [grad_w (d) | grad_b | loss | weight_sum] (sums, not means).
    With ``row_base`` (int64 device scalar) and ``batch``, the pass covers rows
    [row_base, row_base + batch) read at kernel run time — the form a captured SGD graph replays.
    """
    if row_base is not None:
        if not x.is_cuda:
            b0 = int(row_base.item())
            return logreg_grad(x[b0:b0 + batch], d, y[b0:b0 + batch], coef,
                               None if weight is None else weight[b0:b0 + batch])
        return _logreg_grad_dev(x, d, y, coef, weight, batch, row_base)
    n = x.shape[0]
    coef = coef.to(device=x.device, dtype=torch.float64).contiguous()
    if not x.is_cuda or n == 0:
        xf = x[:, :d].to(torch.float64)
        m = xf @ coef[:d] + coef[d]
        yy = y.to(torch.float64)
        ww = torch.ones_like(yy) if weight is None else weight.to(torch.float64)
        p = torch.sigmoid(m)
        r = ww * (p - yy)
        loss = (ww * (torch.nn.functional.softplus(m) - yy * m)).sum()
        return torch.cat([xf.T @ r, r.sum().reshape(1), loss.reshape(1), ww.sum().reshape(1)])
    xx = _prep(x)
    code = _CODE[xx.dtype]
    g = _grid(n, d, code, xx.device, "logreg")
    out = torch.empty((g, d + 3), dtype=torch.float64, device=xx.device)
    yy = y.to(torch.float64).contiguous()
    ww = weight.to(torch.float64).contiguous() if weight is not None else None
    st = _native.kernels().cml_logreg_grad(xx.data_ptr(), n, xx.stride(0), d, code, yy.data_ptr(),
                                           ww.data_ptr() if ww is not None else 0, coef.data_ptr(), out.data_ptr(),
                                           g, 0, _native.stream_ptr())
    _native.check(st, "logreg_grad")
    return partial_colsum(out)


_LOSS = {"logistic": 0, "hinge": 1, "squared": 2}


def loss_grad(x: torch.Tensor, d: int, y: torch.Tensor, coef: torch.Tensor, weight: Optional[torch.Tensor] = None,
              loss: str = "hinge") -> torch.Tensor:
    """K13 with a selectable per-row loss of the margin m = x·w + b: 'logistic' (= logreg_grad),
    'hinge' (LinearSVC; labels {0, 1} mapped to ±1) or 'squared' (½(m − y)²).  Returns the float64
    [grad_w (d) | grad_b | loss | weight_sum] sums of the local shard, X read once."""
    code_l = _LOSS[loss]
    n = x.shape[0]
    coef = coef.to(device=x.device, dtype=torch.float64).contiguous()
    if not x.is_cuda or n == 0:
        xf = x[:, :d].to(torch.float64)
        m = xf @ coef[:d] + coef[d]
        yy = y.to(torch.float64)
        ww = torch.ones_like(yy) if weight is None else weight.to(torch.float64)
        if code_l == 0:
            r = ww * (torch.sigmoid(m) - yy)
            lr = torch.nn.functional.softplus(m) - yy * m
        elif code_l == 1:
            ys = torch.where(yy > 0.5, 1.0, -1.0).to(torch.float64)
            t = 1.0 - ys * m
            r = torch.where(t > 0, -ww * ys, torch.zeros_like(t))
            lr = t.clamp(min=0.0)
        else:
            e = m - yy
            r = ww * e
            lr = 0.5 * e * e
        return torch.cat([xf.T @ r, r.sum().reshape(1), (ww * lr).sum().reshape(1), ww.sum().reshape(1)])
    xx = _prep(x)
    code = _CODE[xx.dtype]
    g = _grid(n, d, code, xx.device, "logreg")
    out = torch.empty((g, d + 3), dtype=torch.float64, device=xx.device)
    yy = y.to(torch.float64).contiguous()
    ww = weight.to(torch.float64).contiguous() if weight is not None else None
    st = _native.kernels().cml_glm_loss_grad(xx.data_ptr(), n, xx.stride(0), d, code, yy.data_ptr(),
                                             ww.data_ptr() if ww is not None else 0, coef.data_ptr(), out.data_ptr(),
                                             g, code_l, _native.stream_ptr())
    _native.check(st, "glm_loss_grad")
    return partial_colsum(out)


def multinomial_grad(x: torch.Tensor, d: int, y: torch.Tensor, coef: torch.Tensor,
                     weight: Optional[torch.Tensor] = None, chunk_rows: int = 1 << 20,
                     prefer_valu: bool = False) -> torch.Tensor:
    """Softmax (multinomial logistic) loss + gradient over the local shard: ``coef`` [C, d+1] (last column
    the intercepts) in the original feature space, labels 0..C-1 (f64). Returns the float64 sums
    [∇W (C·d, row-major) | ∇b (C) | loss | weight sum]. GPU rows run K13m's MFMA form for C <= 64 on bf16 rows
    with d <= 256, d % 8 == 0, and on e4m3 rows with d % 16 == 0 (widened exactly to bf16 as they are staged in
    LDS) (glm_mfma.hip: both products on
    v_mfma_f32_32x32x16_bf16 with the f32 operand — weights, residuals — split into three bf16 terms, so f32
    precision; ``set_multinomial_mfma_mode(1)`` selects the v_mfma_f32_32x32x2_f32 form), else the VALU kernel
    (multinomial_grad_kernel: X read once, gradient partials in f64, fixed-order reduction) where its layout fits
    (C <= 8, d up to 512; also ``prefer_valu=True``); otherwise — and on the CPU — row chunks in f64 (never an f64 copy of the whole X)."""
    C = int(coef.shape[0])
    n = int(x.shape[0])
    coef = coef.to(device=x.device, dtype=torch.float64).contiguous()
    if x.is_cuda and n > 0 and x.dtype in _CODE:
        xx = _prep(x)
        code = _CODE[xx.dtype]
        k = _native.kernels()
        cp = k.cml_multinomial_mfma_supported(d, code, C)
        if cp > 0 and not prefer_valu:
            # bf16 rows, d % 8 == 0, d <= 256: the MFMA form for every C <= 64 (at C = 4 and 8 too: 17.5 ms vs
            # 32 / 56 ms for the VALU kernel over 100M x 256, profiles/r6/multinomial_100Mx256_bf16.log)
            return _multinomial_mfma(xx, d, y, coef, weight, C, cp, int(k.cml_multinomial_mfma_dpad(d, C)))
        if k.cml_multinomial_supported(d, code, C) > 0:
            g = k.cml_multinomial_grid(n, d, code, C, num_cus(xx.device.index or 0))
            m = C * d + C + 2
            out = torch.empty((g, m), dtype=torch.float64, device=xx.device)
            yy = y.to(torch.float64).contiguous()
            ww = weight.to(torch.float64).contiguous() if weight is not None else None
            st = k.cml_multinomial_grad(xx.data_ptr(), n, xx.stride(0), d, code, C, yy.data_ptr(),
                                        ww.data_ptr() if ww is not None else 0, coef.data_ptr(), out.data_ptr(), g,
                                        _native.stream_ptr())
            _native.check(st, "multinomial_grad")
            return partial_colsum(out)
        if cp > 0:
            return _multinomial_mfma(xx, d, y, coef, weight, C, cp, int(k.cml_multinomial_mfma_dpad(d, C)))
    W, b = coef[:, :d], coef[:, d]
    gW = torch.zeros((C, d), dtype=torch.float64, device=x.device)
    gb = torch.zeros(C, dtype=torch.float64, device=x.device)
    loss = torch.zeros((), dtype=torch.float64, device=x.device)
    wsum = torch.zeros((), dtype=torch.float64, device=x.device)
    for r0 in range(0, n, chunk_rows):
        xf = x[r0:r0 + chunk_rows, :d].to(torch.float64)
        yl = y[r0:r0 + chunk_rows].to(torch.int64)
        ww = (weight[r0:r0 + chunk_rows].to(torch.float64) if weight is not None
              else torch.ones(xf.shape[0], dtype=torch.float64, device=x.device))
        mrg = xf @ W.T + b[None, :]
        lse = torch.logsumexp(mrg, 1)
        loss += (ww * (lse - mrg.gather(1, yl[:, None])[:, 0])).sum()
        R = torch.softmax(mrg, 1)
        R[torch.arange(R.shape[0], device=x.device), yl] -= 1.0
        R *= ww[:, None]
        gW += R.T @ xf
        gb += R.sum(0)
        wsum += ww.sum()
    return torch.cat([gW.reshape(-1), gb, loss.reshape(1), wsum.reshape(1)])


def multinomial_predict(x: torch.Tensor, d: int, coef: torch.Tensor):
    """K13t (glm_mfma.hip): the multinomial model's raw margins X·Wᵀ + b and softmax probabilities, f64 [n, C]
    each, in one pass over bf16 / f32 GPU rows (f64 MFMAs; d <= 256, C <= 64). None where unsupported (the
    caller's f64 chunk path then runs)."""
    if not x.is_cuda or x.dtype not in (torch.bfloat16, torch.float32) or x.dim() != 2:
        return None
    C = int(coef.shape[0])
    code = _CODE[x.dtype]
    k = _native.kernels()
    if k.cml_multinomial_predict_lds(d, code, C) <= 0:
        return None
    xx = _prep(x)
    n = int(xx.shape[0])
    cf = coef.to(device=x.device, dtype=torch.float64).contiguous()
    raw = torch.empty((n, C), dtype=torch.float64, device=x.device)
    prob = torch.empty((n, C), dtype=torch.float64, device=x.device)
    _native.check(k.cml_multinomial_predict(xx.data_ptr(), n, xx.stride(0), d, code, C, cf.data_ptr(), raw.data_ptr(),
                                            prob.data_ptr(), num_cus(x.device.index or 0), _native.stream_ptr()),
                  "multinomial_predict")
    return raw, prob


def set_multinomial_mfma_mode(mode: int) -> int:
    """K13m MFMA form: 0 = bf16 three-term products (default; C <= 16 on a 16-class tile of 16x16x32 MFMAs),
    1 = f32 MFMAs, 2 = bf16 with W split in registers on every use, 3 = mode 0 on 32-class tiles of 32x32x16
    MFMAs for every C (A/B). Returns the previous mode."""
    return int(_native.kernels().cml_multinomial_mfma_set_mode(int(mode)))


def _multinomial_mfma(xx: torch.Tensor, d: int, y: torch.Tensor, coef: torch.Tensor, weight, C: int, cp: int,
                      dp: int) -> torch.Tensor:
    """K13m on MFMA (glm_mfma.hip) -> [∇W (C·d) | ∇b (C) | loss | weight sum], the layout of multinomial_grad."""
    n = int(xx.shape[0])
    k = _native.kernels()
    g = k.cml_multinomial_mfma_grid(n, num_cus(xx.device.index or 0))
    out = torch.empty((g, cp * dp + C + 2), dtype=torch.float64, device=xx.device)
    yy = y.to(torch.float64).contiguous()
    ww = weight.to(torch.float64).contiguous() if weight is not None else None
    _native.check(k.cml_multinomial_mfma_grad(xx.data_ptr(), n, xx.stride(0), d, _CODE[xx.dtype], C, yy.data_ptr(),
                                              ww.data_ptr() if ww is not None else 0, coef.data_ptr(), out.data_ptr(),
                                              g, _native.stream_ptr()), "multinomial_mfma_grad")
    msg = partial_colsum(out)
    return torch.cat([msg[: cp * dp].view(cp, dp)[:C, :d].reshape(-1), msg[cp * dp:]])


def _logreg_grad_dev(x, d, y, coef, weight, batch, row_base):
    """Device-offset variant: no host read of the batch position (capturable)."""
    xx = _prep(x)
    code = _CODE[xx.dtype]
    coef = coef.to(device=x.device, dtype=torch.float64).contiguous()
    g = _grid(batch, d, code, xx.device, "logreg")
    out = torch.empty((g, d + 3), dtype=torch.float64, device=xx.device)
    if y.dtype != torch.float64 or not y.is_contiguous():
        raise ValueError("device-offset logreg_grad needs float64 contiguous labels")
    st = _native.kernels().cml_logreg_grad(xx.data_ptr(), batch, xx.stride(0), d, code, y.data_ptr(),
                                           weight.data_ptr() if weight is not None else 0, coef.data_ptr(),
                                           out.data_ptr(), g, row_base.data_ptr(), _native.stream_ptr())
    _native.check(st, "logreg_grad")
    return partial_colsum(out)


def partial_colsum(part: torch.Tensor) -> torch.Tensor:
    """K13b: column sums of the [grid, m] float64 per-block partials, fixed order (deterministic)."""
    if not part.is_cuda:
        return part.sum(0)
    part = part.contiguous()
    nb, m = part.shape
    msg = torch.empty(m, dtype=torch.float64, device=part.device)
    st = _native.kernels().cml_partial_colsum(part.data_ptr(), nb, m, msg.data_ptr(), _native.stream_ptr())
    _native.check(st, "partial_colsum")
    return msg


def sgd_update(msg: torch.Tensor, d: int, coef: torch.Tensor, vel: torch.Tensor, eff: torch.Tensor,
               lr: torch.Tensor, momentum: float, l2: float, fit_intercept: bool,
               gscale: Optional[torch.Tensor], kscale: Optional[torch.Tensor], loss_acc: torch.Tensor,
               base: torch.Tensor, batch: int, wrap: int) -> None:
    """K14: one momentum-SGD step from the all-reduced [grad_w | grad_b | loss | Σw] message, in place:
    vel = μ·vel − lr·(msg/Σw ⊙ gscale + l2·w), coef += vel, eff = coef ⊙ kscale,
    loss_acc += loss/Σw, base = (base + batch) mod wrap.  All device scalars; nothing syncs."""
    if not coef.is_cuda:
        wsum = msg[d + 2].clamp(min=1e-300)
        g = msg[: d + 1] / wsum
        if gscale is not None:
            g = g * gscale
        if l2 > 0:
            g = g + torch.cat([l2 * coef[:d], coef.new_zeros(1)])
        if not fit_intercept:
            g = torch.cat([g[:d], g.new_zeros(1)])
        vel.mul_(momentum).sub_(g * lr)
        coef.add_(vel)
        eff.copy_(coef if kscale is None else coef * kscale)
        loss_acc.add_(msg[d + 1] / wsum)
        base.add_(batch).remainder_(wrap)
        return
    for t in (msg, coef, vel, eff):
        if t.dtype != torch.float64 or not t.is_contiguous():
            raise ValueError("sgd_update needs contiguous float64 state")
    ptr = lambda t: 0 if t is None else t.data_ptr()  # noqa: E731
    st = _native.kernels().cml_sgd_update(msg.data_ptr(), d, coef.data_ptr(), vel.data_ptr(), eff.data_ptr(),
                                          lr.data_ptr(), float(momentum), float(l2), int(bool(fit_intercept)),
                                          ptr(gscale), ptr(kscale), loss_acc.data_ptr(), base.data_ptr(), int(batch),
                                          int(wrap), _native.stream_ptr())
    _native.check(st, "sgd_update")


def linear_predict(x: torch.Tensor, d: int, coef: torch.Tensor, link: str = "identity") -> torch.Tensor:
    n = x.shape[0]
    coef = coef.to(device=x.device, dtype=torch.float64).contiguous()
    if not x.is_cuda or n == 0:
        m = x[:, :d].to(torch.float64) @ coef[:d] + coef[d]
        return torch.sigmoid(m) if link == "logistic" else m
    xx = _prep(x)
    code = _CODE[xx.dtype]
    g = _grid(n, d, code, xx.device, "predict")
    out = torch.empty(n, dtype=torch.float64, device=xx.device)
    st = _native.kernels().cml_linear_predict(xx.data_ptr(), n, xx.stride(0), d, code, coef.data_ptr(),
                                              1 if link == "logistic" else 0, out.data_ptr(), g,
                                              _native.stream_ptr())
    _native.check(st, "linear_predict")
    return out


def gram(x: torch.Tensor, d: int, y: torch.Tensor, weight: Optional[torch.Tensor] = None) -> torch.Tensor:
    """[X 1 y]ᵀ W [X 1 y] (float64, (d+2)×(d+2), symmetric) of the local shard."""
    n = x.shape[0]
    m = d + 2
    if (not x.is_cuda) or d > 30 or n == 0:
        a = torch.cat([x[:, :d].to(torch.float64), torch.ones((n, 1), dtype=torch.float64, device=x.device),
                       y.to(torch.float64).reshape(-1, 1)], 1)
        if weight is not None:
            a = a * weight.to(torch.float64).sqrt().reshape(-1, 1)
        return a.T @ a
    xx = x if x.dtype in _CODE else x.to(torch.float64)
    if xx.stride(1) != 1:
        xx = xx.contiguous()
    grid = max(1, min((n + 2047) // 2048, num_cus(xx.device.index or 0) * 4))
    out = torch.zeros((grid, m * m), dtype=torch.float64, device=xx.device)
    yy = y.to(torch.float64).contiguous()
    ww = weight.to(torch.float64).contiguous() if weight is not None else None
    st = _native.kernels().cml_gram(xx.data_ptr(), n, xx.stride(0), d, _CODE[xx.dtype], yy.data_ptr(),
                                    ww.data_ptr() if ww is not None else 0, out.data_ptr(), grid,
                                    _native.stream_ptr())
    _native.check(st, "gram")
    g = out.sum(0).reshape(m, m)
    return torch.triu(g) + torch.triu(g, 1).T


def set_moments_unroll(u: int) -> None:
    """Ablation knob: K7 (column moments) rows in flight per wave (1, 2; 0 = automatic)."""
    _native.kernels().cml_glm_set_moments_unroll(int(u))


def set_logreg_unroll(u: int) -> None:
    """Force K13's rows-in-flight per wave (1 or 2; 0 = automatic) — for ablations."""
    _native.kernels().cml_glm_set_logreg_unroll(int(u))
    _UNROLL[0] = int(u)


def set_fp8_nch(v: int) -> None:
    """Ablation: 16-byte chunks per lane of the fp8 streaming layout (0 = auto)."""
    _native.kernels().cml_glm_set_fp8_nch(int(v))
