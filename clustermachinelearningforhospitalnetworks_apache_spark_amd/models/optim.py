"""Host-side optimizers for the GLMs (K14 in SURVEY.md §2.5).

The expensive part of every iteration — a full pass over the HBM-resident shard
computing loss and gradient — runs on the device (K13) and is all-reduced; the
optimizer itself works on a (d+1)-vector in float64 on the host, like Spark's
driver-side Breeze L-BFGS.
"""
from __future__ import annotations

from typing import Callable, List, Optional, Tuple

import numpy as np


def lbfgs(fg: Callable[[np.ndarray], Tuple[float, np.ndarray]], x0: np.ndarray, max_iter: int = 100,
          tol: float = 1e-6, m: int = 10, l1: Optional[np.ndarray] = None, state: Optional[dict] = None,
          on_iter: Optional[Callable[[int, dict], None]] = None,
          fault: Optional[str] = None) -> Tuple[np.ndarray, List[float], int]:
    """Minimise f with L-BFGS (OWL-QN when an L1 weight vector ``l1`` is given).

    Convergence (Breeze-style): relative improvement of f below ``tol`` over an
    iteration, or gradient norm below ``tol * max(1, |x|)``.
    Returns (x, objective history, iterations).

    Checkpointing: ``on_iter(it, state)`` runs after every completed iteration with the
    whole optimizer state (``lbfgs_state``: x, f, g, the s/y history, the objective history); passing such
    a state back as ``state`` resumes at the next iteration and retraces the uninterrupted run bit for bit
    (the state is everything an iteration reads). ``fault`` names a crash point (utils/fault.py) armed per
    iteration.
    """
    if state is not None:
        x, f, g = state["x"].copy(), float(state["f"]), state["g"].copy()
        S = [s.copy() for s in state["S"]]
        Y = [y.copy() for y in state["Y"]]
        hist = [float(v) for v in state["hist"]]
        start = int(state["it"]) + 1
    else:
        x = np.asarray(x0, dtype=np.float64).copy()
        f, g = fg(x)
        if l1 is not None:
            f += float(np.sum(l1 * np.abs(x)))
        hist = [f]
        S, Y = [], []
        start = 1
    it = start - 1
    if fault is not None:
        from ..utils.fault import maybe_fail
    for it in range(start, max_iter + 1):
        if fault is not None:
            maybe_fail(fault, it)
        pg = _pseudo_grad(x, g, l1) if l1 is not None else g
        if np.linalg.norm(pg) <= tol * max(1.0, np.linalg.norm(x)):
            it -= 1
            break
        d = -_two_loop(pg, S, Y)
        if l1 is not None:
            d = np.where(d * pg < 0, d, 0.0)  # orthant projection of the direction
        if float(d @ pg) >= 0:
            d = -pg
            S.clear()
            Y.clear()
        step = 1.0 if S else min(1.0, 1.0 / max(np.linalg.norm(pg), 1e-12))
        x_new, f_new, g_new, ok = _line_search(fg, x, f, pg, d, step, l1)
        if not ok:
            break
        s, yv = x_new - x, g_new - g
        if float(s @ yv) > 1e-12:
            S.append(s)
            Y.append(yv)
            if len(S) > m:
                S.pop(0)
                Y.pop(0)
        improvement = abs(f - f_new) / max(abs(f), abs(f_new), 1e-12)
        x, f, g = x_new, f_new, g_new
        hist.append(f)
        if improvement < tol:
            break
        if on_iter is not None:
            on_iter(it, {"x": x, "f": f, "g": g, "S": S, "Y": Y, "hist": hist, "it": it})
    return x, hist, it


def lbfgs_state_arrays(st: dict) -> dict:
    """An L-BFGS state as named numpy arrays (utils/checkpoint.py stores one .npy per array)."""
    n = int(st["x"].shape[0])
    return {"x": st["x"], "f": np.array([st["f"]]), "g": st["g"], "hist": np.asarray(st["hist"], dtype=np.float64),
            "it": np.array([st["it"]], dtype=np.int64),
            "S": np.asarray(st["S"], dtype=np.float64).reshape(-1, n),
            "Y": np.asarray(st["Y"], dtype=np.float64).reshape(-1, n)}


def lbfgs_state_from_arrays(a: dict) -> dict:
    return {"x": a["x"], "f": float(a["f"][0]), "g": a["g"], "hist": list(a["hist"]), "it": int(a["it"][0]),
            "S": list(a["S"]), "Y": list(a["Y"])}


def _two_loop(g, S, Y):
    q = g.copy()
    alphas = []
    for s, y in zip(reversed(S), reversed(Y)):
        rho = 1.0 / float(y @ s)
        a = rho * float(s @ q)
        alphas.append((rho, a))
        q -= a * y
    if S:
        q *= float(S[-1] @ Y[-1]) / float(Y[-1] @ Y[-1])
    for (s, y), (rho, a) in zip(zip(S, Y), reversed(alphas)):
        b = rho * float(y @ q)
        q += (a - b) * s
    return q


def _pseudo_grad(x, g, l1):
    pg = g + l1 * np.sign(x)
    zero = x == 0
    right = g + l1
    left = g - l1
    pg = np.where(zero, np.where(right < 0, right, np.where(left > 0, left, 0.0)), pg)
    return pg


def _line_search(fg, x, f, g, d, step, l1, c1=1e-4, max_ls=30):
    """Backtracking Armijo line search (with orthant projection for OWL-QN)."""
    gd = float(g @ d)
    for _ in range(max_ls):
        xn = x + step * d
        if l1 is not None:
            xn = np.where(np.sign(xn) * np.sign(x) < 0, 0.0, xn)
        fn, gn = fg(xn)
        if l1 is not None:
            fn += float(np.sum(l1 * np.abs(xn)))
        if fn <= f + c1 * step * gd or (l1 is not None and fn < f):
            return xn, fn, gn, True
        step *= 0.5
    return x, f, None, False
