"""Tracing and timing (the reference has none).

* ``trace(name)`` / ``@traced(name)``: a roctx range (``librocprofiler-sdk-roctx``) around an
  estimator phase, so ``rocprofv3 --marker-trace`` timelines show fit / assign / all-reduce /
  update phases next to the K* kernels; no-op when the library is absent or ``CML_ROCTX=0``.
* When timing is on (``CML_TRACE=1`` or ``Tracer.enable()``), every range also records wall time
  into the process-wide ``TRACER`` (optionally synchronising the device at both ends, so GPU work
  is charged to the range that enqueued it). ``TRACER.summary()`` / ``TRACER.report()``.
"""
from __future__ import annotations

import contextlib
import ctypes
import functools
import os
import threading
import time
from typing import Dict, Optional

_LIB = None
_LIB_TRIED = False
_LOCK = threading.Lock()


def _roctx():
    global _LIB, _LIB_TRIED
    if _LIB_TRIED:
        return _LIB
    with _LOCK:
        if _LIB_TRIED:
            return _LIB
        _LIB_TRIED = True
        if os.environ.get("CML_ROCTX", "1") == "0":
            return None
        for name in ("librocprofiler-sdk-roctx.so.1", "librocprofiler-sdk-roctx.so", "libroctx64.so.4"):
            for base in ("", "/opt/rocm/lib/"):
                try:
                    lib = ctypes.CDLL(base + name)
                except OSError:
                    continue
                lib.roctxRangePushA.argtypes = [ctypes.c_char_p]
                lib.roctxRangePushA.restype = ctypes.c_int
                lib.roctxRangePop.argtypes = []
                lib.roctxRangePop.restype = ctypes.c_int
                lib.roctxMarkA.argtypes = [ctypes.c_char_p]
                lib.roctxMarkA.restype = None
                _LIB = lib
                return _LIB
        return None


class Tracer:
    """Aggregates range durations by name (count, total seconds, max seconds)."""

    def __init__(self):
        self.enabled = os.environ.get("CML_TRACE", "0") == "1"
        self.sync = os.environ.get("CML_TRACE_SYNC", "1") == "1"
        self._stats: Dict[str, list] = {}
        self._lock = threading.Lock()

    def enable(self, sync: bool = True) -> None:
        self.enabled, self.sync = True, sync

    def disable(self) -> None:
        self.enabled = False

    def reset(self) -> None:
        with self._lock:
            self._stats.clear()

    def record(self, name: str, seconds: float) -> None:
        with self._lock:
            s = self._stats.setdefault(name, [0, 0.0, 0.0])
            s[0] += 1
            s[1] += seconds
            s[2] = max(s[2], seconds)

    def summary(self) -> Dict[str, dict]:
        with self._lock:
            return {k: {"count": v[0], "total_s": v[1], "max_s": v[2]} for k, v in self._stats.items()}

    def report(self) -> str:
        rows = sorted(self.summary().items(), key=lambda kv: -kv[1]["total_s"])
        out = [f"{'range':40s} {'count':>7s} {'total ms':>10s} {'avg ms':>9s} {'max ms':>9s}"]
        for k, v in rows:
            out.append(f"{k:40s} {v['count']:7d} {v['total_s'] * 1e3:10.2f} {v['total_s'] * 1e3 / v['count']:9.3f} "
                       f"{v['max_s'] * 1e3:9.3f}")
        return "\n".join(out)


TRACER = Tracer()


def _device_sync():
    try:
        import torch
        if torch.cuda.is_available() and torch.cuda.is_initialized():
            torch.cuda.synchronize()
    except Exception:  # pragma: no cover - tracing must never break a run
        pass


def mark(message: str) -> None:
    lib = _roctx()
    if lib is not None:
        lib.roctxMarkA(message.encode())


@contextlib.contextmanager
def trace(name: str, sync: Optional[bool] = None):
    lib = _roctx()
    timing = TRACER.enabled
    do_sync = TRACER.sync if sync is None else sync
    if lib is not None:
        lib.roctxRangePushA(name.encode())
    if timing and do_sync:
        _device_sync()
    t0 = time.perf_counter()
    try:
        yield
    finally:
        if timing:
            if do_sync:
                _device_sync()
            TRACER.record(name, time.perf_counter() - t0)
        if lib is not None:
            lib.roctxRangePop()


def traced(name: Optional[str] = None):
    def deco(fn):
        label = name or f"{fn.__module__.rsplit('.', 1)[-1]}.{fn.__qualname__}"

        @functools.wraps(fn)
        def wrapper(*a, **kw):
            with trace(label):
                return fn(*a, **kw)
        return wrapper
    return deco
