"""Loader for the in-tree native libraries (ctypes, no Python-C++ ABI coupling).

``kernels()`` returns the gfx950 HIP kernel library.  It MUST be loaded after
``import torch``: torch ships ``libamdhip64.so`` with SONAME ``libamdhip64.so.7``
and our library NEEDs that SONAME, so the dynamic loader binds our kernels to
the very HIP runtime (and device context / allocator) torch already uses.

When a GPU is present and the library cannot be built or loaded, every GPU op
raises — there is no silent eager fallback on a GPU box.
"""
from __future__ import annotations

import contextlib
import ctypes
import os
import threading
from pathlib import Path

import torch  # noqa: F401  (must precede the CDLL load, see module docstring)

HERE = Path(__file__).resolve().parent
_lock = threading.Lock()
_kernels = None
_host = None

c_int = ctypes.c_int
c_ll = ctypes.c_longlong
c_vp = ctypes.c_void_p
c_dbl = ctypes.c_double
c_float = ctypes.c_float


class NativeError(RuntimeError):
    pass


# name -> (restype, [argtypes]); each ops module registers the symbols it binds.
_KERNEL_SIGS = {}

_HOST_SIGS = {}


def register_kernel_sigs(sigs: dict) -> None:
    _KERNEL_SIGS.update(sigs)
    if _kernels is not None:
        _declare(_kernels, sigs)


def register_host_sigs(sigs: dict) -> None:
    _HOST_SIGS.update(sigs)
    if _host is not None:
        _declare(_host, sigs)


def _declare(lib, sigs):
    for name, (res, args) in sigs.items():
        fn = getattr(lib, name, None)
        if fn is None:
            raise NativeError(f"symbol {name} missing from {lib._name}; rebuild with _native.build --force")
        fn.restype = res
        fn.argtypes = args


class _Recorder:
    """Stands in for the kernel library while a launch sequence is recorded (see ``recording``): every
    ``cml_*`` call is converted to ctypes once and kept instead of run, and returns status 0."""

    def __init__(self, lib):
        self._lib = lib
        self.calls = []

    def __getattr__(self, name):
        fn = getattr(self._lib, name)
        types = fn.argtypes or []

        def rec(*args):
            conv = tuple(a if isinstance(a, t) else t(a) for a, t in zip(args, types))
            self.calls.append((fn, conv, name))
            return 0
        return rec


class Recorded:
    """A recorded launch sequence: replaying it calls the same C entry points with the same (pre-converted)
    arguments — no Python wrapper, no tensor attribute reads, no argument conversion. For hot loops whose
    buffers are fixed (the device pruned Lloyd step: ~10 launches at ~20-30 us of host time each eagerly)."""

    __slots__ = ("calls",)

    def __init__(self, calls):
        self.calls = tuple(calls)

    def __call__(self) -> None:
        for fn, conv, name in self.calls:
            st = fn(*conv)
            if st != 0:
                raise NativeError(f"{name} failed with hipError {st}")


_recording = threading.local()


@contextlib.contextmanager
def recording():
    """``with recording() as rec: <wrapper calls>``; then ``Recorded(rec.calls)`` replays them. Only for
    wrappers whose sole effect is their kernel launches (their return values are not produced)."""
    rec = _Recorder(_real_kernels())
    prev = getattr(_recording, "rec", None)
    _recording.rec = rec
    try:
        yield rec
    finally:
        _recording.rec = prev


def kernels():
    """The gfx950 kernel library (built in-tree on first use if missing)."""
    rec = getattr(_recording, "rec", None)
    if rec is not None:
        return rec
    return _real_kernels()


def _real_kernels():
    global _kernels
    if _kernels is not None:
        return _kernels
    with _lock:
        if _kernels is None:
            from . import build as _build
            path = HERE / "libcml_kernels.so"
            if os.environ.get("CML_NO_AUTOBUILD") != "1":
                _build.build_kernels()
            if not path.exists():
                raise NativeError(f"{path} missing and could not be built")
            lib = ctypes.CDLL(str(path), mode=ctypes.RTLD_GLOBAL)
            _declare(lib, _KERNEL_SIGS)
            _kernels = lib
    return _kernels


def host():
    """Host-side C++ runtime library (CSV parser, RNG helpers)."""
    global _host
    if _host is not None:
        return _host
    with _lock:
        if _host is None:
            from . import build as _build
            path = HERE / "libcml_host.so"
            if os.environ.get("CML_NO_AUTOBUILD") != "1":
                _build.build_host()
            if not path.exists():
                raise NativeError(f"{path} missing and could not be built")
            lib = ctypes.CDLL(str(path))
            _declare(lib, _HOST_SIGS)
            _host = lib
    return _host


def check(status: int, what: str) -> None:
    if status != 0:
        raise NativeError(f"{what} failed with hipError {status}")


def stream_ptr(stream=None) -> int:
    s = stream if stream is not None else torch.cuda.current_stream()
    return s.cuda_stream


def ptr(t) -> int:
    return t.data_ptr() if t is not None else 0
