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


class _TorchOpCounter:
    """Counts the torch operations (other than views) run while a launch sequence is recorded: their effects
    (a fill, a temporary's allocation, a host read) happen at record time only and are not replayed, so a
    recording that saw one must not be cached."""

    def __init__(self):
        self.ops = []
        self._mode = None

    def __enter__(self):
        from torch.utils._python_dispatch import TorchDispatchMode
        counter = self

        class _Mode(TorchDispatchMode):
            def __torch_dispatch__(self, func, types, args=(), kwargs=None):
                if not getattr(func, "is_view", False) and func not in _VIEW_LIKE:
                    counter.ops.append(str(func))
                return func(*args, **(kwargs or {}))

        self._mode = _Mode()
        self._mode.__enter__()
        return self

    def __exit__(self, *exc):
        self._mode.__exit__(*exc)
        return False


_VIEW_LIKE = set()
for _name in ("detach.default", "alias.default", "slice.Tensor", "select.int", "view.default", "as_strided.default"):
    _pkt, _ov = _name.split(".")
    _VIEW_LIKE.add(getattr(getattr(torch.ops.aten, _pkt), _ov))


@contextlib.contextmanager
def recording():
    """``with recording() as rec: <wrapper calls>``; then ``Recorded(rec.calls)`` replays them. Only for
    wrappers whose sole effect is their kernel launches (their return values are not produced). ``rec.torch_ops``
    lists the torch operations that ran meanwhile (a recording with any is not replayable)."""
    rec = _Recorder(_real_kernels())
    prev = getattr(_recording, "rec", None)
    _recording.rec = rec
    cnt = _TorchOpCounter()
    try:
        with cnt:
            yield rec
    finally:
        _recording.rec = prev
        rec.torch_ops = cnt.ops


class ReplayGuard:
    """When a recorded sequence may be replayed: it froze raw pointers (and the stream) at record time, so it is
    valid only while every tensor behind its pointer arguments is still the one it was recorded with. The guard
    finds, for each pointer argument, a tensor attribute of ``roots`` whose storage holds it (engine buffers,
    step state) and keeps (holder, attribute, index, data_ptr); ``valid()`` re-reads those attributes (a few
    microseconds) — a re-allocated buffer fails it and the caller records again. ``ok`` is False when the
    recording cannot be replayed at all: a pointer that belongs to no root tensor (a temporary the wrappers
    allocated, which would dangle), a torch operation during the recording, or a stream other than ``stream``."""

    __slots__ = ("ok", "why", "watch")

    def __init__(self, rec, roots, stream: int):
        self.ok, self.why, self.watch = True, "", ()
        if getattr(rec, "torch_ops", None):
            self.ok, self.why = False, f"torch ops while recording: {rec.torch_ops[:4]}"
            return
        ptrs = set()
        for _fn, conv, name in rec.calls:
            for a in conv:
                if isinstance(a, ctypes.c_void_p) and a.value:
                    ptrs.add(a.value)
        ptrs.discard(stream)
        spans = []
        for obj in roots:
            if obj is None:
                continue
            for attr, v in vars(obj).items():
                items = [(None, v)] if torch.is_tensor(v) else (
                    list(enumerate(v)) if isinstance(v, (list, tuple)) else [])
                for idx, t in items:
                    if torch.is_tensor(t) and t.numel():
                        stg = t.untyped_storage()
                        spans.append((stg.data_ptr(), stg.data_ptr() + stg.nbytes(), obj, attr, idx, t.data_ptr()))
        watch = {}
        for p in ptrs:
            hit = next((sp for sp in spans if sp[0] <= p < sp[1]), None)
            if hit is None:
                self.ok, self.why = False, f"pointer {p:#x} is no root tensor's (a temporary)"
                return
            watch[(id(hit[2]), hit[3], hit[4])] = hit[2:]
        self.watch = tuple(watch.values())

    def valid(self) -> bool:
        for obj, attr, idx, ptr in self.watch:
            v = getattr(obj, attr, None)
            if idx is not None:
                v = v[idx] if isinstance(v, (list, tuple)) and len(v) > idx else None
            if not torch.is_tensor(v) or v.data_ptr() != ptr:
                return False
        return True


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
