"""Iteration checkpoints for long fits ("per-iteration optional estimator
checkpoint so a killed fit can resume"; the reference has no training checkpoint at all).

Layout of a checkpoint ``<dir>/<name>/``::

    v-00000012/state.json      iteration, the key that identifies the fit (data size, k, seed, params)
    v-00000012/<array>.npy     one file per state array (loaded with ``allow_pickle=False``)
    LATEST                     name of the newest complete version ("v-00000012")

Crash safety: rank 0 writes a new version into ``v-<it>.tmp-<pid>``, fsyncs its files and the
directory, renames it to a name no earlier save used (``v-<it>``, or ``v-<it>-<generation>`` when
that iteration was saved before — a resumed fit — so a rename never replaces or deletes anything),
fsyncs the parent, then atomically replaces the ``LATEST`` pointer file (written, fsynced, renamed,
parent fsynced), and only then deletes versions older than the previous one. At every instant —
power loss included — at least one complete, durable version exists and ``load`` finds it: through
``LATEST``, or — if the pointer is missing, torn or names a version that is gone — by scanning for the
newest ``v-*`` directory that has its ``state.json`` (written last inside the version, so its
presence means the version is complete).

Names are derived from the fit's key (``name_for``), not from an estimator uid, so a restarted
process (a new uid) finds the checkpoint of the same fit.  ``load_shared`` makes the resume
decision on rank 0 and broadcasts it with the arrays, so every rank resumes from the same
iteration or none does (a per-rank decision would desynchronise the collective sequence).
Enabled through the session conf ``cml.ml.checkpointDir`` (+ ``cml.ml.checkpointInterval``).
"""
from __future__ import annotations

import hashlib
import json
import os
import re
import shutil
from typing import Dict, Optional, Tuple

import numpy as np

_VER = re.compile(r"^v-(\d{8,})(?:-(\d+))?$")


def name_for(prefix: str, key: str) -> str:
    """Stable checkpoint name of a fit: the same key in any process or rank gives the same name."""
    return f"{prefix}-{hashlib.sha1(key.encode()).hexdigest()[:16]}"


def _versions(root: str):
    """Complete versions under ``root``, newest first."""
    out = []
    try:
        entries = os.listdir(root)
    except FileNotFoundError:
        return out
    for e in entries:
        m = _VER.match(e)
        if m and os.path.exists(os.path.join(root, e, "state.json")):
            out.append(((int(m.group(1)), int(m.group(2) or 0)), e))
    return [e for _, e in sorted(out, reverse=True)]


def _fsync_dir(path: str) -> None:
    try:
        fd = os.open(path, os.O_RDONLY)
    except OSError:
        return
    try:
        os.fsync(fd)
    except OSError:
        pass
    finally:
        os.close(fd)


def _write_durable(path: str, write) -> None:
    with open(path, "wb") as fh:
        write(fh)
        fh.flush()
        os.fsync(fh.fileno())


def save(directory: str, name: str, key: str, iteration: int, arrays: Dict[str, np.ndarray], comm=None) -> None:
    if comm is not None and not comm.is_root:
        return
    root = os.path.join(directory, name)
    os.makedirs(root, exist_ok=True)
    base = f"v-{int(iteration):08d}"
    gens = [int(m.group(2) or 0) for m in (_VER.match(e) for e in os.listdir(root)) if m and
            int(m.group(1)) == int(iteration)]
    ver = base if not gens else f"{base}-{max(gens) + 1}"  # never an existing name
    final = os.path.join(root, ver)
    tmp = os.path.join(root, f"{ver}.tmp-{os.getpid()}")
    shutil.rmtree(tmp, ignore_errors=True)
    os.makedirs(tmp)
    for k, v in arrays.items():
        _write_durable(os.path.join(tmp, f"{k}.npy"), lambda fh, v=v: np.save(fh, np.asarray(v), allow_pickle=False))
    meta = json.dumps({"key": key, "iteration": int(iteration), "arrays": sorted(arrays)}).encode()
    _write_durable(os.path.join(tmp, "state.json"), lambda fh: fh.write(meta))  # last: marks the version complete
    _fsync_dir(tmp)
    os.rename(tmp, final)
    _fsync_dir(root)
    ptr_tmp = os.path.join(root, f"LATEST.tmp-{os.getpid()}")
    _write_durable(ptr_tmp, lambda fh: fh.write((ver + "\n").encode()))
    os.replace(ptr_tmp, os.path.join(root, "LATEST"))
    _fsync_dir(root)
    keep = set(_versions(root)[:2]) | {ver, "LATEST"}  # the new version and the one before it
    for e in os.listdir(root):  # older versions and leftovers of crashed writers
        if e not in keep:
            p = os.path.join(root, e)
            if os.path.isdir(p):
                shutil.rmtree(p, ignore_errors=True)
            else:
                try:
                    os.remove(p)
                except FileNotFoundError:
                    pass


def load(directory: str, name: str, key: str) -> Optional[Tuple[int, Dict[str, np.ndarray]]]:
    root = os.path.join(directory, name)
    cands = []
    try:
        with open(os.path.join(root, "LATEST")) as fh:
            cands.append(fh.read().strip())
    except (FileNotFoundError, OSError):
        pass
    cands += [v for v in _versions(root) if v not in cands]
    for ver in cands:
        meta = os.path.join(root, ver, "state.json")
        try:
            with open(meta) as fh:
                st = json.load(fh)
        except (FileNotFoundError, ValueError, OSError):
            continue  # missing or torn: try the next complete version
        if st.get("key") != key:
            return None
        try:
            arrays = {k: np.load(os.path.join(root, ver, f"{k}.npy"), allow_pickle=False) for k in st["arrays"]}
        except (FileNotFoundError, ValueError, OSError):
            continue
        return int(st["iteration"]), arrays
    return None


def load_shared(directory: str, name: str, key: str, comm=None) -> Optional[Tuple[int, Dict[str, np.ndarray]]]:
    """``load`` on rank 0, broadcast to every rank (decision and arrays)."""
    if comm is None or not comm.is_distributed:
        return load(directory, name, key)
    res = load(directory, name, key) if comm.is_root else None
    return comm.broadcast_object(res, src=0)


def clear(directory: str, name: str, comm=None) -> None:
    if comm is not None and not comm.is_root:
        return
    shutil.rmtree(os.path.join(directory, name), ignore_errors=True)


def data_fingerprint(x, comm) -> str:
    """Global (Σx, Σx²) of a device/host tensor in float64 (a collective): two fits with the same shape and
    params but different data never share a checkpoint."""
    import torch
    x2 = x.reshape(x.shape[0], -1) if x.dim() != 2 else x
    s = torch.zeros(2, dtype=torch.float64, device=x.device)
    step = max(1, (1 << 24) // max(int(x2.shape[1]), 1))  # row chunks of 16M elements: bounded f64 temporaries
    for r0 in range(0, int(x2.shape[0]), step):
        xf = x2[r0:r0 + step].to(torch.float64)
        s[0] += xf.sum()
        s[1] += (xf * xf).sum()
    comm.allreduce_(s)
    return f"{float(s[0]):.17g},{float(s[1]):.17g}"


class FitCheckpoint:
    """Iteration checkpoints of one estimator fit, enabled by the session conf
    ``cml.ml.checkpointDir`` (every ``cml.ml.checkpointInterval`` iterations, default 10). The key is the
    estimator kind, its objective-defining params, the global row count and a fingerprint of every input
    tensor, so a restarted process (new estimator uid) finds the checkpoint of the same fit and a different
    fit never does. Every rank constructs it (the fingerprint is a collective); rank 0 writes, and
    ``load`` broadcasts rank 0's decision (every rank resumes from the same point or none does)."""

    def __init__(self, df, prefix: str, key: str, tensors=()):
        conf = df._session.conf
        self.dir = conf.get("cml.ml.checkpointDir", None)
        self.every = max(1, int(conf.get("cml.ml.checkpointInterval", 10)))
        self.comm = df._comm
        self.enabled = bool(self.dir)
        self.key = self.name = None
        if self.enabled:
            n = int(self.comm.sum_scalar(float(df._nrows)))
            fp = "|".join(data_fingerprint(t, self.comm) for t in tensors if t is not None)
            self.key = f"{prefix}|n={n}|{key}|data={fp}"
            self.name = name_for(prefix, self.key)

    def load(self) -> Optional[Tuple[int, Dict[str, np.ndarray]]]:
        if not self.enabled:
            return None
        return load_shared(self.dir, self.name, self.key, self.comm)

    def due(self, iteration: int) -> bool:
        return self.enabled and iteration % self.every == 0

    def save(self, iteration: int, arrays: Dict[str, np.ndarray]) -> None:
        if self.enabled:
            save(self.dir, self.name, self.key, iteration, arrays, self.comm)

    def clear(self) -> None:
        if self.enabled:
            self.comm.barrier()
            clear(self.dir, self.name, self.comm)
