"""Iteration checkpoints for long fits ("per-iteration optional estimator
checkpoint so a killed fit can resume"; the reference has no training checkpoint at all).

A checkpoint is a directory ``<dir>/<name>/`` holding ``state.json`` (iteration, a key that
identifies the fit: data size, k, seed, params) and one ``<array>.npy`` per state array (loaded
with ``allow_pickle=False``). Rank 0 writes into a temp directory and renames it over the old
one, so a crash while checkpointing leaves the previous checkpoint intact. Enabled through the
session conf ``cml.ml.checkpointDir`` (+ ``cml.ml.checkpointInterval``, default 10 iterations).
"""
from __future__ import annotations

import json
import os
import shutil
from typing import Dict, Optional, Tuple

import numpy as np


def save(directory: str, name: str, key: str, iteration: int, arrays: Dict[str, np.ndarray], comm=None) -> None:
    if comm is not None and not comm.is_root:
        return
    final = os.path.join(directory, name)
    tmp = final + f".tmp-{os.getpid()}"
    if os.path.exists(tmp):
        shutil.rmtree(tmp)
    os.makedirs(tmp)
    for k, v in arrays.items():
        np.save(os.path.join(tmp, f"{k}.npy"), np.asarray(v), allow_pickle=False)
    with open(os.path.join(tmp, "state.json"), "w") as fh:
        json.dump({"key": key, "iteration": int(iteration), "arrays": sorted(arrays)}, fh)
    old = final + f".old-{os.getpid()}"
    if os.path.exists(final):
        os.replace(final, old)
    os.replace(tmp, final)
    shutil.rmtree(old, ignore_errors=True)


def load(directory: str, name: str, key: str) -> Optional[Tuple[int, Dict[str, np.ndarray]]]:
    final = os.path.join(directory, name)
    meta = os.path.join(final, "state.json")
    if not os.path.exists(meta):
        return None
    with open(meta) as fh:
        st = json.load(fh)
    if st.get("key") != key:
        return None
    arrays = {k: np.load(os.path.join(final, f"{k}.npy"), allow_pickle=False) for k in st["arrays"]}
    return int(st["iteration"]), arrays


def clear(directory: str, name: str, comm=None) -> None:
    if comm is not None and not comm.is_root:
        return
    shutil.rmtree(os.path.join(directory, name), ignore_errors=True)
