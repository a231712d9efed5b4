"""Power iteration clustering (pyspark.ml.clustering.PowerIterationClustering, Lin & Cohen 2010):
clusters the vertices of an affinity graph given as (src, dst, weight) rows — e.g. hospitals linked
by patient-transfer volume.

Spark semantics kept: self-loops are dropped, every edge is used in both directions (duplicates
add up), W is row-normalised by the degree D, the start vector is random (L1-normalised) or the
normalised degree, the iteration v ← W v / ‖W v‖₁ stops after ``maxIter`` steps or when the change
of ‖v_t − v_{t−1}‖₁ between two steps drops below max(1e-5 / n, 1e-8), and the final 1-D
embedding is clustered with k-means.

Device design: each rank keeps its shard of the edges on the device as COO index/value tensors;
one sparse mat-vec is an ``index_add_`` over the shard, and the [n] partial products of all ranks are
summed with one all-reduce per iteration (n doubles — latency-bound, so there is exactly one
collective per step). The vertex index is the sorted union of all ranks' ids, identical on every
rank, and the random start vector is a counter-based normal of the vertex id, so the result does
not depend on the number of ranks.
"""
from __future__ import annotations

import math
from typing import List

import numpy as np
import torch

from ..sql import types as T
from ..utils import rng as R
from .param import Params
from .util import MLReadable, MLWritable


def _kmeans_1d(v: np.ndarray, k: int, seed: int = 0, iters: int = 100) -> np.ndarray:
    """k-means++ seeding (seeded) then Lloyd iterations on a 1-D embedding; labels per point."""
    n = v.shape[0]
    rs = np.random.default_rng(seed)
    centers = [v[rs.integers(n)]]
    for _ in range(1, k):
        d2 = np.min((v[:, None] - np.asarray(centers)[None, :]) ** 2, axis=1)
        tot = d2.sum()
        centers.append(v[rs.integers(n)] if tot == 0 else v[np.searchsorted(np.cumsum(d2), rs.random() * tot)
                                                               .clip(0, n - 1)])
    c = np.asarray(centers, dtype=np.float64)
    lab = np.zeros(n, dtype=np.int64)
    for _ in range(iters):
        lab = np.argmin(np.abs(v[:, None] - c[None, :]), axis=1)
        nc = c.copy()
        for j in range(k):
            m = lab == j
            if m.any():
                nc[j] = v[m].mean()
        if np.allclose(nc, c, rtol=0, atol=0):
            break
        c = nc
    return lab


class PowerIterationClustering(Params, MLWritable, MLReadable):
    """``PowerIterationClustering(k=2, maxIter=20, initMode="random", srcCol="src", dstCol="dst",
    weightCol=None).assignClusters(df)`` → DataFrame(id: bigint, cluster: int)."""
    _params = {
        "k": (2, "The number of clusters to create. Must be > 1.", int),
        "maxIter": (20, "max number of iterations (>= 0)", int),
        "initMode": ("random", "The initialization algorithm. This can be either 'random' to use a random "
                               "vector as vertex properties, or 'degree' to use a normalized sum of similarities "
                               "with other vertices.", str),
        "srcCol": ("src", "Name of the input column for source vertex IDs.", str),
        "dstCol": ("dst", "Name of the input column for destination vertex IDs.", str),
        "weightCol": (None, "weight column name. If this is not set or empty, we treat all instance weights "
                            "as 1.0.", str),
    }

    def __init__(self, k=None, maxIter=None, initMode=None, srcCol=None, dstCol=None, weightCol=None):
        super().__init__(k=k, maxIter=maxIter, initMode=initMode, srcCol=srcCol, dstCol=dstCol,
                         weightCol=weightCol)
        self._defaultParamMap.pop("weightCol", None)

    def setParams(self, **kwargs):
        self._set(**{k: v for k, v in kwargs.items() if v is not None})
        return self

    def assignClusters(self, dataset):
        k = self.getK()
        if k < 2:
            raise ValueError("PowerIterationClustering: k must be > 1")
        mode = self.getInitMode()
        if mode not in ("random", "degree"):
            raise ValueError(f"initMode must be 'random' or 'degree', got {mode!r}")
        comm = dataset._comm
        dev = dataset._device
        src = dataset._column_data(self.getSrcCol()).values.to(torch.int64).to(dev)
        dst = dataset._column_data(self.getDstCol()).values.to(torch.int64).to(dev)
        wc = self.getOrDefault("weightCol") if self.isSet("weightCol") else None
        w = dataset._column_data(wc).values.to(torch.float64).to(dev) if wc else \
            torch.ones(src.shape[0], dtype=torch.float64, device=dev)
        if bool((w < 0).any()):
            raise ValueError("PowerIterationClustering: similarities must be nonnegative")
        keep = src != dst
        src, dst, w = src[keep], dst[keep], w[keep]
        # global vertex index (sorted union of every rank's ids)
        local_ids = torch.unique(torch.cat([src, dst])).cpu().numpy()
        ids = np.unique(np.concatenate([np.asarray(p, dtype=np.int64) for p in comm.allgather_object(local_ids)]))
        n = ids.shape[0]
        if n == 0:
            return self._frame(dataset, ids, np.zeros(0, dtype=np.int64))
        idt = torch.as_tensor(ids, device=dev)
        rows = torch.searchsorted(idt, torch.cat([src, dst]))
        cols = torch.searchsorted(idt, torch.cat([dst, src]))
        vals = torch.cat([w, w])
        deg = torch.zeros(n, dtype=torch.float64, device=dev).index_add_(0, rows, vals)
        comm.allreduce_(deg)
        wn = vals / torch.clamp(deg[rows], min=2.220446049250313e-16)
        if mode == "degree":
            v = deg / deg.sum()
        else:
            u1 = R.uniform(idt, 0, 1).clamp(min=1e-300)
            u2 = R.uniform(idt, 0, 2)
            g = torch.sqrt(-2.0 * torch.log(u1)) * torch.cos(2.0 * math.pi * u2)
            v = g / g.abs().sum()
        tol = max(1e-5 / n, 1e-8)
        prev_delta, diff = float("inf"), float("inf")
        for _ in range(self.getMaxIter()):
            if abs(diff) <= tol:
                break
            nv = torch.zeros(n, dtype=torch.float64, device=dev).index_add_(0, rows, wn * v[cols])
            comm.allreduce_(nv)
            nv = nv / nv.abs().sum()
            delta = float((nv - v).abs().sum())
            diff = abs(delta - prev_delta)
            prev_delta = delta
            v = nv
        labels = _kmeans_1d(v.cpu().numpy(), k)
        return self._frame(dataset, ids, labels)

    @staticmethod
    def _frame(dataset, ids: np.ndarray, labels: np.ndarray):
        from ..sql.builder import rows_round_robin
        schema = T.StructType([T.StructField("id", T.LongType(), False), T.StructField("cluster", T.IntegerType(), False)])
        return rows_round_robin(dataset._session, schema, [[int(i), int(c)] for i, c in zip(ids, labels)])


__all__: List[str] = ["PowerIterationClustering"]
