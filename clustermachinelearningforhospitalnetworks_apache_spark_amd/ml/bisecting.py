"""BisectingKMeans (Spark ``org.apache.spark.ml.clustering.BisectingKMeans``).

Divisive hierarchical clustering for segmenting hospitals / admissions when the
number of natural groups is unknown (the reference's feature table, ref.py:134-136).
Level by level, the leaves with the largest within-cluster cost are split in two
(as many as are needed to reach ``k``, each at least ``minDivisibleClusterSize``)
by a 2-means fit of that leaf's rows.  Each 2-means is the framework's distributed
Lloyd engine (K9 MFMA assign + K10 sums + one all-reduce per iteration) over the
leaf's rows gathered on the device, so every rank works on its own shard.
Prediction walks the tree from the root, taking the closer child at every level
(Spark's ``BisectingKMeansModel.predict``).
"""
from __future__ import annotations

from typing import List, Optional

import numpy as np
import torch

from ..sql import types as T
from ..sql.column import ColumnData
from . import util as U
from .base import Estimator, Model
from .clustering import KMeans, java_hash
from .feature import _replace_col
from .linalg import as_array


class _Node:
    def __init__(self, center: np.ndarray, size: float, cost: float):
        self.center, self.size, self.cost = center, size, cost
        self.children: List["_Node"] = []
        self.index = -1


def _leaf_stats(x: torch.Tensor, mask: torch.Tensor, comm):
    xs = x[mask].to(torch.float64)
    d = x.shape[1]
    msg = torch.zeros(d + 1, dtype=torch.float64, device=x.device)
    msg[:d] = xs.sum(0)
    msg[d] = float(xs.shape[0])
    comm.allreduce_(msg)
    n = float(msg[d])
    c = msg[:d] / max(n, 1.0)
    cost = ((xs - c) ** 2).sum().reshape(1)
    comm.allreduce_(cost)
    return c.cpu().numpy(), n, float(cost[0])


class BisectingKMeans(Estimator):
    _params = {
        "featuresCol": ("features", "features column name", str),
        "predictionCol": ("prediction", "prediction column name", str),
        "k": (4, "the desired number of leaf clusters (> 1)", int),
        "maxIter": (20, "max number of iterations of every 2-means split (>= 0)", int),
        "seed": (java_hash("org.apache.spark.ml.clustering.BisectingKMeans"), "random seed", int),
        "minDivisibleClusterSize": (1.0, "minimum points (>= 1.0) or fraction (< 1.0) of a divisible cluster", float),
        "distanceMeasure": ("euclidean", "distance measure (euclidean)", str),
    }

    def _fit(self, df):
        if self.getDistanceMeasure() != "euclidean":
            raise NotImplementedError("BisectingKMeans supports distanceMeasure='euclidean'")
        k = self.getK()
        if k < 2:
            raise ValueError("k must be > 1")
        x = df._feature_matrix(self.getFeaturesCol())
        comm = df._comm
        leaf_of = torch.zeros(x.shape[0], dtype=torch.int64, device=x.device)
        c, n, cost = _leaf_stats(x, leaf_of == 0, comm)
        root = _Node(c, n, cost)
        leaves = {0: root}
        divisible = {0: True}
        next_id, level = 1, 0
        mds = self.getMinDivisibleClusterSize()
        min_size = mds if mds >= 1.0 else mds * n
        while len(leaves) < k:
            cand = [i for i, nd in leaves.items() if divisible[i] and nd.size >= max(min_size, 2.0) and nd.cost > 0]
            if not cand:
                break
            cand.sort(key=lambda i: -leaves[i].cost)
            for j, lid in enumerate(cand[: k - len(leaves)]):
                mask = leaf_of == lid
                rows = torch.nonzero(mask).flatten()
                km = KMeans(k=2, maxIter=self.getMaxIter(), seed=self.getSeed() + 1000 * level + j,
                            featuresCol=self.getFeaturesCol()).fit(df._take_rows(rows))
                cs = np.stack(km.clusterCenters())
                if cs.shape[0] < 2:
                    divisible[lid] = False
                    continue
                lab = torch.argmin(torch.cdist(x[rows].to(torch.float64), torch.as_tensor(cs, device=x.device)), 1)
                stats = []
                for h in range(2):
                    sel = torch.zeros(x.shape[0], dtype=torch.bool, device=x.device)
                    sel[rows[lab == h]] = True
                    stats.append((sel,) + _leaf_stats(x, sel, comm))
                if min(s[2] for s in stats) == 0:
                    divisible[lid] = False
                    continue
                parent = leaves.pop(lid)
                del divisible[lid]
                for sel, cc, nn, co in stats:
                    child = _Node(cc, nn, co)
                    parent.children.append(child)
                    leaves[next_id] = child
                    divisible[next_id] = True
                    leaf_of[sel] = next_id
                    next_id += 1
            level += 1
        m = BisectingKMeansModel(root)
        self._copyValues(m)
        m._training_cost = float(sum(nd.cost for nd in leaves.values()))
        return m


class BisectingKMeansModel(Model):
    _params = BisectingKMeans._params

    def __init__(self, root: Optional[_Node] = None):
        super().__init__()
        self._root = root
        self._training_cost = float("nan")
        self._leaves: List[_Node] = []
        if root is not None:
            self._index()

    def _index(self):
        self._leaves = []

        def walk(nd):
            if not nd.children:
                nd.index = len(self._leaves)
                self._leaves.append(nd)
            for ch in nd.children:
                walk(ch)
        walk(self._root)

    def clusterCenters(self) -> List[np.ndarray]:
        return [nd.center.copy() for nd in self._leaves]

    @property
    def numFeatures(self) -> int:
        return int(self._root.center.size)

    @property
    def trainingCost(self) -> float:
        return self._training_cost

    def _predict_tensor(self, x: torch.Tensor) -> torch.Tensor:
        x = x.to(torch.float64)
        out = torch.empty(x.shape[0], dtype=torch.int64, device=x.device)

        def walk(nd, rows):
            if rows.numel() == 0:
                return
            if not nd.children:
                out[rows] = nd.index
                return
            cs = torch.as_tensor(np.stack([ch.center for ch in nd.children]), device=x.device)
            go = torch.argmin(torch.cdist(x[rows], cs), 1)
            for h, ch in enumerate(nd.children):
                walk(ch, rows[go == h])
        walk(self._root, torch.arange(x.shape[0], device=x.device))
        return out

    def predict(self, value) -> int:
        return int(self._predict_tensor(torch.as_tensor(as_array(value)).reshape(1, -1))[0])

    def computeCost(self, dataset) -> float:
        x = dataset._feature_matrix(self.getFeaturesCol()).to(torch.float64)
        lab = self._predict_tensor(x)
        cs = torch.as_tensor(np.stack([nd.center for nd in self._leaves]), device=x.device)
        c = ((x - cs[lab]) ** 2).sum().reshape(1)
        dataset._comm.allreduce_(c)
        return float(c[0])

    def _transform(self, df):
        lab = self._predict_tensor(df._feature_matrix(self.getFeaturesCol())).to(torch.int32)
        return _replace_col(df, self.getPredictionCol(), ColumnData(lab, None, T.IntegerType()))

    def _save_impl(self, path):
        import pyarrow as pa
        U.write_metadata(self, path, extra={"rootId": 0, "trainingCost": self._training_cost})
        nodes = []

        def walk(nd):
            nodes.append(nd)
            for ch in nd.children:
                walk(ch)
        walk(self._root)
        ids = {id(nd): i for i, nd in enumerate(nodes)}
        rows = [{"index": ids[id(nd)], "size": int(round(nd.size)), "center": U.vector_struct(nd.center),
                 "norm": float(np.linalg.norm(nd.center)), "cost": float(nd.cost), "height": 0.0,
                 "children": [ids[id(ch)] for ch in nd.children]} for nd in nodes]
        U.write_parquet(path, "data", pa.Table.from_pylist(rows, schema=pa.schema([
            pa.field("index", pa.int32(), nullable=False), pa.field("size", pa.int64(), nullable=False),
            ("center", U.vector_arrow_type()), pa.field("norm", pa.float64(), nullable=False),
            pa.field("cost", pa.float64(), nullable=False), pa.field("height", pa.float64(), nullable=False),
            ("children", pa.list_(pa.int32()))])))

    @classmethod
    def _load_impl(cls, path, md):
        rows = {r["index"]: r for r in U.read_parquet(path, "data").to_pylist()}
        nodes = {i: _Node(U.vector_from_struct(r["center"]), float(r["size"]), r["cost"]) for i, r in rows.items()}
        for i, r in rows.items():
            nodes[i].children = [nodes[ch] for ch in r["children"]]
        m = cls(nodes[int(md.get("rootId", 0))])
        m._training_cost = float(md.get("trainingCost", float("nan")))
        U.apply_params(m, md)
        return m
