"""BisectingKMeans (Spark ``org.apache.spark.ml.clustering.BisectingKMeans``).

Divisive hierarchical clustering for segmenting hospitals / admissions when the number of
natural groups is unknown (the reference's feature table, ref.py:134-136).  The algorithm is
Spark's ``mllib.clustering.BisectingKMeans.runWithWeight`` step for step:

* nodes carry Spark's raw indices (root 1, children 2i and 2i+1); a level works on the
  ACTIVE set only — the clusters created on the previous level.  Every active cluster leaves
  the active set at the end of the level, divided or not: an undivided one is a permanent leaf.
* divisible: ``size >= minSize`` and ``cost > EPSILON * size``, where ``minSize`` is
  ``ceil(minDivisibleClusterSize)`` (or ``ceil(fraction * n)`` below 1.0) and EPSILON is the
  double machine epsilon (MLUtils.EPSILON).  When more clusters are divisible than leaves are
  still needed, the LARGEST (by size) are divided.
* each divided cluster is seeded by ``splitCenter``: centre ∓ 1e-4·‖centre‖·u with u uniform
  [0, 1)^d drawn from ``java.util.Random(seed)`` (reimplemented bit-exactly, ``JavaRandom``),
  then ALL divided clusters of the level run exactly ``maxIter`` restricted 2-means iterations
  together (each row chooses between its own cluster's two children, the left one on ties; a
  child that attracts no row drops out, as in Spark's updateAssignments).  One iteration is one
  pass over the local rows plus ONE all-reduce of every child's (Σx, count, Σ‖x‖²).
* summaries are Spark's ClusterSummary: centre Σx/n, cost max(Σ‖x‖² − n‖c‖², 0).
* the tree (buildTree): internal iff the left child exists; leaves are numbered 0.. in
  left-first depth order, internal nodes -1, -2, ...; height = max distance centre -> child.

Parity notes (pyspark is not importable here, so parity is unpinned by fixture): Spark divides
the clusters of a level in its Map's iteration order when drawing the split noise; here they are
drawn in ascending node-index order.  Prediction walks the tree from the root, taking the
closer child at every level (``ClusteringTreeNode.predict``).  Save: ml metadata under
``path/metadata`` and the mllib ``BisectingKMeansModel`` (SaveLoadV3_0: JSON metadata with
rootId, k, distanceMeasure, trainingCost + one parquet row per node) under ``path/data``.
"""
from __future__ import annotations

import json
import math
import os
from typing import Dict, List, Optional

import numpy as np
import torch

from ..ops.group_ops import group_sum_rows

from ..sql import types as T
from ..sql.column import ColumnData
from . import util as U
from .util import java_hash
from .base import Estimator, Model
from .feature import _replace_col
from .util import JavaRandom  # noqa: F401 (re-exported)
from .linalg import as_array

EPSILON = np.finfo(np.float64).eps  # MLUtils.EPSILON: 2.220446049250313e-16
LEVEL_LIMIT = 63                    # log2(Long.MaxValue): raw indices stay below 2^63
_CHUNK = 1 << 24                    # elements per f64 row chunk (bounded temporaries)


class _Node:
    def __init__(self, center: np.ndarray, size: float, cost: float, index: int = -1, height: float = 0.0):
        self.center, self.size, self.cost = np.asarray(center, dtype=np.float64), size, cost
        self.children: List["_Node"] = []
        self.index = index
        self.height = height


class _Summary:
    def __init__(self, size: int, center: np.ndarray, cost: float):
        self.size, self.center, self.cost = size, center, cost


def _summarize(x: torch.Tensor, idx: torch.Tensor, keys: List[int], comm) -> Dict[int, _Summary]:
    """Spark ``summarize`` restricted to the clusters ``keys``: per cluster (Σx, n, Σ‖x‖²),
    all-reduced in one message; clusters with no row anywhere are absent from the result."""
    d = int(x.shape[1])
    m = len(keys)
    acc = torch.zeros((m, d + 2), dtype=torch.float64, device=x.device)
    if m and x.shape[0]:
        kt = torch.as_tensor(sorted(keys), dtype=torch.int64, device=x.device)
        step = max(1, _CHUNK // max(d, 1))
        for r0 in range(0, int(x.shape[0]), step):
            ii = idx[r0:r0 + step]
            slot = torch.searchsorted(kt, ii).clamp(max=m - 1)
            sel = kt[slot] == ii
            if not bool(sel.any()):
                continue
            xs = x[r0:r0 + step][sel].to(torch.float64)
            part = torch.cat([xs, torch.ones((xs.shape[0], 1), dtype=torch.float64, device=x.device),
                              (xs * xs).sum(1, keepdim=True)], 1)
            acc += group_sum_rows(slot[sel], part, m)  # K25 per-cluster column sums on the GPU
    comm.allreduce_(acc)
    a = acc.cpu().numpy()
    out = {}
    for j, key in enumerate(sorted(keys)):
        n = a[j, d]
        if n <= 0:
            continue
        c = a[j, :d] / n
        out[key] = _Summary(int(round(n)), c, max(float(a[j, d + 1]) - n * float(c @ c), 0.0))
    return out


def _update_assignments(x: torch.Tensor, idx: torch.Tensor, divisible: List[int],
                        centers: Dict[int, np.ndarray]) -> torch.Tensor:
    """Spark ``updateAssignments``: rows of a divided cluster i move to the closer of its
    children 2i / 2i+1 that still exist (left on ties); every other row keeps its index."""
    out = idx.clone()
    if not divisible or x.shape[0] == 0:
        return out
    d = int(x.shape[1])
    dv = torch.as_tensor(sorted(divisible), dtype=torch.int64, device=x.device)
    m = dv.numel()
    inf = float("inf")
    lc = np.full((m, d), np.nan)
    rc = np.full((m, d), np.nan)
    for j, i in enumerate(sorted(divisible)):
        if 2 * i in centers:
            lc[j] = centers[2 * i]
        if 2 * i + 1 in centers:
            rc[j] = centers[2 * i + 1]
    L = torch.as_tensor(lc, device=x.device)
    R = torch.as_tensor(rc, device=x.device)
    has_l = ~torch.isnan(L[:, 0])
    has_r = ~torch.isnan(R[:, 0])
    step = max(1, _CHUNK // max(d, 1))
    for r0 in range(0, int(x.shape[0]), step):
        ii = idx[r0:r0 + step]
        slot = torch.searchsorted(dv, ii).clamp(max=m - 1)
        sel = (dv[slot] == ii) & (has_l[slot] | has_r[slot])
        if not bool(sel.any()):
            continue
        rows = torch.nonzero(sel).flatten()
        s = slot[rows]
        xs = x[r0:r0 + step][rows].to(torch.float64)
        dl = torch.where(has_l[s], ((xs - torch.nan_to_num(L[s])) ** 2).sum(1), torch.full_like(xs[:, 0], inf))
        dr = torch.where(has_r[s], ((xs - torch.nan_to_num(R[s])) ** 2).sum(1), torch.full_like(xs[:, 0], inf))
        child = 2 * ii[rows] + (dr < dl).to(torch.int64)
        out[r0 + rows] = child
    return out


def _split_center(center: np.ndarray, rnd: JavaRandom):
    level = 1e-4 * float(np.linalg.norm(center))
    noise = np.array([rnd.next_double() for _ in range(center.size)])
    return center - level * noise, center + level * noise


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
        max_iter = self.getMaxIter()
        x = df._feature_matrix(self.getFeaturesCol())
        comm = df._comm
        idx = torch.ones(x.shape[0], dtype=torch.int64, device=x.device)  # ROOT_INDEX = 1
        active = _summarize(x, idx, [1], comm)
        if not active:
            raise ValueError("BisectingKMeans needs at least one row")
        n = active[1].size
        mds = self.getMinDivisibleClusterSize()
        min_size = math.ceil(mds) if mds >= 1.0 else math.ceil(mds * n)
        inactive: Dict[int, _Summary] = {}
        rnd = JavaRandom(self.getSeed())
        needed, level = k - 1, 1
        while active and needed > 0 and level < LEVEL_LIMIT:
            div = {i: s for i, s in active.items() if s.size >= min_size and s.cost > EPSILON * s.size}
            if len(div) > needed:  # take the larger ones (stable by index on equal sizes)
                div = dict(sorted(div.items(), key=lambda kv: (-kv[1].size, kv[0]))[:needed])
            if not div:
                inactive.update(active)
                active = {}
                break
            dvi = sorted(div)
            centers: Dict[int, np.ndarray] = {}
            for i in dvi:
                centers[2 * i], centers[2 * i + 1] = _split_center(div[i].center, rnd)
            new = {}
            for _ in range(max(max_iter, 1)):
                child_idx = _update_assignments(x, idx, dvi, centers)
                new = _summarize(x, child_idx, [c for i in dvi for c in (2 * i, 2 * i + 1)], comm)
                centers = {c: s.center for c, s in new.items()}
            idx = _update_assignments(x, idx, dvi, centers)
            inactive.update(active)
            active = new
            needed -= len(div)
            level += 1
        clusters = {**inactive, **active}
        root = _build_tree(clusters)
        m = BisectingKMeansModel(root)
        self._copyValues(m)
        m._training_cost = float(sum(nd.cost for nd in m._leaves))
        m._summary = BisectingKMeansSummary(m, df, len(m._leaves), max_iter, m._training_cost)
        return m


def _build_tree(clusters: Dict[int, _Summary]) -> _Node:
    """Spark ``buildTree``: internal iff the left child exists; leaf indices 0.. in left-first
    depth order, internal indices -1, -2, ...; height = max distance to a child centre."""
    counters = {"leaf": 0, "internal": -1}

    def build(raw: int) -> _Node:
        s = clusters[raw]
        if 2 * raw in clusters:
            node = _Node(s.center, s.size, s.cost, counters["internal"])
            counters["internal"] -= 1
            kids = [c for c in (2 * raw, 2 * raw + 1) if c in clusters]
            node.height = max(float(np.linalg.norm(s.center - clusters[c].center)) for c in kids)
            node.children = [build(c) for c in kids]
            return node
        node = _Node(s.center, s.size, s.cost, counters["leaf"])
        counters["leaf"] += 1
        return node

    return build(1)


class BisectingKMeansSummary:
    def __init__(self, model, df, k, num_iter, cost):
        self._model, self._df = model, df
        self.k, self.numIter, self.trainingCost = k, num_iter, cost
        self.featuresCol = model.getFeaturesCol()
        self.predictionCol = model.getPredictionCol()

    @property
    def predictions(self):
        return self._model.transform(self._df)

    @property
    def cluster(self):
        return self.predictions.select(self.predictionCol)

    @property
    def clusterSizes(self) -> List[int]:
        lab = self._model._predict_tensor(self._df._feature_matrix(self.featuresCol))
        sizes = torch.bincount(lab, minlength=self.k).to(torch.float64)
        self._df._comm.allreduce_(sizes)
        return [int(v) for v in sizes.cpu().tolist()]


class BisectingKMeansModel(Model):
    _params = BisectingKMeans._params

    def __init__(self, root: Optional[_Node] = None):
        super().__init__()
        self._root = root
        self._training_cost = float("nan")
        self._leaves: List[_Node] = []
        self._summary = None
        if root is not None:
            self._index()

    def _index(self):
        self._leaves = []

        def walk(nd):
            if not nd.children:
                self._leaves.append(nd)
            for ch in nd.children:
                walk(ch)
        walk(self._root)
        self._leaves.sort(key=lambda nd: nd.index)

    def clusterCenters(self) -> List[np.ndarray]:
        return [nd.center.copy() for nd in self._leaves]

    @property
    def numFeatures(self) -> int:
        return int(self._root.center.size)

    @property
    def trainingCost(self) -> float:
        return self._training_cost

    @property
    def hasSummary(self) -> bool:
        return self._summary is not None

    @property
    def summary(self) -> BisectingKMeansSummary:
        if self._summary is None:
            raise RuntimeError("No training summary available for this BisectingKMeansModel")
        return self._summary

    def _predict_tensor(self, x: torch.Tensor) -> torch.Tensor:
        out = torch.empty(x.shape[0], dtype=torch.int64, device=x.device)
        step = max(1, _CHUNK // max(int(x.shape[1]), 1))

        def walk(nd, rows, xs):
            if rows.numel() == 0:
                return
            if not nd.children:
                out[rows] = nd.index
                return
            cs = torch.as_tensor(np.stack([ch.center for ch in nd.children]), device=x.device)
            go = torch.argmin(((xs[:, None, :] - cs[None]) ** 2).sum(-1), 1)
            for h, ch in enumerate(nd.children):
                sel = go == h
                walk(ch, rows[sel], xs[sel])
        for r0 in range(0, int(x.shape[0]), step):
            xs = x[r0:r0 + step].to(torch.float64)
            walk(self._root, torch.arange(r0, r0 + xs.shape[0], device=x.device), xs)
        return out

    def predict(self, value) -> int:
        return int(self._predict_tensor(torch.as_tensor(as_array(value)).reshape(1, -1))[0])

    def computeCost(self, dataset) -> float:
        x = dataset._feature_matrix(self.getFeaturesCol())
        lab = self._predict_tensor(x)
        cs = torch.as_tensor(np.stack([nd.center for nd in self._leaves]), device=x.device)
        c = torch.zeros(1, dtype=torch.float64, device=x.device)
        step = max(1, _CHUNK // max(int(x.shape[1]), 1))
        for r0 in range(0, int(x.shape[0]), step):
            xs = x[r0:r0 + step].to(torch.float64)
            c += ((xs - cs[lab[r0:r0 + step]]) ** 2).sum()
        dataset._comm.allreduce_(c)
        return float(c[0])

    def _transform(self, df):
        lab = self._predict_tensor(df._feature_matrix(self.getFeaturesCol())).to(torch.int32)
        return _replace_col(df, self.getPredictionCol(), ColumnData(lab, None, T.IntegerType()))

    def _nodes(self) -> List[_Node]:
        nodes = []

        def walk(nd):
            nodes.append(nd)
            for ch in nd.children:
                walk(ch)
        walk(self._root)
        return nodes

    def _save_impl(self, path):
        import pyarrow as pa
        U.write_metadata(self, path)
        data = os.path.join(path, "data")
        md = {"class": "org.apache.spark.mllib.clustering.BisectingKMeansModel", "version": "3.0",
              "rootId": int(self._root.index), "k": len(self._leaves),
              "distanceMeasure": self.getDistanceMeasure(), "trainingCost": self._training_cost}
        os.makedirs(os.path.join(data, "metadata"), exist_ok=True)
        with open(os.path.join(data, "metadata", "part-00000"), "w") as fh:
            fh.write(json.dumps(md, separators=(",", ":")) + "\n")
        open(os.path.join(data, "metadata", "_SUCCESS"), "w").close()
        rows = [{"index": int(nd.index), "size": int(round(nd.size)), "center": U.vector_struct(nd.center),
                 "norm": float(np.linalg.norm(nd.center)), "cost": float(nd.cost), "height": float(nd.height),
                 "children": [int(ch.index) for ch in nd.children]} for nd in self._nodes()]
        U.write_parquet(data, "data", pa.Table.from_pylist(rows, schema=pa.schema([
            pa.field("index", pa.int32(), nullable=False), pa.field("size", pa.int64(), nullable=False),
            ("center", U.vector_arrow_type()), pa.field("norm", pa.float64(), nullable=False),
            pa.field("cost", pa.float64(), nullable=False), pa.field("height", pa.float64(), nullable=False),
            ("children", pa.list_(pa.field("element", pa.int32(), nullable=False)))])))

    @classmethod
    def _load_impl(cls, path, md):
        data = os.path.join(path, "data")
        with open(os.path.join(data, "metadata", "part-00000")) as fh:
            dmd = json.loads(fh.readline())
        rows = {r["index"]: r for r in U.read_parquet(data, "data").to_pylist()}
        nodes = {i: _Node(U.vector_from_struct(r["center"]), float(r["size"]), r["cost"], int(i), r["height"])
                 for i, r in rows.items()}
        for i, r in rows.items():
            nodes[i].children = [nodes[ch] for ch in r["children"]]
        m = cls(nodes[int(dmd["rootId"])])
        m._training_cost = float(dmd.get("trainingCost", float("nan")))
        U.apply_params(m, md)
        return m
