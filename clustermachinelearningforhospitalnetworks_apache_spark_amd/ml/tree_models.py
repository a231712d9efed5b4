"""Shared machinery of the four tree estimators: params, fit via the forest engine,
transform via K21, featureImportances, and Spark's NodeData Parquet layout
(``data/`` rows of NodeData for a single tree; ``(treeID, nodeData)`` rows plus
``treesMetadata/`` for ensembles — SURVEY.md §5.4).
"""
from __future__ import annotations

import json
from typing import List, Optional

import numpy as np
import torch

from ..models import trees as TR
from ..sql import types as T
from ..sql.column import ColumnData
from . import util as U
from .base import Estimator, Model
from .clustering import java_hash
from .feature import _replace_col
from .linalg import DenseVector, as_array

TREE_PARAMS = {
    "featuresCol": ("features", "features column name", str),
    "labelCol": ("label", "label column name", str),
    "predictionCol": ("prediction", "prediction column name", str),
    "maxDepth": (5, "maximum depth of the tree (>= 0)", int),
    "maxBins": (32, "max number of bins for discretizing continuous features (>= 2)", int),
    "minInstancesPerNode": (1, "minimum number of instances each child must have after split", int),
    "minWeightFractionPerNode": (0.0, "minimum fraction of the weighted sample count per child", float),
    "minInfoGain": (0.0, "minimum information gain for a split to be considered", float),
    "maxMemoryInMB": (256, "maximum memory in MB allocated to histogram aggregation", int),
    "cacheNodeIds": (False, "whether to cache node IDs per instance", bool),
    "checkpointInterval": (10, "checkpoint interval (>= 1) or -1", int),
    "weightCol": (None, "weight column name", None),
    "leafCol": ("", "leaf index column name", str),
}
CLASSIF_PARAMS = {
    "probabilityCol": ("probability", "column name for predicted class conditional probabilities", str),
    "rawPredictionCol": ("rawPrediction", "raw prediction (a.k.a. confidence) column name", str),
    "thresholds": (None, "thresholds in multi-class classification", None),
}
FOREST_PARAMS = {
    "numTrees": (20, "number of trees to train (>= 1)", int),
    "subsamplingRate": (1.0, "fraction of the training data used for learning each tree", float),
    "featureSubsetStrategy": ("auto", "number of features to consider for splits at each tree node", str),
    "bootstrap": (True, "whether bootstrap samples are used when building trees", bool),
}


GBT_PARAMS = {
    "maxIter": (20, "max number of boosting iterations (>= 0)", int),
    "stepSize": (0.1, "learning rate (a.k.a. shrinkage) in (0, 1]", float),
    "subsamplingRate": (1.0, "fraction of the training data used for learning each tree", float),
    "featureSubsetStrategy": ("all", "number of features to consider for splits at each tree node", str),
    "validationTol": (0.01, "threshold for stopping early when fit with validation is used", float),
    "validationIndicatorCol": (None, "name of the boolean column marking validation rows", None),
    "impurity": ("variance", "criterion used for information gain (variance)", str),
}


def _default_seed(jvm_name: str) -> int:
    return java_hash(jvm_name)


class TreeEstimatorMixin:
    _task = "regression"
    _forest = False

    def _tree_fit(self, df):
        x = df._feature_matrix(self.getFeaturesCol())
        ycd = df._column_data(self.getLabelCol())
        y = ycd.values.to(torch.float64)
        w = df._column_data(self.getOrDefault("weightCol")).values.to(torch.float64) \
            if self.isSet("weightCol") else None
        comm = df._comm
        num_classes = 2
        if self._task == "classification":
            ymax = float(y.max().item()) if y.numel() else 0.0
            num_classes = max(2, int(comm.max_scalar(ymax)) + 1)
            if y.numel() and bool(((y < 0) | (y != torch.floor(y))).any()):
                raise ValueError("classification labels must be non-negative integers (0, 1, 2, ...)")
        p = TR.TreeParams(task=self._task, num_classes=num_classes, impurity=self.getImpurity(),
                          max_depth=self.getMaxDepth(), max_bins=self.getMaxBins(),
                          min_instances=self.getMinInstancesPerNode(),
                          min_weight_fraction=self.getMinWeightFractionPerNode(),
                          min_info_gain=self.getMinInfoGain(), seed=int(self.getSeed()))
        if self._forest:
            p.num_trees = self.getNumTrees()
            p.subsampling_rate = self.getSubsamplingRate()
            p.bootstrap = self.getBootstrap()
            p.feature_subset = self.getFeatureSubsetStrategy()
        eng = TR.ForestEngine(x, y, p, comm, row_ids=df._row_ids, weights=w)
        # level checkpoints (cml.ml.checkpointDir): the K19 results of the completed levels
        from ..utils.checkpoint import FitCheckpoint
        ck = FitCheckpoint(df, "forest", f"{type(self).__name__}|{sorted(p.__dict__.items())}", (x, y, w))
        replay = None
        got = ck.load()
        if got is not None:
            replay = [got[1][f"l{i}"] for i in range(int(got[1]["levels"][0]))]

        def on_level(levels, done):
            if ck.due(levels):
                ck.save(levels, {"levels": np.array([levels]), **{f"l{i}": r for i, r in enumerate(done)}})
        trees = eng.fit(replay=replay, on_level=on_level if ck.enabled else None)
        ck.clear()
        return trees, x.shape[1], num_classes


class GBTEstimatorMixin(TreeEstimatorMixin):
    """Boosted ensembles (Spark ``GBTRegressor`` / ``GBTClassifier``) on the same level-wise
    histogram kernels as the forests; see ``models.trees.fit_gbt``."""
    _classification = False

    def _gbt_fit(self, df):
        x = df._feature_matrix(self.getFeaturesCol())
        y = df._column_data(self.getLabelCol()).values.to(torch.float64)
        if self._classification:
            if y.numel() and bool(((y != 0) & (y != 1)).any()):
                raise ValueError("GBTClassifier supports binary labels {0, 1} only")
            y = 2.0 * y - 1.0
        w = df._column_data(self.getOrDefault("weightCol")).values.to(torch.float64) \
            if self.isSet("weightCol") else None
        valid = df._column_data(self.getOrDefault("validationIndicatorCol")).values.to(torch.bool) \
            if self.isSet("validationIndicatorCol") else None
        loss = self.getLossType().lower()
        p = TR.TreeParams(task="regression", impurity="variance", max_depth=self.getMaxDepth(),
                          max_bins=self.getMaxBins(), min_instances=self.getMinInstancesPerNode(),
                          min_weight_fraction=self.getMinWeightFractionPerNode(),
                          min_info_gain=self.getMinInfoGain(), subsampling_rate=self.getSubsamplingRate(),
                          feature_subset=self.getFeatureSubsetStrategy(), seed=int(self.getSeed()))
        from ..utils.checkpoint import FitCheckpoint
        ck = FitCheckpoint(df, "gbt", f"{type(self).__name__}|{loss}|step={self.getStepSize()}|"
                                      f"vtol={self.getValidationTol()}|{sorted(p.__dict__.items())}", (x, y, w, valid))
        trees, tw = TR.fit_gbt(x, y, p, self.getMaxIter(), self.getStepSize(), loss, df._comm,
                               row_ids=df._row_ids, weights=w, valid=valid,
                               validation_tol=self.getValidationTol(), ckpt=ck if ck.enabled else None)
        ck.clear()
        return trees, tw, x.shape[1]


class TreeModelMixin:
    _task = "regression"
    _forest = False

    def _init_trees(self, trees: List[TR.Node], num_features: int, num_classes: int = 2,
                    tree_weights: Optional[List[float]] = None):
        self._trees = trees
        self._num_features = num_features
        self._num_classes = num_classes
        self._tree_weights = tree_weights or [1.0] * len(trees)

    @property
    def numFeatures(self) -> int:
        return self._num_features

    @property
    def featureImportances(self) -> DenseVector:
        return DenseVector(TR.feature_importances(self._trees, self._num_features))

    @property
    def depth(self) -> int:
        return TR.tree_depth(self._trees[0])

    @property
    def numNodes(self) -> int:
        return TR.num_nodes(self._trees[0])

    @property
    def toDebugString(self) -> str:
        lines = [f"{type(self).__name__}: uid={self.uid}, " + (f"numTrees={len(self._trees)}, " if self._forest else
                                                                f"depth={self.depth}, numNodes={self.numNodes}, ")
                 + f"numFeatures={self._num_features}"]
        for ti, t in enumerate(self._trees):
            if self._forest:
                lines.append(f"  Tree {ti} (weight 1.0):")
            lines += _debug(t, 2 if self._forest else 1)
        return "\n".join(lines) + "\n"

    @property
    def trees(self):
        out = []
        for t in self._trees:
            m = self._single_tree_class()()
            m._init_trees([t], self._num_features, self._num_classes)
            self._copyValues(m)
            out.append(m)
        return out

    @property
    def treeWeights(self) -> List[float]:
        return list(self._tree_weights)

    @property
    def getNumTrees(self):
        return len(self._trees)

    @property
    def totalNumNodes(self) -> int:
        return sum(TR.num_nodes(t) for t in self._trees)

    def _raw(self, x):
        kind = "variance" if self._task == "regression" else "gini"
        return TR.predict_forest(self._trees, x, kind, self._num_classes, average=True,
                                 normalize_leaves=self._forest)

    def predict(self, value) -> float:
        v = torch.as_tensor(as_array(value), dtype=torch.float64).reshape(1, -1)
        raw = self._raw(v)[0].numpy()
        return float(raw[0]) if self._task == "regression" else float(np.argmax(raw))

    def _transform(self, df):
        x = df._feature_matrix(self.getFeaturesCol())
        if self._task == "regression":
            pred = self._raw(x)[:, 0]
            return _replace_col(df, self.getPredictionCol(), ColumnData(pred.contiguous(), None, T.DoubleType()))
        kind = "gini"
        raw = TR.predict_forest(self._trees, x, kind, self._num_classes, average=False,
                                normalize_leaves=self._forest)
        thr = self.getOrDefault("thresholds") if self.isDefined("thresholds") else None
        prob, pred = TR.forest_vote(raw, thr)
        out = df
        if self.getRawPredictionCol():
            out = _replace_col(out, self.getRawPredictionCol(), ColumnData(raw, None, T.VectorUDT()))
        if self.getProbabilityCol():
            out = _replace_col(out, self.getProbabilityCol(), ColumnData(prob, None, T.VectorUDT()))
        return _replace_col(out, self.getPredictionCol(), ColumnData(pred, None, T.DoubleType()))

    # ------------------------------------------------------------------ persistence
    def _save_impl(self, path):
        import pyarrow as pa
        extra = {"numFeatures": self._num_features}
        if self._task == "classification":
            extra["numClasses"] = self._num_classes
        if self._forest:
            extra["numTrees"] = len(self._trees)
        U.write_metadata(self, path, extra=extra)
        if not self._forest:
            rows = [_node_row(n) for n in TR.preorder(self._trees[0])]
            U.write_parquet(path, "data", pa.Table.from_pylist(rows, schema=node_schema()))
            return
        rows = []
        for ti, t in enumerate(self._trees):
            for n in TR.preorder(t):
                rows.append({"treeID": ti, "nodeData": _node_row(n)})
        U.write_parquet(path, "data", pa.Table.from_pylist(
            rows, schema=pa.schema([pa.field("treeID", pa.int32(), nullable=False),
                                    pa.field("nodeData", pa.struct(list(node_schema())))])))
        meta_rows = []
        est_cls = self._single_tree_class().__name__
        for ti in range(len(self._trees)):
            md = {"class": U._JVM.get(est_cls, est_cls), "timestamp": 0, "sparkVersion": U.SPARK_VERSION,
                  "uid": f"{est_cls}_tree{ti}", "paramMap": {}, "defaultParamMap": {}}
            meta_rows.append({"treeID": ti, "metadata": json.dumps(md), "weights": float(self._tree_weights[ti])})
        U.write_parquet(path, "treesMetadata", pa.Table.from_pylist(
            meta_rows, schema=pa.schema([pa.field("treeID", pa.int32(), nullable=False), ("metadata", pa.string()),
                                         pa.field("weights", pa.float64(), nullable=False)])))

    @classmethod
    def _load_impl(cls, path, md):
        m = cls()
        U.apply_params(m, md)
        nf = int(md.get("numFeatures", 0))
        nc = int(md.get("numClasses", 2))
        if not cls._forest:
            rows = U.read_parquet(path, "data").to_pylist()
            m._init_trees([_rebuild(rows, cls._task)], nf, nc)
            return m
        rows = U.read_parquet(path, "data").to_pylist()
        by_tree = {}
        for r in rows:
            by_tree.setdefault(r["treeID"], []).append(r["nodeData"])
        weights = {r["treeID"]: r["weights"] for r in U.read_parquet(path, "treesMetadata").to_pylist()}
        ids = sorted(by_tree)
        m._init_trees([_rebuild(by_tree[i], cls._task) for i in ids], nf, nc, [weights.get(i, 1.0) for i in ids])
        return m


def node_schema():
    import pyarrow as pa
    return pa.schema([
        pa.field("id", pa.int32(), nullable=False), pa.field("prediction", pa.float64(), nullable=False),
        pa.field("impurity", pa.float64(), nullable=False),
        ("impurityStats", pa.list_(pa.field("element", pa.float64(), nullable=False))),
        pa.field("rawCount", pa.int64(), nullable=False), pa.field("gain", pa.float64(), nullable=False),
        pa.field("leftChild", pa.int32(), nullable=False), pa.field("rightChild", pa.int32(), nullable=False),
        ("split", pa.struct([pa.field("featureIndex", pa.int32(), nullable=False),
                             ("leftCategoriesOrThreshold", pa.list_(pa.field("element", pa.float64(),
                                                                             nullable=False))),
                             pa.field("numCategories", pa.int32(), nullable=False)])),
    ])


def _node_row(n: TR.Node) -> dict:
    leaf = n.is_leaf
    return {"id": n.id, "prediction": float(n.prediction), "impurity": float(n.impurity),
            "impurityStats": [float(v) for v in np.asarray(n.stats, dtype=np.float64)],
            "rawCount": int(round(n.count)), "gain": float(n.gain) if not leaf else -1.0,
            "leftChild": n.left.id if not leaf else -1, "rightChild": n.right.id if not leaf else -1,
            "split": {"featureIndex": n.feature if not leaf else -1,
                      "leftCategoriesOrThreshold": [float(n.threshold)] if not leaf else [],
                      "numCategories": -1}}


def _rebuild(rows: List[dict], task: str) -> TR.Node:
    by_id = {r["id"]: r for r in rows}
    nodes = {}
    for r in rows:
        st = np.asarray(r["impurityStats"], dtype=np.float64)
        nodes[r["id"]] = TR.Node(id=r["id"], prediction=r["prediction"], impurity=r["impurity"], stats=st,
                                 count=float(st[0]) if task == "regression" else float(st.sum()), gain=r["gain"])
    for r in rows:
        n = nodes[r["id"]]
        if r["leftChild"] >= 0:
            n.feature = r["split"]["featureIndex"]
            n.threshold = r["split"]["leftCategoriesOrThreshold"][0]
            n.left = nodes[r["leftChild"]]
            n.right = nodes[r["rightChild"]]
    return nodes[0] if 0 in nodes else nodes[min(nodes)]


def _debug(n: TR.Node, indent: int) -> List[str]:
    pad = "  " * indent
    if n.is_leaf:
        return [f"{pad}Predict: {n.prediction}"]
    out = [f"{pad}If (feature {n.feature} <= {n.threshold})"]
    out += _debug(n.left, indent + 1)
    out.append(f"{pad}Else (feature {n.feature} > {n.threshold})")
    out += _debug(n.right, indent + 1)
    return out


class GBTModelMixin(TreeModelMixin):
    """Margin F(x) = sum_m w_m tree_m(x) (one K21 launch over all trees, leaf values pre-scaled by
    the tree weights).  Trees are regression trees, so persistence is the ensemble layout with
    ``treesMetadata.weights`` = the boosting weights."""
    _task = "regression"
    _forest = True
    _classification = False

    def _margin(self, x):
        return TR.predict_forest(self._trees, x, "variance", 1, average=False, normalize_leaves=False,
                                 tree_weights=self._tree_weights)[:, 0]

    def _raw(self, x):
        return self._margin(x)[:, None]

    @property
    def featureImportances(self) -> DenseVector:
        return DenseVector(TR.feature_importances(self._trees, self._num_features, per_tree_normalization=False))

    def predict(self, value) -> float:
        v = torch.as_tensor(as_array(value), dtype=torch.float64).reshape(1, -1)
        f = float(self._margin(v)[0])
        return f if not self._classification else float(f > 0)

    def evaluateEachIteration(self, dataset, loss: Optional[str] = None) -> List[float]:
        """Mean loss of the first m trees for m = 1..numTrees (Spark ``evaluateEachIteration``)."""
        x = dataset._feature_matrix(self.getFeaturesCol())
        y = dataset._column_data(self.getLabelCol()).values.to(torch.float64)
        if self._classification:
            y = 2.0 * y - 1.0
        loss = (loss or self.getLossType()).lower()
        comm = dataset._comm
        f = torch.zeros_like(y)
        den = max(comm.sum_scalar(float(y.numel())), 1.0)
        out = []
        for t, w in zip(self._trees, self._tree_weights):
            f += w * TR.predict_tree(t, x.to(torch.float64))
            out.append(comm.sum_scalar(float(TR.gbt_loss(loss, f, y).sum().item())) / den)
        return out

    def _transform(self, df):
        x = df._feature_matrix(self.getFeaturesCol())
        f = self._margin(x)
        if not self._classification:
            return _replace_col(df, self.getPredictionCol(), ColumnData(f.contiguous(), None, T.DoubleType()))
        raw = torch.stack([-f, f], 1)
        p1 = 1.0 / (1.0 + torch.exp(torch.clamp(-2.0 * f, max=700.0)))
        prob = torch.stack([1.0 - p1, p1], 1)
        thr = self.getOrDefault("thresholds") if self.isDefined("thresholds") else None
        if thr:
            t = torch.as_tensor(np.asarray(thr, dtype=np.float64), device=prob.device)
            pred = torch.argmax(prob / t.clamp(min=1e-300), 1).to(torch.float64)
        else:
            pred = (f > 0).to(torch.float64)
        out = df
        if self.getRawPredictionCol():
            out = _replace_col(out, self.getRawPredictionCol(), ColumnData(raw, None, T.VectorUDT()))
        if self.getProbabilityCol():
            out = _replace_col(out, self.getProbabilityCol(), ColumnData(prob, None, T.VectorUDT()))
        return _replace_col(out, self.getPredictionCol(), ColumnData(pred, None, T.DoubleType()))
