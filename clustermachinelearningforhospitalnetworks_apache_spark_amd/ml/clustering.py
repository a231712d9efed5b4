"""KMeans estimator/model (the [NS] headline workload; no KMeans in the reference,
SURVEY.md §0.3) on the distributed Lloyd engine of ``models/kmeans.py``.

Spark defaults: k=2, maxIter=20, tol=1e-4, initMode="k-means||", initSteps=2,
distanceMeasure="euclidean", seed = Java hashCode of the class name.
Precision (session conf ``cml.ml.kmeans.precision``, default "auto"): f32/f64 feature
vectors — the reference's assembled DoubleType/IntegerType columns (ref.py:64-72,
ref.py:134-136), and this engine's default ``cml.ml.features.dtype`` — run the f64
reference algorithm on the device (``kmeans_exact.hip``: f64 distances, deterministic
f64 sums of the rows as given), so GPU fits agree with the CPU f64 fit
(tests/test_kmeans_exact_gpu.py). bf16 / fp8 feature vectors (or ``precision=bf16``)
run the MFMA path: distances of the bf16-rounded rows and centres, exact f64 sums of
those rounded rows — values outside bf16's 8 mantissa bits are rounded first (an
occupancy of 387 becomes 388).
"""
from __future__ import annotations

import os
from typing import List, Optional

import numpy as np
import torch

from ..models.kmeans import LloydEngine
from ..utils import checkpoint as ckpt
from ..utils.trace import trace
from ..sql import types as T
from ..sql.column import ColumnData
from . import util as U
from .base import Estimator, Model
from .feature import _replace_col
from .linalg import DenseVector, as_array


from .util import java_hash  # noqa: E402  (re-exported: Spark's default seeds are class-name hashes)


_KMEANS_PARAMS = {
    "featuresCol": ("features", "features column name", str),
    "predictionCol": ("prediction", "prediction column name", str),
    "k": (2, "number of clusters to create (> 1)", int),
    "maxIter": (20, "max number of iterations (>= 0)", int),
    "tol": (1e-4, "convergence tolerance for iterative algorithms (>= 0)", float),
    "initMode": ("k-means||", "initialization algorithm: 'random' or 'k-means||'", str),
    "initSteps": (2, "number of steps for k-means|| (> 0)", int),
    "seed": (java_hash("org.apache.spark.ml.clustering.KMeans"), "random seed", int),
    "distanceMeasure": ("euclidean", "'euclidean' or 'cosine'", str),
    "weightCol": (None, "weight column name", None),
    "solver": ("auto", "'auto', 'row' or 'block'", str),
    "maxBlockSizeInMB": (0.0, "maximum memory in MB for stacking input data into blocks", float),
}


class KMeans(Estimator):
    _params = _KMEANS_PARAMS

    def __init__(self, featuresCol=None, predictionCol=None, k=None, initMode=None, initSteps=None, tol=None,
                 maxIter=None, seed=None, distanceMeasure=None, weightCol=None, solver=None, maxBlockSizeInMB=None):
        super().__init__(featuresCol=featuresCol, predictionCol=predictionCol, k=k, initMode=initMode,
                         initSteps=initSteps, tol=tol, maxIter=maxIter, seed=seed, distanceMeasure=distanceMeasure,
                         weightCol=weightCol, solver=solver, maxBlockSizeInMB=maxBlockSizeInMB)
        self._defaultParamMap.pop("weightCol", None)

    def _fit(self, df):
        measure = self.getOrDefault("distanceMeasure")
        if measure not in ("euclidean", "cosine"):
            raise ValueError(f"distanceMeasure must be 'euclidean' or 'cosine', got {measure!r}")
        spherical = measure == "cosine"
        x = df._feature_matrix(self.getFeaturesCol())
        weights = None
        if self.isSet("weightCol") and self.getOrDefault("weightCol"):
            weights = _weights(df, self.getOrDefault("weightCol"), x.device)
        d = x.shape[1]
        k = self.getK()
        comm = df._comm
        seed = int(self.getSeed())
        conf = df._session.conf
        # exact bound-pruned Lloyd steps (models/kmeans.py _step_prune): same centres, fewer rows read
        pv = conf.get("cml.ml.kmeans.prune", None)
        prune = None if pv is None else str(pv).lower() in ("1", "true")
        precision = conf.get("cml.ml.kmeans.precision", "auto")
        rv = conf.get("cml.ml.kmeans.refreshInterval", None)
        refresh = None if rv is None else int(rv)
        # an out-of-core feature column (host rows on a GPU session): streamed Lloyd passes
        dev = df._device if (not x.is_cuda and df._device.type == "cuda") else None
        eng = LloydEngine(x, d, k, comm, row_ids=df._row_ids, spherical=spherical, prune=prune,
                          precision=precision, weights=weights, refresh_interval=refresh, device=dev)
        ckdir = conf.get("cml.ml.checkpointDir", None)
        every = int(conf.get("cml.ml.checkpointInterval", 10))
        ckname = ckkey = None
        if ckdir:
            n_global = int(comm.sum_scalar(float(eng.n)))
            # the key identifies the fit (shape, params and a data fingerprint), and the checkpoint name
            # is derived from it: a restarted process, whose estimator has a new uid, finds it again
            fp = _fingerprint(x, comm)
            if weights is not None:
                fp += "|w=" + _fingerprint(weights.reshape(-1, 1), comm)
            ckkey = (f"kmeans|n={n_global}|d={d}|k={k}|seed={seed}|init={self.getInitMode()}|"
                     f"steps={self.getInitSteps()}|tol={self.getTol()}|measure={measure}|data={fp}")
            ckname = ckpt.name_for("kmeans", ckkey)
        # rank 0 decides and broadcasts, so every rank resumes from the same iteration or none does
        resumed = ckpt.load_shared(ckdir, ckname, ckkey, comm) if ckdir else None
        start = 0
        if resumed is not None:
            start, arrs = resumed
            init = arrs["centers"]
            if init.shape[0] < k:
                eng = LloydEngine(x, d, init.shape[0], comm, row_ids=df._row_ids, spherical=spherical, prune=prune,
                                  precision=precision, weights=weights, refresh_interval=refresh, device=dev)
        elif self.getInitMode() == "random":
            with trace("kmeans.init"):
                init = eng.init_random(seed)
        else:
            with trace("kmeans.init"):
                init = eng.init_kmeans_parallel(seed, self.getInitSteps(), as_device=True)
            k_eff = getattr(eng, "k_effective", k)
            if k_eff < k:
                init = init[:k_eff]
                eng = LloydEngine(x, d, k_eff, comm, row_ids=df._row_ids, spherical=spherical, prune=prune,
                                  precision=precision, weights=weights, device=dev)
        eng.set_centers(init)

        def on_iter(it):
            if ckdir and (it % max(every, 1) == 0):
                ckpt.save(ckdir, ckname, ckkey, it, {"centers": eng.centers.cpu().numpy()}, comm)

        # without checkpoints a tol > 0 fit reads its convergence flag lagged (models/kmeans.py _fit_lagged)
        iters = eng.fit(self.getMaxIter(), self.getTol(), start_iter=start, on_iter=on_iter if ckdir else None)
        if ckdir:
            comm.barrier()
            ckpt.clear(ckdir, ckname, comm)
        # trainingCost is the last iteration's cost (Spark computes it while training: here from the f64
        # sums and norms the engine holds, no pass over X); clusterSizes: one pruned assign against the
        # final centres, its counts and their all-reduce are enqueued here on every rank (no host read),
        # so reading the summary later is no collective and the engine is released when fit returns. The cost
        # is enqueued first: the final assignment then updates the engine's own labels and bounds in place
        # (consume=True: nothing steps this engine again). On a GPU the centres and the cost go to pinned
        # host memory BEFORE the final assignment is enqueued, and the host waits for those copies only: the
        # model and the summary are built while the device runs the final assignment
        cost = eng.last_cost
        if eng.device.type == "cuda":
            c_h = torch.empty(eng.centers.shape, dtype=torch.float64, pin_memory=True)
            c_h.copy_(eng.centers, non_blocking=True)
            cost_h = None
            if cost is not None:
                cost_h = torch.empty((), dtype=cost.dtype, pin_memory=True)
                cost_h.copy_(cost, non_blocking=True)
            ready = torch.cuda.Event()
            ready.record()
            sizes = eng.cluster_sizes_async(consume=True)
            ready.synchronize()
            centers = c_h.numpy()
            tc = float("nan") if cost_h is None else float(cost_h) / (2.0 if eng.spherical else 1.0)
        else:
            sizes = eng.cluster_sizes_async(consume=True)
            centers = eng.centers.cpu().numpy()
            tc = eng.training_cost()
        model = KMeansModel(centers)
        self._copyValues(model)
        model._attach_summary(KMeansSummary(model, df, eng.k, iters, tc, sizes))
        return model


def _weights(df, col: str, device) -> torch.Tensor:
    """The weight column as f64 (Spark's checkNonNegativeWeight: finite, >= 0, not null).

    The check is agreed over every rank before anything is raised (one max all-reduce of a
    [has null, has bad value] flag pair): a bad weight on one shard makes every rank raise the same
    ValueError instead of leaving the others blocked in the init collectives."""
    cd = df._column_data(col)
    nulls = False
    if cd.is_host:
        from ..sql.dataframe import column_to_python
        vals = column_to_python(cd)
        nulls = any(v is None for v in vals)
        w = torch.as_tensor(np.asarray([0.0 if v is None else v for v in vals], dtype=np.float64), device=device)
    else:
        nulls = cd.valid is not None and not bool(cd.valid.all())
        w = cd.values.to(device=device, dtype=torch.float64).reshape(-1)
    bad = bool(w.numel()) and not bool(((w >= 0) & torch.isfinite(w)).all())
    comm = df._comm
    flags = torch.tensor([float(nulls), float(bad)], dtype=torch.float64, device=comm.device)
    if comm.is_distributed:
        comm.allreduce_(flags, op="max")
    if flags[0].item() > 0:
        raise ValueError(f"weight column {col!r} contains nulls")
    if flags[1].item() > 0:
        raise ValueError(f"weights must be finite and non-negative (column {col!r})")
    return w


def _fingerprint(x: torch.Tensor, comm) -> str:
    """Global (Σx, Σx²) of the feature matrix in float64 (utils/checkpoint.py data_fingerprint)."""
    return ckpt.data_fingerprint(x, comm)


class KMeansModel(Model):
    _params = _KMEANS_PARAMS

    def __init__(self, centers=None):
        super().__init__()
        self._centers = np.asarray(centers if centers is not None else np.zeros((0, 0)), dtype=np.float64)
        self._summary = None

    def clusterCenters(self) -> List[np.ndarray]:
        return [c.copy() for c in self._centers]

    @property
    def numFeatures(self) -> int:
        return int(self._centers.shape[1])

    def _cosine(self) -> bool:
        return self.getOrDefault("distanceMeasure") == "cosine"

    def predict(self, value) -> int:
        v = as_array(value)
        if self._cosine():  # CosineDistanceMeasure: 1 - cos, centres are unit length
            nv = np.linalg.norm(v)
            if nv == 0:
                raise ValueError("Cosine distance is not defined for zero-length vectors.")
            return int((1.0 - self._centers @ v / nv).argmin())
        return int(((self._centers - v) ** 2).sum(1).argmin())

    def _assign(self, df, want_dist: bool = True):
        """(labels, distance) per local row: squared euclidean, or 1 - cos for distanceMeasure="cosine"
        (unit rows against the unit centres: ||x - c||² / 2). f32/f64 device rows (the reference's Double
        features) are assigned on the MFMA screen with the exact path's labels and distances
        (LloydEngine.screen_assign); ``want_dist=False`` skips the distances where only labels are read."""
        x = df._feature_matrix(self.getFeaturesCol())
        if not x.is_cuda and df._device.type == "cuda" and not self._cosine():
            # out-of-core column: the streamed MFMA assign (models/kmeans.py _assign_all)
            eng = LloydEngine(x, x.shape[1], len(self._centers), df._comm, device=df._device)
            lab, dist = eng.assign(torch.as_tensor(self._centers))
            return lab.long(), dist.to(torch.float64)
        c = torch.as_tensor(self._centers, device=x.device)
        cos = self._cosine()
        prec = df._session.conf.get("cml.ml.kmeans.precision", "auto").lower()
        if x.is_cuda and (prec == "bf16" or x.dtype not in (torch.float32, torch.float64)):
            from ..models.kmeans import assign_gpu, to_device_matrix, unit_rows
            xm = to_device_matrix(unit_rows(x) if cos else x, x.shape[1])
            lab, dist = assign_gpu(xm, xm.shape[1], x.shape[1], c)
            dist = dist.to(torch.float64)
            return lab.long(), (dist / 2.0 if cos else dist)
        from ..ops.kmeans_ops import assign_reference
        if (x.is_cuda and not cos and x.dtype in (torch.float32, torch.float64) and prec in ("auto", "screen")
                and os.environ.get("CML_KMEANS_SCREEN", "1") != "0"
                and LloydEngine.screen_applies(int(x.shape[1]), len(self._centers))):
            from ..parallel.comm import local_comm
            eng = LloydEngine(x, int(x.shape[1]), len(self._centers), local_comm(), precision="screen")
            return eng.screen_assign(c, want_dist=want_dist)
        if cos:
            from ..models.kmeans import unit_rows
            lab, dist = assign_reference(unit_rows(x), c)
            return lab, dist / 2.0
        return assign_reference(x, c)

    def _transform(self, df):
        """The prediction column is lazy (sql/column.py LazyColumnData): assigned on first read, never
        when nothing downstream reads it (a Pipeline stage whose output the next stage ignores)."""
        from ..sql.column import LazyColumnData

        def thunk():
            lab, _ = self._assign(df, want_dist=False)
            return lab.to(torch.int32), None
        return _replace_col(df, self.getPredictionCol(), LazyColumnData(thunk, df._nrows, T.IntegerType()))

    def computeCost(self, df) -> float:
        _, dist = self._assign(df)
        return df._comm.sum_scalar(float(dist.sum().item()) if dist.numel() else 0.0)

    def _save_impl(self, path):
        import pyarrow as pa
        U.write_metadata(self, path)
        rows = [{"clusterIdx": i, "clusterCenter": U.vector_struct(c)} for i, c in enumerate(self._centers)]
        U.write_parquet(path, "data", pa.Table.from_pylist(
            rows, schema=pa.schema([pa.field("clusterIdx", pa.int32(), nullable=False),
                                    ("clusterCenter", U.vector_arrow_type())])))

    @classmethod
    def _load_impl(cls, path, md):
        rows = sorted(U.read_parquet(path, "data").to_pylist(), key=lambda r: r["clusterIdx"])
        m = cls(np.stack([U.vector_from_struct(r["clusterCenter"]) for r in rows]) if rows else None)
        U.apply_params(m, md)
        return m


class KMeansSummary:
    """Spark's KMeansSummary. ``clusterSizes`` may be given as a zero-argument callable: it is then
    evaluated on first read (Spark's lazy val). KMeans.fit passes the reader of counts whose all-reduce
    every rank already enqueued, so any subset of ranks may read it."""

    def __init__(self, model, df, k, num_iter, cost, sizes):
        self._model = model
        self._df = df
        self.k = k
        self.numIter = num_iter
        self.trainingCost = cost
        self._sizes = sizes
        self.featuresCol = model.getFeaturesCol()
        self.predictionCol = model.getPredictionCol()

    @property
    def clusterSizes(self) -> List[int]:
        if callable(self._sizes):
            self._sizes = list(self._sizes())
        return self._sizes

    @property
    def predictions(self):
        return self._model.transform(self._df)

    @property
    def cluster(self):
        return self.predictions.select(self.predictionCol)


from .bisecting import BisectingKMeans, BisectingKMeansModel  # noqa: E402,F401
from .gmm import GaussianMixture, GaussianMixtureModel, GaussianMixtureSummary  # noqa: E402,F401
from .lda import LDA, DistributedLDAModel, LocalLDAModel  # noqa: E402,F401
from .pic import PowerIterationClustering  # noqa: E402,F401
