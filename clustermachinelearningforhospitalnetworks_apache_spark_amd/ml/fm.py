"""Factorization machines: FMRegressor and FMClassifier (pyspark.ml.regression / classification).

A second-order FM models pairwise feature interactions (occupancy x emergency visits, season x
admissions) with a rank-``factorSize`` factorisation on top of the linear model the reference
fits (ref.py:145-148):

    ŷ = b + Σ_i w_i x_i + ½ Σ_f [ (Σ_i v_if x_i)² − Σ_i v_if² x_i² ]

MI355X-first: the interaction term is two [n, d] x [d, f] GEMMs on the device (hipBLASLt) — X·V
and X²·V² — instead of Spark's per-row loops, and the gradient of the flat parameter vector comes
from autograd over the same GEMMs; every iteration all-reduces one (1 + d + d·f + 1)-vector of
gradient sums. Spark's optimiser semantics: ``solver='adamW'`` (β1 0.9, β2 0.999, ε 1e-8, weight
decay regParam) or ``'gd'`` (step stepSize / sqrt(iteration)), mini-batches of ``miniBatchFraction``
drawn per iteration by hash(seed + iteration, row id) (GPU-count invariant), stop when the parameter
change is below tol · max(‖w‖, 1).
"""
from __future__ import annotations

import math
from typing import Optional

import numpy as np
import torch

from ..sql import types as T
from ..sql.column import ColumnData
from . import util as U
from .base import Estimator, Model
from .feature import _replace_col
from .linalg import DenseMatrix, DenseVector, as_array

_FM_PARAMS = {
    "featuresCol": ("features", "features column name", str),
    "labelCol": ("label", "label column name", str),
    "predictionCol": ("prediction", "prediction column name", str),
    "factorSize": (8, "dimensionality of the factor vectors", int),
    "fitIntercept": (True, "whether to fit an intercept term", bool),
    "fitLinear": (True, "whether to fit linear term (aka 1-way term)", bool),
    "regParam": (0.0, "the magnitude of L2-regularization", float),
    "miniBatchFraction": (1.0, "fraction of the input data set used for one iteration of gradient descent", float),
    "initStd": (0.01, "standard deviation of initial coefficients", float),
    "maxIter": (100, "max number of iterations (>= 0)", int),
    "stepSize": (1.0, "step size to be used for each iteration of optimization (> 0)", float),
    "tol": (1e-6, "convergence tolerance for iterative algorithms (>= 0)", float),
    "solver": ("adamW", "the solver algorithm for optimization: gd, adamW", str),
    "seed": (None, "random seed", None),
}
_FMC_PARAMS = dict(_FM_PARAMS, **{
    "probabilityCol": ("probability", "column name for predicted class conditional probabilities", str),
    "rawPredictionCol": ("rawPrediction", "raw prediction (a.k.a. confidence) column name", str),
    "thresholds": (None, "thresholds in multi-class classification", None),
})


def _fm_scores(x: torch.Tensor, b, w, V) -> torch.Tensor:
    xv = x @ V
    x2v2 = (x * x) @ (V * V)
    return b + x @ w + 0.5 * (xv * xv - x2v2).sum(1)


class _FMBase(Estimator):
    _loss = "squared"

    def __init__(self, **kwargs):
        super().__init__(**kwargs)
        for k in ("seed", "thresholds"):
            self._defaultParamMap.pop(k, None)

    def _fit(self, df):
        from ..utils import rng
        from .tree_models import _default_seed
        x = df._feature_matrix(self.getFeaturesCol()).to(torch.float64)
        n, d = x.shape
        y = df._column_data(self.getLabelCol()).values.to(torch.float64)
        comm = df._comm
        if self._loss == "logistic":
            bad = comm.max_scalar(float(((y != 0) & (y != 1)).any().item()) if y.numel() else 0.0)
            if bad:
                raise ValueError("FMClassifier only supports binary labels 0 and 1")
        f = self.getFactorSize()
        seed = int(self.getOrDefault("seed")) if self.isSet("seed") else _default_seed(U.jvm_class(self))
        g = np.random.default_rng(seed & 0xFFFFFFFF)
        p = np.zeros(1 + d + d * f)
        p[1 + d:] = g.normal(0.0, self.getInitStd(), d * f)
        fi, fl = self.getFitIntercept(), self.getFitLinear()
        lam, lr0, frac = self.getRegParam(), self.getStepSize(), self.getMiniBatchFraction()
        solver = self.getSolver()
        if solver not in ("adamW", "gd"):
            raise ValueError(f"FM: unknown solver {solver!r}")
        m1 = np.zeros_like(p)
        m2 = np.zeros_like(p)
        hist = []
        rows = df._row_ids
        it = 0
        for it in range(1, self.getMaxIter() + 1):
            if frac < 1.0:
                sel = rng.uniform(rows, seed + it, stream=11) < frac
                xb, yb = x[sel], y[sel]
            else:
                xb, yb = x, y
            pt = torch.as_tensor(p, device=x.device).requires_grad_(True)
            s = _fm_scores(xb, pt[0], pt[1:1 + d], pt[1 + d:].reshape(d, f))
            if self._loss == "logistic":
                loss = (torch.nn.functional.softplus(s) - yb * s).sum()
            else:
                loss = 0.5 * ((s - yb) ** 2).sum()
            grad, = torch.autograd.grad(loss, pt)
            msg = torch.cat([grad.detach(), loss.detach().reshape(1),
                             torch.tensor([float(yb.numel())], dtype=torch.float64, device=x.device)])
            comm.allreduce_(msg)
            o = msg.cpu().numpy()
            cnt = max(o[-1], 1.0)
            gv = o[:-2] / cnt
            hist.append(float(o[-2]) / cnt)
            if not fi:
                gv[0] = 0.0
            if not fl:
                gv[1:1 + d] = 0.0
            prev = p.copy()
            if solver == "adamW":
                b1, b2, eps = 0.9, 0.999, 1e-8
                m1 = b1 * m1 + (1 - b1) * gv
                m2 = b2 * m2 + (1 - b2) * gv * gv
                mh = m1 / (1 - b1 ** it)
                vh = m2 / (1 - b2 ** it)
                p = p - lr0 * (mh / (np.sqrt(vh) + eps) + lam * p)
            else:
                p = p - (lr0 / math.sqrt(it)) * (gv + lam * p)
            if not fi:
                p[0] = 0.0
            if not fl:
                p[1:1 + d] = 0.0
            if np.linalg.norm(p - prev) < self.getTol() * max(np.linalg.norm(p), 1.0):
                break
        model = self._model_cls(float(p[0]), p[1:1 + d], p[1 + d:].reshape(d, f))
        self._copyValues(model)
        model._hist, model._iters = hist, it
        return model


class _FMModelBase(Model):
    def __init__(self, intercept: float = 0.0, linear=None, factors=None):
        super().__init__()
        self._b = float(intercept)
        self._w = np.asarray(linear if linear is not None else [], dtype=np.float64)
        self._V = np.asarray(factors if factors is not None else np.zeros((0, 0)), dtype=np.float64)
        self._hist, self._iters = [], 0

    @property
    def intercept(self) -> float:
        return self._b

    @property
    def linear(self) -> DenseVector:
        return DenseVector(self._w)

    @property
    def factors(self) -> DenseMatrix:
        return DenseMatrix(self._V.shape[0], self._V.shape[1], self._V.T.reshape(-1))

    @property
    def numFeatures(self) -> int:
        return int(self._w.size)

    def _scores(self, x: torch.Tensor) -> torch.Tensor:
        dev = x.device
        return _fm_scores(x.to(torch.float64), self._b, torch.as_tensor(self._w, device=dev),
                          torch.as_tensor(self._V, device=dev))

    def _save_impl(self, path):
        import pyarrow as pa
        U.write_metadata(self, path)
        U.write_parquet(path, "data", pa.Table.from_pylist(
            [{"intercept": self._b, "linear": U.vector_struct(self._w), "factors": U.matrix_struct(self._V)}],
            schema=pa.schema([pa.field("intercept", pa.float64(), False), ("linear", U.vector_arrow_type()),
                              ("factors", U.matrix_arrow_type())])))

    @classmethod
    def _load_impl(cls, path, md):
        r = U.read_parquet(path, "data").to_pylist()[0]
        m = cls(r["intercept"], U.vector_from_struct(r["linear"]), U.matrix_from_struct(r["factors"]))
        U.apply_params(m, md)
        return m


class FMRegressionModel(_FMModelBase):
    _params = _FM_PARAMS

    def _transform(self, df):
        s = self._scores(df._feature_matrix(self.getFeaturesCol()))
        return _replace_col(df, self.getPredictionCol(), ColumnData(s, None, T.DoubleType()))

    def predict(self, value) -> float:
        return float(self._scores(torch.as_tensor(as_array(value), dtype=torch.float64)[None, :])[0])


class FMClassificationModel(_FMModelBase):
    _params = _FMC_PARAMS

    @property
    def numClasses(self) -> int:
        return 2

    def _transform(self, df):
        s = self._scores(df._feature_matrix(self.getFeaturesCol()))
        p1 = torch.sigmoid(s)
        prob = torch.stack([1 - p1, p1], 1)
        out = df
        if self.getRawPredictionCol():
            out = _replace_col(out, self.getRawPredictionCol(), ColumnData(torch.stack([-s, s], 1), None,
                                                                          T.VectorUDT()))
        if self.getProbabilityCol():
            out = _replace_col(out, self.getProbabilityCol(), ColumnData(prob, None, T.VectorUDT()))
        thr = self.getOrDefault("thresholds") if self.isSet("thresholds") else None
        if thr:
            pred = torch.argmax(prob / torch.as_tensor(np.asarray(thr, dtype=np.float64), device=prob.device), 1)
        else:
            pred = (p1 > 0.5).to(torch.int64)
        return _replace_col(out, self.getPredictionCol(), ColumnData(pred.to(torch.float64), None, T.DoubleType()))

    def predict(self, value) -> float:
        s = float(self._scores(torch.as_tensor(as_array(value), dtype=torch.float64)[None, :])[0])
        return float(s > 0.0)

    def predictProbability(self, value) -> DenseVector:
        s = float(self._scores(torch.as_tensor(as_array(value), dtype=torch.float64)[None, :])[0])
        p1 = 1.0 / (1.0 + math.exp(-s))
        return DenseVector([1 - p1, p1])


class FMRegressor(_FMBase):
    _params = _FM_PARAMS
    _loss = "squared"
    _model_cls = FMRegressionModel


class FMClassifier(_FMBase):
    _params = _FMC_PARAMS
    _loss = "logistic"
    _model_cls = FMClassificationModel


__all__ = ["FMRegressor", "FMRegressionModel", "FMClassifier", "FMClassificationModel"]
