"""NaiveBayes (Spark ``org.apache.spark.ml.classification.NaiveBayes``): multinomial,
bernoulli and gaussian model types.

A classifier for the reference's high/low-LOS label (ref.py:176-190) that trains in
one or two passes.  Per-class statistics are device ``index_add`` reductions of the
resident shard into a [C, d] float64 buffer followed by one all-reduce (gaussian: a
second pass of squared deviations about the global class means, so the variance is
exact and independent of the world size).  Spark's formulas: multinomial/bernoulli
use additive smoothing ``smoothing``; gaussian adds ``1e-9 * max feature variance``
to every variance and uses unsmoothed priors.
"""
from __future__ import annotations

import math

import numpy as np
import torch

from ..sql import types as T
from ..sql.column import ColumnData
from . import util as U
from .base import Estimator, Model
from .feature import _replace_col
from .linalg import DenseMatrix, DenseVector, as_array

_NB_PARAMS = {
    "featuresCol": ("features", "features column name", str),
    "labelCol": ("label", "label column name", str),
    "predictionCol": ("prediction", "prediction column name", str),
    "probabilityCol": ("probability", "column name for predicted class conditional probabilities", str),
    "rawPredictionCol": ("rawPrediction", "raw prediction (a.k.a. confidence) column name", str),
    "smoothing": (1.0, "the smoothing parameter (>= 0)", float),
    "modelType": ("multinomial", "multinomial | bernoulli | gaussian", str),
    "thresholds": (None, "thresholds in multi-class classification", None),
    "weightCol": (None, "weight column name", None),
}


class NaiveBayes(Estimator):
    _params = dict(_NB_PARAMS)

    def __init__(self, **kwargs):
        super().__init__(**kwargs)
        for k in ("weightCol", "thresholds"):
            self._defaultParamMap.pop(k, None)

    def _fit(self, df):
        mt = self.getModelType().lower()
        if mt not in ("multinomial", "bernoulli", "gaussian"):
            raise ValueError(f"unsupported modelType {mt!r}")
        x = df._feature_matrix(self.getFeaturesCol()).to(torch.float64)
        y = df._column_data(self.getLabelCol()).values.to(torch.float64)
        w = df._column_data(self.getOrDefault("weightCol")).values.to(torch.float64) \
            if self.isSet("weightCol") else torch.ones_like(y)
        comm = df._comm
        if y.numel() and bool(((y < 0) | (y != torch.floor(y))).any()):
            raise ValueError("NaiveBayes labels must be non-negative integers")
        if mt == "multinomial" and x.numel() and bool((x < 0).any()):
            raise ValueError("multinomial NaiveBayes requires non-negative feature values")
        if mt == "bernoulli" and x.numel() and bool(((x != 0) & (x != 1)).any()):
            raise ValueError("bernoulli NaiveBayes requires 0/1 feature values")
        C = int(comm.max_scalar(float(y.max().item()) if y.numel() else 0.0)) + 1
        d = x.shape[1]
        yi = y.long()
        msg = torch.zeros(C * (d + 1), dtype=torch.float64, device=x.device)
        sums = msg[:C * d].view(C, d)
        cnt = msg[C * d:]
        from ..ops.group_ops import group_reduce, group_sum_rows  # K25 on the GPU (few classes)
        if yi.numel():
            sums.copy_(group_sum_rows(yi, x * w[:, None], C))
            cnt.copy_(group_reduce(yi, w, C, "sum", floating=True))
        comm.allreduce_(msg)
        S, n = sums.cpu().numpy(), cnt.cpu().numpy()
        lam = self.getSmoothing()
        N = n.sum()
        sigma = np.zeros((0, 0))
        if mt == "gaussian":
            nz = np.where(n > 0, n, 1.0)
            mean = S / nz[:, None]
            mean_t = torch.as_tensor(mean, device=x.device)
            sq = torch.zeros(C * d, dtype=torch.float64, device=x.device).view(C, d)
            if yi.numel():
                sq.copy_(group_sum_rows(yi, (x - mean_t[yi]) ** 2 * w[:, None], C))
            comm.allreduce_(sq)
            var = sq.cpu().numpy() / nz[:, None]
            # Spark: epsilon = 1e-9 * max variance of any feature over all rows
            gm = S.sum(0) / max(N, 1e-300)
            gvar = (var * n[:, None]).sum(0) / max(N, 1e-300) + \
                (n[:, None] * (mean - gm) ** 2).sum(0) / max(N, 1e-300)
            eps = 1e-9 * float(gvar.max()) if d else 0.0
            pi = np.log(np.where(n > 0, n, 1e-300)) - math.log(N)
            theta, sigma = mean, var + eps
        else:
            pi = np.log(n + lam) - math.log(N + C * lam)
            if mt == "multinomial":
                theta = np.log(S + lam) - np.log(S.sum(1) + d * lam)[:, None]
            else:
                theta = np.log(S + lam) - np.log(n + 2.0 * lam)[:, None]
        m = NaiveBayesModel(pi, theta, sigma)
        self._copyValues(m)
        return m


class NaiveBayesModel(Model):
    _params = NaiveBayes._params

    def __init__(self, pi=None, theta=None, sigma=None):
        super().__init__()
        self._pi = np.asarray(pi if pi is not None else [], dtype=np.float64)
        self._theta = np.atleast_2d(np.asarray(theta if theta is not None else np.zeros((0, 0)), dtype=np.float64))
        self._sigma = np.asarray(sigma if sigma is not None else np.zeros((0, 0)), dtype=np.float64)

    @property
    def pi(self) -> DenseVector:
        return DenseVector(self._pi)

    @property
    def theta(self) -> DenseMatrix:
        return DenseMatrix(*self._theta.shape, self._theta.T.reshape(-1))

    @property
    def sigma(self) -> DenseMatrix:
        return DenseMatrix(*self._sigma.shape, self._sigma.T.reshape(-1))

    @property
    def numClasses(self) -> int:
        return int(self._pi.size)

    @property
    def numFeatures(self) -> int:
        return int(self._theta.shape[1])

    def _raw(self, x: torch.Tensor) -> torch.Tensor:
        x = x.to(torch.float64)
        pi = torch.as_tensor(self._pi, device=x.device)
        th = torch.as_tensor(self._theta, device=x.device)
        mt = self.getModelType().lower()
        if mt == "multinomial":
            return x @ th.T + pi
        if mt == "bernoulli":
            neg = torch.log1p(-torch.exp(th))
            return x @ (th - neg).T + neg.sum(1) + pi
        var = torch.as_tensor(self._sigma, device=x.device)
        ll = -0.5 * (torch.log(2 * math.pi * var).sum(1))[None, :]
        quad = ((x[:, None, :] - th[None]) ** 2 / var[None]).sum(2)
        return ll - 0.5 * quad + pi

    def predict(self, value) -> float:
        r = self._raw(torch.as_tensor(as_array(value), dtype=torch.float64).reshape(1, -1))
        return float(torch.argmax(r[0]))

    def _transform(self, df):
        x = df._feature_matrix(self.getFeaturesCol())
        raw = self._raw(x)
        prob = torch.softmax(raw, 1)
        thr = self.getOrDefault("thresholds") if self.isDefined("thresholds") else None
        if thr:
            t = torch.as_tensor(np.asarray(thr, dtype=np.float64), device=prob.device)
            pred = torch.argmax(prob / t.clamp(min=1e-300), 1).to(torch.float64)
        else:
            pred = torch.argmax(raw, 1).to(torch.float64)
        out = df
        if self.getRawPredictionCol():
            out = _replace_col(out, self.getRawPredictionCol(), ColumnData(raw, None, T.VectorUDT()))
        if self.getProbabilityCol():
            out = _replace_col(out, self.getProbabilityCol(), ColumnData(prob, None, T.VectorUDT()))
        return _replace_col(out, self.getPredictionCol(), ColumnData(pred, None, T.DoubleType()))

    def _save_impl(self, path):
        import pyarrow as pa
        U.write_metadata(self, path)
        U.write_parquet(path, "data", pa.Table.from_pylist(
            [{"pi": U.vector_struct(self._pi), "theta": U.matrix_struct(self._theta),
              "sigma": U.matrix_struct(self._sigma)}],
            schema=pa.schema([("pi", U.vector_arrow_type()), ("theta", U.matrix_arrow_type()),
                              ("sigma", U.matrix_arrow_type())])))

    @classmethod
    def _load_impl(cls, path, md):
        row = U.read_parquet(path, "data").to_pylist()[0]
        m = cls(U.vector_from_struct(row["pi"]), U.matrix_from_struct(row["theta"]),
                U.matrix_from_struct(row["sigma"]))
        U.apply_params(m, md)
        return m
