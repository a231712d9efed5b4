"""More pyspark.ml.regression: AFTSurvivalRegression and IsotonicRegression.

The reference regresses length of stay (ref.py:145-158), a duration; an accelerated-failure-time
model is the MLlib estimator for durations with right-censoring (patients still admitted), and
isotonic regression fits a monotone dose-response curve (e.g. LOS vs occupancy). MI355X-first:

* AFTSurvivalRegression: Weibull AFT negative log-likelihood over the standardized features.
  Each L-BFGS evaluation is two device GEMVs over the HBM-resident shard (margins, then
  Xᵀ·residual) + one all-reduce of the (d+3)-vector; the optimizer runs on the host.
* IsotonicRegression: the (feature, label, weight) triples are gathered once, sorted on the
  device, equal features pooled, and pool-adjacent-violators runs in one host pass (O(n));
  prediction is one device ``searchsorted`` + linear interpolation.
"""
from __future__ import annotations

import math
from typing import List, Optional

import numpy as np
import torch

from ..models.optim import lbfgs
from ..sql import types as T
from ..sql.column import ColumnData
from . import util as U
from .base import Estimator, Model
from .feature import _replace_col
from .linalg import DenseVector, as_array

_Q_DEFAULT = [0.01, 0.05, 0.1, 0.25, 0.5, 0.75, 0.9, 0.95, 0.99]

_AFT_PARAMS = {
    "featuresCol": ("features", "features column name", str),
    "labelCol": ("label", "label column name", str),
    "predictionCol": ("prediction", "prediction column name", str),
    "censorCol": ("censor", "censor column name: 1 = event occurred (uncensored), 0 = censored", str),
    "quantileProbabilities": (_Q_DEFAULT, "quantile probabilities array, values in (0, 1)", None),
    "quantilesCol": (None, "quantiles column name", None),
    "fitIntercept": (True, "whether to fit an intercept term", bool),
    "maxIter": (100, "max number of iterations (>= 0)", int),
    "tol": (1e-6, "convergence tolerance for iterative algorithms (>= 0)", float),
    "aggregationDepth": (2, "suggested depth for treeAggregate (>= 2)", int),
    "maxBlockSizeInMB": (0.0, "maximum memory in MB for stacking input data into blocks", float),
}


class AFTSurvivalRegression(Estimator):
    """Weibull accelerated failure time model: log T = β·x + b + σ·ε with ε extreme-value
    distributed. Minimises the mean negative log-likelihood over θ = (β, b, log σ)
    ℓ = δ·log σ − δ·ε + exp(ε), ε = (log t − β·x − b)/σ, δ = censor (Spark's AFTAggregator)."""
    _params = _AFT_PARAMS

    def __init__(self, **kwargs):
        super().__init__(**kwargs)
        self._defaultParamMap.pop("quantilesCol", None)

    def _fit(self, df):
        from .classification_more import _std
        x = df._feature_matrix(self.getFeaturesCol()).to(torch.float64)
        d = x.shape[1]
        t = df._column_data(self.getLabelCol()).values.to(torch.float64)
        delta = df._column_data(self.getCensorCol()).values.to(torch.float64)
        comm = df._comm
        bad = comm.max_scalar(float((t <= 0).any().item()) if t.numel() else 0.0)
        if bad:
            raise ValueError("AFTSurvivalRegression: labels (survival times) must be positive")
        badc = comm.max_scalar(float(((delta != 0) & (delta != 1)).any().item()) if delta.numel() else 0.0)
        if badc:
            raise ValueError("AFTSurvivalRegression: censor values must be 0 or 1")
        std = _std(df, x)
        sd = np.where(std > 0, std, 1.0)
        active = std > 0
        fi = self.getFitIntercept()
        logt = torch.log(t)
        cnt = torch.tensor([float(t.numel())], dtype=torch.float64, device=x.device)
        comm.allreduce_(cnt)
        N = max(float(cnt.item()), 1.0)
        dev = x.device

        def fg(p):
            beta = np.where(active, p[:d] / sd, 0.0)
            b = p[d] if fi else 0.0
            ls = p[d + 1]
            sigma = math.exp(ls)
            m = x @ torch.as_tensor(beta, device=dev) + b
            eps = (logt - m) / sigma
            ee = torch.exp(eps)
            loss = (delta * ls - delta * eps + ee).sum()
            r = (delta - ee) / sigma  # dℓ/dm
            msg = torch.cat([x.T @ r, r.sum().reshape(1), (delta + (delta - ee) * eps).sum().reshape(1),
                             loss.reshape(1)])
            comm.allreduce_(msg)
            o = msg.cpu().numpy()
            g = np.zeros(d + 2)
            g[:d] = np.where(active, o[:d] / sd, 0.0) / N
            g[d] = o[d] / N if fi else 0.0
            g[d + 1] = o[d + 1] / N
            return float(o[d + 2]) / N, g

        p, hist, iters = lbfgs(fg, np.zeros(d + 2), self.getMaxIter(), self.getTol())
        model = AFTSurvivalRegressionModel(np.where(active, p[:d] / sd, 0.0), float(p[d]) if fi else 0.0,
                                           math.exp(p[d + 1]))
        self._copyValues(model)
        return model


class AFTSurvivalRegressionModel(Model):
    _params = _AFT_PARAMS

    def __init__(self, coefficients=None, intercept: float = 0.0, scale: float = 1.0):
        super().__init__()
        self._coef = np.asarray(coefficients if coefficients is not None else [], dtype=np.float64)
        self._icpt, self._scale = float(intercept), float(scale)

    @property
    def coefficients(self) -> DenseVector:
        return DenseVector(self._coef)

    @property
    def intercept(self) -> float:
        return self._icpt

    @property
    def scale(self) -> float:
        return self._scale

    @property
    def numFeatures(self) -> int:
        return int(self._coef.size)

    def _lam(self, x: torch.Tensor) -> torch.Tensor:
        return torch.exp(x.to(torch.float64) @ torch.as_tensor(self._coef, device=x.device) + self._icpt)

    def _qfac(self) -> np.ndarray:
        q = np.asarray(self.getQuantileProbabilities(), dtype=np.float64)
        return np.exp(np.log(-np.log1p(-q)) * self._scale)

    def _transform(self, df):
        lam = self._lam(df._feature_matrix(self.getFeaturesCol()))
        out = _replace_col(df, self.getPredictionCol(), ColumnData(lam, None, T.DoubleType()))
        if self.isSet("quantilesCol") and self.getOrDefault("quantilesCol"):
            qf = torch.as_tensor(self._qfac(), device=lam.device)
            out = _replace_col(out, self.getOrDefault("quantilesCol"),
                               ColumnData((lam[:, None] * qf[None, :]).contiguous(), None, T.VectorUDT()))
        return out

    def predict(self, features) -> float:
        return float(math.exp(np.asarray(as_array(features), dtype=np.float64) @ self._coef + self._icpt))

    def predictQuantiles(self, features) -> DenseVector:
        return DenseVector(self.predict(features) * self._qfac())

    def _save_impl(self, path):
        import pyarrow as pa
        U.write_metadata(self, path)
        U.write_parquet(path, "data", pa.Table.from_pylist(
            [{"coefficients": U.vector_struct(self._coef), "intercept": self._icpt, "scale": self._scale}],
            schema=pa.schema([("coefficients", U.vector_arrow_type()), pa.field("intercept", pa.float64(), False),
                              pa.field("scale", pa.float64(), False)])))

    @classmethod
    def _load_impl(cls, path, md):
        r = U.read_parquet(path, "data").to_pylist()[0]
        m = cls(U.vector_from_struct(r["coefficients"]), r["intercept"], r["scale"])
        U.apply_params(m, md)
        return m


# --------------------------------------------------------------------------------- IsotonicRegression

_ISO_PARAMS = {
    "featuresCol": ("features", "features column name", str),
    "labelCol": ("label", "label column name", str),
    "predictionCol": ("prediction", "prediction column name", str),
    "weightCol": (None, "weight column name", None),
    "isotonic": (True, "whether the output sequence should be isotonic/increasing (true) or "
                       "antitonic/decreasing (false)", bool),
    "featureIndex": (0, "index of the feature if featuresCol is a vector column, no effect otherwise", int),
}


def _feature_values(df, col: str, idx: int) -> torch.Tensor:
    cd = df._column_data(col)
    v = cd.values.to(torch.float64)
    return v[:, idx].contiguous() if v.dim() == 2 else v


def pava(x: np.ndarray, y: np.ndarray, w: np.ndarray):
    """Pool-adjacent-violators on points sorted by x with equal x already pooled; returns the
    compressed (boundaries, predictions): the first and last x of every constant block."""
    # blocks as a stack of (y_mean, weight, start, end)
    ys, ws, st, en = [], [], [], []
    for i in range(x.size):
        ys.append(y[i])
        ws.append(w[i])
        st.append(i)
        en.append(i)
        while len(ys) > 1 and ys[-2] >= ys[-1]:
            wt = ws[-2] + ws[-1]
            ym = (ys[-2] * ws[-2] + ys[-1] * ws[-1]) / wt
            ys[-2:] = [ym]
            ws[-2:] = [wt]
            en[-2:] = [en[-1]]
            st.pop()
    bnd, pred = [], []
    for yv, a, b in zip(ys, st, en):
        bnd.append(x[a])
        pred.append(yv)
        if b != a:
            bnd.append(x[b])
            pred.append(yv)
    return np.asarray(bnd, dtype=np.float64), np.asarray(pred, dtype=np.float64)


class IsotonicRegression(Estimator):
    """Weighted isotonic (or antitonic) least-squares fit of the label against one feature.
    Points with equal feature values are pooled (weighted mean label) before PAV, as Spark 3 does;
    zero-weight points are dropped."""
    _params = _ISO_PARAMS

    def __init__(self, **kwargs):
        super().__init__(**kwargs)
        self._defaultParamMap.pop("weightCol", None)

    def _fit(self, df):
        x = _feature_values(df, self.getFeaturesCol(), self.getFeatureIndex())
        y = df._column_data(self.getLabelCol()).values.to(torch.float64)
        w = df._column_data(self.getOrDefault("weightCol")).values.to(torch.float64) \
            if self.isSet("weightCol") and self.getOrDefault("weightCol") else torch.ones_like(y)
        comm = df._comm
        trip = comm.allgather_cat(torch.stack([x, y, w], 1).contiguous())
        trip = trip[trip[:, 2] > 0]
        if trip.shape[0] == 0:
            raise ValueError("IsotonicRegression: no rows with positive weight")
        if bool((trip[:, 2] < 0).any()):
            raise ValueError("IsotonicRegression: negative weight")
        sign = 1.0 if self.getIsotonic() else -1.0
        xs, order = torch.sort(trip[:, 0], stable=True)
        ys, ws = trip[order, 1] * sign, trip[order, 2]
        ux, inv = torch.unique_consecutive(xs, return_inverse=True)
        wsum = torch.zeros(ux.numel(), dtype=torch.float64, device=xs.device).index_add_(0, inv, ws)
        ysum = torch.zeros_like(wsum).index_add_(0, inv, ys * ws)
        bnd, pred = pava(ux.cpu().numpy(), (ysum / wsum).cpu().numpy(), wsum.cpu().numpy())
        model = IsotonicRegressionModel(bnd, pred * sign)
        self._copyValues(model)
        return model


class IsotonicRegressionModel(Model):
    _params = _ISO_PARAMS

    def __init__(self, boundaries=None, predictions=None):
        super().__init__()
        self._b = np.asarray(boundaries if boundaries is not None else [], dtype=np.float64)
        self._p = np.asarray(predictions if predictions is not None else [], dtype=np.float64)

    @property
    def boundaries(self) -> DenseVector:
        return DenseVector(self._b)

    @property
    def predictions(self) -> DenseVector:
        return DenseVector(self._p)

    @property
    def numFeatures(self) -> int:
        return 1

    def _predict_t(self, v: torch.Tensor) -> torch.Tensor:
        b = torch.as_tensor(self._b, device=v.device)
        p = torch.as_tensor(self._p, device=v.device)
        n = b.numel()
        if n == 1:
            return torch.full_like(v, float(p[0]))
        i = torch.searchsorted(b, v.contiguous(), right=True).clamp(1, n - 1)  # b[i-1] <= v < b[i]
        lo, hi = b[i - 1], b[i]
        frac = torch.where(hi > lo, (v - lo) / (hi - lo), torch.zeros_like(v))
        out = p[i - 1] + frac * (p[i] - p[i - 1])
        out = torch.where(v <= b[0], p[0], out)
        out = torch.where(v >= b[-1], p[-1], out)
        return torch.where(v == b[i - 1], p[i - 1], out)

    def _transform(self, df):
        v = _feature_values(df, self.getFeaturesCol(), self.getFeatureIndex())
        return _replace_col(df, self.getPredictionCol(), ColumnData(self._predict_t(v), None, T.DoubleType()))

    def predict(self, value) -> float:
        return float(self._predict_t(torch.tensor([float(value)], dtype=torch.float64))[0])

    def _save_impl(self, path):
        import pyarrow as pa
        U.write_metadata(self, path)
        U.write_parquet(path, "data", pa.Table.from_pylist(
            [{"boundaries": self._b.tolist(), "predictions": self._p.tolist(), "isotonic": bool(self.getIsotonic())}],
            schema=pa.schema([("boundaries", pa.list_(pa.float64())), ("predictions", pa.list_(pa.float64())),
                              pa.field("isotonic", pa.bool_(), False)])))

    @classmethod
    def _load_impl(cls, path, md):
        r = U.read_parquet(path, "data").to_pylist()[0]
        m = cls(r["boundaries"], r["predictions"])
        U.apply_params(m, md)
        return m


__all__: List[str] = ["AFTSurvivalRegression", "AFTSurvivalRegressionModel", "IsotonicRegression",
                      "IsotonicRegressionModel", "pava"]
