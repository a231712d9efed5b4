"""GeneralizedLinearRegression (Spark ``org.apache.spark.ml.regression.GeneralizedLinearRegression``).

Beyond the reference's OLS (ref.py:145-148): length of stay is positive and skewed
(gamma / log link) and admission counts are counts (poisson / log), so this is the
model family a user of the reference's LOS regression reaches for next.

Fit = iteratively reweighted least squares, Spark's algorithm (IRLS with absolute
coefficient change < tol, maxIter 25).  Every IRLS step is ONE pass of the K15 Gram
kernel over the device-resident rows: ``[X 1 z]ᵀ W [X 1 z]`` accumulated in float64
with the working response z and working weights W computed elementwise on the
device, one all-reduce of (d+2)² doubles, then a (d+1)×(d+1) solve on the host.
regParam is Spark's L2 penalty on standardized coefficients (WeightedLeastSquares
with standardizeFeatures = true).
"""
from __future__ import annotations

import numpy as np
import torch

from ..ops import glm_ops
from ..sql import types as T
from ..sql.column import ColumnData
from . import util as U
from .base import Estimator, Model
from .feature import _replace_col
from .linalg import DenseVector, as_array

_DEFAULT_LINK = {"gaussian": "identity", "binomial": "logit", "poisson": "log", "gamma": "inverse"}
_LINKS = ("identity", "log", "logit", "inverse", "sqrt")


def _link(name, mu):
    if name == "identity":
        return mu
    if name == "log":
        return torch.log(mu)
    if name == "logit":
        return torch.log(mu / (1.0 - mu))
    if name == "inverse":
        return 1.0 / mu
    return torch.sqrt(mu)


def _unlink(name, eta):
    if name == "identity":
        return eta
    if name == "log":
        return torch.exp(eta)
    if name == "logit":
        return torch.sigmoid(eta)
    if name == "inverse":
        return 1.0 / eta
    return eta * eta


def _deriv(name, mu):
    if name == "identity":
        return torch.ones_like(mu)
    if name == "log":
        return 1.0 / mu
    if name == "logit":
        return 1.0 / (mu * (1.0 - mu))
    if name == "inverse":
        return -1.0 / (mu * mu)
    return 0.5 / torch.sqrt(mu)


def _variance(family, mu):
    if family == "gaussian":
        return torch.ones_like(mu)
    if family == "binomial":
        return mu * (1.0 - mu)
    if family == "poisson":
        return mu
    return mu * mu


def _project(family, mu):
    eps = 1e-16
    if family == "binomial":
        return mu.clamp(eps, 1.0 - eps)
    if family in ("poisson", "gamma"):
        return mu.clamp(min=eps)
    return mu


def _init_mu(family, y, w):
    if family == "binomial":
        return (w * y + 0.5) / (w + 1.0)
    if family == "poisson":
        return y.clamp(min=0.1)
    return y.clone()


def _unit_deviance(family, y, mu):
    if family == "gaussian":
        return (y - mu) ** 2
    if family == "binomial":
        def ylogy(a, b):
            return torch.where(a > 0, a * torch.log(a / b), torch.zeros_like(a))
        return 2.0 * (ylogy(y, mu) + ylogy(1.0 - y, 1.0 - mu))
    if family == "poisson":
        return 2.0 * (torch.where(y > 0, y * torch.log(y / mu), torch.zeros_like(y)) - (y - mu))
    return 2.0 * (-torch.log(y / mu) + (y - mu) / mu)


def _check_labels(family, y):
    if family == "binomial" and bool(((y < 0) | (y > 1)).any()):
        raise ValueError("binomial family needs labels in [0, 1]")
    if family == "poisson" and bool((y < 0).any()):
        raise ValueError("poisson family needs non-negative labels")
    if family == "gamma" and bool((y <= 0).any()):
        raise ValueError("gamma family needs positive labels")


def _wls(G: np.ndarray, d: int, reg: float, fit_intercept: bool):
    """Weighted least squares from the Gram of [X 1 z] (weights folded in), L2 on standardized
    coefficients."""
    W = G[d, d]
    mx = G[:d, d] / W
    mz = G[d, d + 1] / W
    if fit_intercept:
        A = G[:d, :d] / W - np.outer(mx, mx)
        b = G[:d, d + 1] / W - mx * mz
    else:
        A = G[:d, :d] / W
        b = G[:d, d + 1] / W
    var_x = np.maximum(np.diag(G[:d, :d]) / W - mx * mx, 0.0)
    A = A + reg * np.diag(var_x)
    beta = np.linalg.lstsq(A, b, rcond=None)[0] if np.linalg.matrix_rank(A) < d else np.linalg.solve(A, b)
    b0 = (mz - mx @ beta) if fit_intercept else 0.0
    return beta, float(b0)


class GeneralizedLinearRegression(Estimator):
    _params = {
        "featuresCol": ("features", "features column name", str),
        "labelCol": ("label", "label column name", str),
        "predictionCol": ("prediction", "prediction column name", str),
        "family": ("gaussian", "gaussian | binomial | poisson | gamma", str),
        "link": (None, "identity | log | logit | inverse | sqrt (default: the family's canonical link)", None),
        "linkPredictionCol": (None, "link prediction (linear predictor) column name", None),
        "fitIntercept": (True, "whether to fit an intercept term", bool),
        "maxIter": (25, "maximum number of IRLS iterations (>= 0)", int),
        "tol": (1e-6, "convergence tolerance of the IRLS iterations", float),
        "regParam": (0.0, "L2 regularization parameter (>= 0)", float),
        "weightCol": (None, "weight column name", None),
        "solver": ("irls", "the solver algorithm for optimization (irls)", str),
    }

    def _fit(self, df):
        family = self.getFamily().lower()
        if family not in _DEFAULT_LINK:
            raise ValueError(f"unsupported family {family!r}")
        link = (self.getOrDefault("link") if self.isSet("link") else None) or _DEFAULT_LINK[family]
        if link not in _LINKS:
            raise ValueError(f"unsupported link {link!r}")
        x = df._feature_matrix(self.getFeaturesCol())
        d = x.shape[1]
        y = df._column_data(self.getLabelCol()).values.to(torch.float64)
        w = df._column_data(self.getOrDefault("weightCol")).values.to(torch.float64) \
            if self.isSet("weightCol") else torch.ones_like(y)
        _check_labels(family, y)
        comm = df._comm
        fi = self.getFitIntercept()
        reg = self.getRegParam()
        def eta_of(beta, b0):  # K24 linear predictor (reads X in its stored dtype)
            return glm_ops.linear_predict(x, d, torch.as_tensor(np.r_[beta, b0], dtype=torch.float64))
        it = 0
        if family == "gaussian" and link == "identity":
            G = glm_ops.gram(x, d, y, w)
            comm.allreduce_(G)
            beta, b0 = _wls(G.cpu().numpy(), d, reg, fi)
            it = 1
        else:
            mu = _init_mu(family, y, w)
            eta = _link(link, mu)
            beta, b0 = np.zeros(d), 0.0
            for it in range(1, self.getMaxIter() + 1):
                dmu = _deriv(link, mu)
                z = eta + (y - mu) * dmu
                wt = w / (dmu * dmu * _variance(family, mu))
                G = glm_ops.gram(x, d, z, wt)
                comm.allreduce_(G)
                nb, n0 = _wls(G.cpu().numpy(), d, reg, fi)
                delta = max(float(np.max(np.abs(nb - beta))) if d else 0.0, abs(n0 - b0))
                beta, b0 = nb, n0
                eta = eta_of(beta, b0)
                mu = _project(family, _unlink(link, eta))
                if delta < self.getTol():
                    break
        m = GeneralizedLinearRegressionModel(beta, b0)
        self._copyValues(m)
        m._fam, m._lnk, m._iters = family, link, it
        # training summary: deviance / null deviance / dispersion (one fused pass + all-reduce)
        mu = _project(family, _unlink(link, eta_of(beta, b0)))
        wy = (w * y).sum()
        msg = torch.stack([(w * _unit_deviance(family, y, mu)).sum(), wy, w.sum(),
                           torch.tensor(float(y.numel()), dtype=torch.float64, device=y.device)])
        comm.allreduce_(msg)
        dev, swy, sw, n = (float(v) for v in msg.cpu())
        ybar = swy / max(sw, 1e-300) if fi else None
        mu0 = torch.full_like(y, ybar) if fi else _project(family, _unlink(link, torch.zeros_like(y)))
        nd = torch.stack([(w * _unit_deviance(family, y, _project(family, mu0))).sum()])
        comm.allreduce_(nd)
        rank = d + (1 if fi else 0)
        dof = n - rank
        disp = 1.0 if family in ("binomial", "poisson") else None
        if disp is None:
            r = (w * (y - mu) ** 2 / _variance(family, mu)).sum().reshape(1)
            comm.allreduce_(r)
            disp = float(r[0]) / max(dof, 1.0)
        m._summary = GeneralizedLinearRegressionTrainingSummary(it, dev, float(nd[0]), disp, dof, n - (1 if fi else 0))
        return m


class GeneralizedLinearRegressionTrainingSummary:
    def __init__(self, num_iterations, deviance, null_deviance, dispersion, dof, null_dof):
        self.numIterations = num_iterations
        self.deviance = deviance
        self.nullDeviance = null_deviance
        self.dispersion = dispersion
        self.residualDegreeOfFreedom = int(dof)
        self.residualDegreeOfFreedomNull = int(null_dof)
        self.solver = "irls"


class GeneralizedLinearRegressionModel(Model):
    _params = GeneralizedLinearRegression._params

    def __init__(self, coefficients=None, intercept: float = 0.0):
        super().__init__()
        self._coef = np.asarray(coefficients if coefficients is not None else [], dtype=np.float64)
        self._b0 = float(intercept)
        self._fam = None
        self._lnk = None
        self._iters = 0
        self._summary = None

    @property
    def coefficients(self) -> DenseVector:
        return DenseVector(self._coef)

    @property
    def intercept(self) -> float:
        return self._b0

    @property
    def numFeatures(self) -> int:
        return int(self._coef.size)

    @property
    def hasSummary(self) -> bool:
        return self._summary is not None

    @property
    def summary(self) -> GeneralizedLinearRegressionTrainingSummary:
        if self._summary is None:
            raise RuntimeError("No training summary available for this GeneralizedLinearRegressionModel")
        return self._summary

    def _family_link(self):
        fam = self._fam or self.getFamily().lower()
        lnk = self._lnk or (self.getOrDefault("link") if self.isSet("link") else None) or _DEFAULT_LINK[fam]
        return fam, lnk

    def predict(self, value) -> float:
        fam, lnk = self._family_link()
        eta = float(np.dot(as_array(value), self._coef)) + self._b0
        return float(_unlink(lnk, torch.tensor(eta, dtype=torch.float64)))

    def _transform(self, df):
        x = df._feature_matrix(self.getFeaturesCol())
        fam, lnk = self._family_link()
        eta = glm_ops.linear_predict(x, x.shape[1], torch.as_tensor(np.r_[self._coef, self._b0]))
        out = df
        if self.isSet("linkPredictionCol") and self.getOrDefault("linkPredictionCol"):
            out = _replace_col(out, self.getOrDefault("linkPredictionCol"), ColumnData(eta, None, T.DoubleType()))
        return _replace_col(out, self.getPredictionCol(), ColumnData(_unlink(lnk, eta).contiguous(), None,
                                                                     T.DoubleType()))

    def _save_impl(self, path):
        import pyarrow as pa
        U.write_metadata(self, path)
        U.write_parquet(path, "data", pa.Table.from_pylist(
            [{"intercept": self._b0, "coefficients": U.vector_struct(self._coef)}],
            schema=pa.schema([pa.field("intercept", pa.float64(), nullable=False),
                              ("coefficients", U.vector_arrow_type())])))

    @classmethod
    def _load_impl(cls, path, md):
        row = U.read_parquet(path, "data").to_pylist()[0]
        m = cls(U.vector_from_struct(row["coefficients"]), row["intercept"])
        U.apply_params(m, md)
        return m

