"""GaussianMixture (pyspark.ml.clustering): soft clustering of hospital feature vectors.

KMeans (the [NS] flagship) gives hard hospital-regime assignments; a Gaussian mixture gives
per-regime covariances and membership probabilities. Design, MI355X-first: one EM iteration is,
per component, a triangular solve of the shard against the component's Cholesky factor (device
TRSM), a log-sum-exp over components for the responsibilities, and the weighted moments
R_kᵀ·X and (R_k ∘ X)ᵀ·X as device GEMMs (hipBLASLt) — all k·(1 + d + d²) sufficient statistics
plus the log-likelihood go into ONE all-reduce per iteration. The M-step (k small d×d matrices)
runs on the host in float64.

Spark semantics: k=2, maxIter=100, tol=0.01 (stop when the log-likelihood improves by less than
tol), init = means of k disjoint groups of ``nSamples`` = 5 rows sampled with replacement from the
data (seeded) and the diagonal of the data variance as every initial covariance, uniform weights.
"""
from __future__ import annotations

import math
from typing import List, Optional

import numpy as np
import torch

from ..sql import types as T
from ..sql.column import ColumnData
from . import util as U
from .base import Estimator, Model
from .feature import _replace_col
from .linalg import DenseMatrix, DenseVector

_GMM_PARAMS = {
    "featuresCol": ("features", "features column name", str),
    "predictionCol": ("prediction", "prediction column name", str),
    "probabilityCol": ("probability", "column name for predicted class conditional probabilities", str),
    "k": (2, "number of independent Gaussians in the mixture model (> 1)", int),
    "maxIter": (100, "max number of iterations (>= 0)", int),
    "seed": (None, "random seed", None),
    "tol": (0.01, "convergence tolerance for iterative algorithms (>= 0)", float),
    "aggregationDepth": (2, "suggested depth for treeAggregate (>= 2)", int),
    "weightCol": (None, "weight column name", None),
}

_LOG2PI = math.log(2.0 * math.pi)


def _chol(cov: np.ndarray) -> np.ndarray:
    """Cholesky factor, with a growing ridge for (near-)singular covariances."""
    d = cov.shape[0]
    ridge = 0.0
    scale = max(float(np.trace(cov)) / max(d, 1), 1e-300)
    for _ in range(12):
        try:
            return np.linalg.cholesky(cov + ridge * np.eye(d))
        except np.linalg.LinAlgError:
            ridge = scale * 1e-10 if ridge == 0.0 else ridge * 10.0
    raise np.linalg.LinAlgError("GaussianMixture: covariance is not positive definite")


def _log_pdf(x: torch.Tensor, mus: np.ndarray, covs: np.ndarray) -> torch.Tensor:
    """[n, k] log N(x | mu_j, Sigma_j) via device triangular solves."""
    n, d = x.shape
    out = torch.empty((n, len(mus)), dtype=torch.float64, device=x.device)
    for j, (mu, cov) in enumerate(zip(mus, covs)):
        L = _chol(cov)
        Lt = torch.as_tensor(L, device=x.device)
        z = torch.linalg.solve_triangular(Lt, (x - torch.as_tensor(mu, device=x.device)).T, upper=False)
        logdet = 2.0 * float(np.log(np.diag(L)).sum())
        out[:, j] = -0.5 * (d * _LOG2PI + logdet + (z * z).sum(0))
    return out


class GaussianMixture(Estimator):
    _params = _GMM_PARAMS

    def __init__(self, **kwargs):
        super().__init__(**kwargs)
        for k in ("seed", "weightCol"):
            self._defaultParamMap.pop(k, None)

    def _init(self, df, x: torch.Tensor, w: torch.Tensor, k: int, seed: int):
        comm = df._comm
        d = x.shape[1]
        n_samples = 5
        counts = comm.allgather_object(int(x.shape[0]))
        total = sum(counts)
        if total < k:
            raise ValueError(f"GaussianMixture: {total} rows < k = {k}")
        rng = np.random.default_rng(seed & 0xFFFFFFFF)
        picks = rng.integers(0, total, size=k * n_samples)  # global row ids, drawn order kept
        off = sum(counts[:comm.rank])
        pos = np.nonzero((picks >= off) & (picks < off + x.shape[0]))[0]
        rows = x[torch.as_tensor(picks[pos] - off, dtype=torch.int64, device=x.device)].cpu().numpy()
        samp = np.zeros((k * n_samples, d))
        for p_, r_ in comm.allgather_object((pos, rows)):
            samp[p_] = r_
        mus = samp.reshape(k, n_samples, d).mean(1)
        # diagonal of the (weighted) data variance
        W = w.sum()
        s1 = (w[:, None] * x).sum(0)
        s2 = (w[:, None] * x * x).sum(0)
        msg = torch.cat([W.reshape(1), s1, s2])
        comm.allreduce_(msg)
        o = msg.cpu().numpy()
        mean = o[1:1 + d] / o[0]
        var = np.clip(o[1 + d:] / o[0] - mean * mean, 1e-12, None)
        covs = np.stack([np.diag(var)] * k)
        return np.full(k, 1.0 / k), mus, covs

    def _fit(self, df):
        from .tree_models import _default_seed
        x = df._feature_matrix(self.getFeaturesCol()).to(torch.float64)
        n, d = x.shape
        k = self.getK()
        if k < 2:
            raise ValueError("GaussianMixture: k must be > 1")
        w = df._column_data(self.getOrDefault("weightCol")).values.to(torch.float64) \
            if self.isSet("weightCol") and self.getOrDefault("weightCol") else torch.ones(n, dtype=torch.float64,
                                                                                         device=x.device)
        seed = int(self.getOrDefault("seed")) if self.isSet("seed") else _default_seed(U.jvm_class(self))
        comm = df._comm
        weights, mus, covs = self._init(df, x, w, k, seed)
        ll_prev, ll = -np.inf, -np.inf
        it = 0
        for it in range(1, self.getMaxIter() + 1):
            lp = _log_pdf(x, mus, covs) + torch.as_tensor(np.log(np.clip(weights, 1e-300, None)), device=x.device)
            lse = torch.logsumexp(lp, 1)
            R = torch.exp(lp - lse[:, None]) * w[:, None]  # weighted responsibilities [n, k]
            S0 = R.sum(0)
            S1 = R.T @ x
            S2 = torch.stack([(R[:, j:j + 1] * x).T @ x for j in range(k)])
            msg = torch.cat([S0, S1.reshape(-1), S2.reshape(-1), (w * lse).sum().reshape(1), w.sum().reshape(1)])
            comm.allreduce_(msg)
            o = msg.cpu().numpy()
            s0 = o[:k]
            s1 = o[k:k + k * d].reshape(k, d)
            s2 = o[k + k * d:k + k * d + k * d * d].reshape(k, d, d)
            ll, wt = float(o[-2]), float(o[-1])
            s0c = np.clip(s0, 1e-300, None)
            mus = s1 / s0c[:, None]
            covs = s2 / s0c[:, None, None] - np.einsum("ki,kj->kij", mus, mus)
            covs = 0.5 * (covs + np.transpose(covs, (0, 2, 1)))
            weights = s0 / wt
            if abs(ll - ll_prev) < self.getTol():
                break
            ll_prev = ll
        model = GaussianMixtureModel(weights, mus, covs)
        self._copyValues(model)
        model._attach_summary(GaussianMixtureSummary(model, df, ll, it))
        return model


class GaussianMixtureModel(Model):
    _params = _GMM_PARAMS

    def __init__(self, weights=None, mus=None, covs=None):
        super().__init__()
        self._w = np.asarray(weights if weights is not None else [], dtype=np.float64)
        self._mu = np.asarray(mus if mus is not None else np.zeros((0, 0)), dtype=np.float64)
        self._cov = np.asarray(covs if covs is not None else np.zeros((0, 0, 0)), dtype=np.float64)
        self._summary = None

    @property
    def weights(self) -> List[float]:
        return self._w.tolist()

    @property
    def gaussians(self):
        return [(DenseVector(m), DenseMatrix(c.shape[0], c.shape[1], c.T.reshape(-1))) for m, c in
                zip(self._mu, self._cov)]

    @property
    def gaussiansDF(self):
        from ..sql.builder import rows_round_robin
        schema = T.StructType([T.StructField("mean", T.VectorUDT(), False), T.StructField("cov", T.MatrixUDT(), False)])
        sess = self._session()
        return rows_round_robin(sess, schema, [[m, c] for m, c in self.gaussians])

    @staticmethod
    def _session():
        from ..sql.session import SparkSession
        return SparkSession.builder.getOrCreate()

    def _probs(self, x: torch.Tensor) -> torch.Tensor:
        lp = _log_pdf(x.to(torch.float64), self._mu, self._cov) + torch.as_tensor(
            np.log(np.clip(self._w, 1e-300, None)), device=x.device)
        return torch.softmax(lp, 1)

    def _transform(self, df):
        p = self._probs(df._feature_matrix(self.getFeaturesCol()))
        out = df
        if self.getProbabilityCol():
            out = _replace_col(out, self.getProbabilityCol(), ColumnData(p.contiguous(), None, T.VectorUDT()))
        return _replace_col(out, self.getPredictionCol(),
                            ColumnData(torch.argmax(p, 1).to(torch.int32), None, T.IntegerType()))

    def predict(self, value) -> int:
        from .linalg import as_array
        return int(torch.argmax(self._probs(torch.as_tensor(as_array(value), dtype=torch.float64)[None, :]), 1)[0])

    def predictProbability(self, value) -> DenseVector:
        from .linalg import as_array
        return DenseVector(self._probs(torch.as_tensor(as_array(value), dtype=torch.float64)[None, :])[0].numpy())

    def _save_impl(self, path):
        import pyarrow as pa
        U.write_metadata(self, path)
        U.write_parquet(path, "data", pa.Table.from_pylist(
            [{"weights": self._w.tolist(), "mus": [U.vector_struct(m) for m in self._mu],
              "sigmas": [U.matrix_struct(c) for c in self._cov]}],
            schema=pa.schema([("weights", pa.list_(pa.float64())), ("mus", pa.list_(U.vector_arrow_type())),
                              ("sigmas", pa.list_(U.matrix_arrow_type()))])))

    @classmethod
    def _load_impl(cls, path, md):
        r = U.read_parquet(path, "data").to_pylist()[0]
        m = cls(r["weights"], np.stack([U.vector_from_struct(v) for v in r["mus"]]),
                np.stack([U.matrix_from_struct(s) for s in r["sigmas"]]))
        U.apply_params(m, md)
        return m


class GaussianMixtureSummary:
    def __init__(self, model, df, ll, iters):
        self._model, self._df = model, df
        self.logLikelihood = float(ll)
        self.numIter = int(iters)
        self.k = len(model._w)
        self.featuresCol = model.getFeaturesCol()
        self.predictionCol = model.getPredictionCol()
        self.probabilityCol = model.getProbabilityCol()
        self._pred = None

    @property
    def predictions(self):
        if self._pred is None:
            self._pred = self._model.transform(self._df)
        return self._pred

    @property
    def cluster(self):
        return self.predictions.select(self.predictionCol)

    @property
    def probability(self):
        return self.predictions.select(self.probabilityCol)

    @property
    def clusterSizes(self) -> List[int]:
        pred = self.predictions._column_data(self.predictionCol).values.to(torch.int64)
        c = torch.bincount(pred, minlength=self.k).to(torch.float64)
        self._df._comm.allreduce_(c)
        return [int(v) for v in c.cpu().tolist()]


__all__ = ["GaussianMixture", "GaussianMixtureModel", "GaussianMixtureSummary"]
