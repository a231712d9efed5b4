"""Latent Dirichlet allocation (pyspark.ml.clustering.LDA / LocalLDAModel) with the online
variational Bayes optimizer (Hoffman, Blei & Bach 2010 — Spark's default ``optimizer="online"``),
e.g. "topics" of admission-reason term counts per hospital ward.

Device design: the E-step runs on a whole mini-batch of documents at once — the [B, V] count
matrix against expElogbeta [k, V] is two GEMMs per fixed-point sweep (phinorm = θ·β and
γ = α + θ ⊙ ((X / phinorm)·βᵀ)), with a per-document convergence mask so every document stops
exactly when Spark's per-document loop would (mean |Δγ| <= 1e-3). The sufficient statistics θᵀ·(X /
phinorm) are one more GEMM and are all-reduced across ranks with the log-p̂ terms and the
document count in one message; λ and α updates (Spark's ``updateLambda`` / Newton ``updateAlpha``)
are tiny and run identically on every rank.

Randomness is counter-based (``utils.rng``: a hash of (seed, row id)) for the mini-batch
Bernoulli draw and the per-document Gamma(100, 1/100) initial γ, so a fit is the same on any
number of ranks; λ's Gamma(100, 1/100) init comes from a seeded generator shared by all ranks.
Spark's Breeze random streams cannot be reproduced, so fitted topics are "parity unpinned" and the
tests check the model's defining properties instead (tests/test_lda_pic.py).
"""
from __future__ import annotations

import math
from typing import List, Optional

import numpy as np
import torch

from ..sql import types as T
from ..sql.column import ColumnData
from ..utils import rng as R
from . import util as U
from .base import Estimator, Model
from .colutil import _replace_col
from .linalg import DenseMatrix, DenseVector
from .param import NO_DEFAULT

GAMMA_SHAPE = 100.0
_E_TOL = 1e-3
_E_MAX_SWEEPS = 1000
_CHUNK = 8192

_LDA_PARAMS = {
    "featuresCol": ("features", "features column name", str),
    "maxIter": (20, "max number of iterations (>= 0)", int),
    "seed": (None, "random seed", None),
    "checkpointInterval": (10, "set checkpoint interval (>= 1) or disable checkpoint (-1)", int),
    "k": (10, "The number of topics (clusters) to infer. Must be > 1.", int),
    "optimizer": ("online", "Optimizer or inference algorithm used to estimate the LDA model. Supported: online",
                  str),
    "learningOffset": (1024.0, "A (positive) learning parameter that downweights early iterations.", float),
    "learningDecay": (0.51, "Learning rate, set as an exponential decay rate, in (0.5, 1.0].", float),
    "subsamplingRate": (0.05, "Fraction of the corpus to be sampled and used in each iteration of "
                              "mini-batch gradient descent, in range (0, 1].", float),
    "optimizeDocConcentration": (True, "Indicates whether the docConcentration (Dirichlet parameter for "
                                       "document-topic distribution) will be optimized during training.", bool),
    "docConcentration": (None, "Concentration parameter (commonly named \"alpha\") for the prior placed on "
                               "documents' distributions over topics (\"theta\").", "listfloat"),
    "topicConcentration": (None, "Concentration parameter (commonly named \"beta\" or \"eta\") for the prior "
                                 "placed on topic' distributions over terms.", float),
    "topicDistributionCol": ("topicDistribution", "Output column with estimates of the topic mixture "
                                                  "distribution for each document.", str),
    "keepLastCheckpoint": (True, "(For EM optimizer) If using checkpointing, this indicates whether to keep "
                                 "the last checkpoint.", bool),
}


def dirichlet_expectation(a: torch.Tensor) -> torch.Tensor:
    """E[log p] under Dirichlet(a), row-wise: ψ(a) − ψ(Σ a)."""
    return torch.special.digamma(a) - torch.special.digamma(a.sum(-1, keepdim=True))


def _gamma_init(row_ids: torch.Tensor, k: int, seed: int) -> torch.Tensor:
    """Gamma(100, 1/100) draws per (document, topic) from counter-based normals (Wilson–Hilferty
    cube transform; at shape 100 it is accurate to well below the E-step tolerance)."""
    cols = []
    for j in range(k):
        u1 = R.uniform(row_ids, seed, 2 * j + 1).clamp(min=1e-300)
        u2 = R.uniform(row_ids, seed, 2 * j + 2)
        z = torch.sqrt(-2.0 * torch.log(u1)) * torch.cos(2.0 * math.pi * u2)
        c = 1.0 / (9.0 * GAMMA_SHAPE)
        cols.append(torch.clamp(1.0 - c + z * math.sqrt(c), min=1e-3) ** 3)
    return torch.stack(cols, 1).to(torch.float64)


def e_step(X: torch.Tensor, exp_elog_beta: torch.Tensor, alpha: torch.Tensor, gamma0: torch.Tensor):
    """Batched variational E-step: (γ [B, k], sstats [k, V], θ-expectations [B, k], phinorm [B, V]).
    A document stops updating once its mean |Δγ| <= 1e-3, exactly like Spark's per-document loop."""
    gamma = gamma0.clone()
    e_theta = torch.exp(dirichlet_expectation(gamma))
    phinorm = e_theta @ exp_elog_beta + 1e-100
    active = torch.ones(X.shape[0], dtype=torch.bool, device=X.device)
    for _ in range(_E_MAX_SWEEPS):
        new_gamma = e_theta * ((X / phinorm) @ exp_elog_beta.T) + alpha[None, :]
        change = (new_gamma - gamma).abs().mean(1)
        gamma = torch.where(active[:, None], new_gamma, gamma)
        e_theta = torch.where(active[:, None], torch.exp(dirichlet_expectation(gamma)), e_theta)
        phinorm = e_theta @ exp_elog_beta + 1e-100
        active = active & (change > _E_TOL)
        if not bool(active.any()):
            break
    sstats = e_theta.T @ (X / phinorm)
    return gamma, sstats, e_theta, phinorm


class LDA(Estimator):
    """``LDA(k=10, maxIter=20, optimizer="online", learningOffset=1024, learningDecay=0.51,
    subsamplingRate=0.05, optimizeDocConcentration=True)`` over term-count vectors."""
    _params = _LDA_PARAMS

    def __init__(self, **kwargs):
        super().__init__(**kwargs)
        for k in ("seed", "docConcentration", "topicConcentration"):
            self._defaultParamMap.pop(k, None)

    def _seed(self) -> int:
        from .tree_models import _default_seed
        return int(self.getOrDefault("seed")) if self.isSet("seed") else _default_seed(U.jvm_class(self))

    def _fit(self, df):
        opt = self.getOptimizer().lower()
        if opt == "em":
            return self._fit_em(df)
        if opt != "online":
            raise ValueError(f"LDA: optimizer must be 'online' or 'em', got {opt!r}")
        k = self.getK()
        if k < 2:
            raise ValueError("LDA: k must be > 1")
        comm = df._comm
        X = df._feature_matrix(self.getFeaturesCol()).to(torch.float64)
        ids = df._row_ids
        nonempty = X.sum(1) > 0
        X, ids = X[nonempty], ids[nonempty]
        V = X.shape[1]
        dev = X.device
        seed = self._seed()
        alpha = self._alpha0(k).to(dev)
        eta = self.getOrDefault("topicConcentration") if self.isSet("topicConcentration") else None
        eta = 1.0 / k if eta is None or eta < 0 else float(eta)
        cnt = torch.tensor([float(df._nrows)], dtype=torch.float64, device=dev)
        comm.allreduce_(cnt)
        corpus = float(cnt[0])
        gen = np.random.default_rng(seed & 0xFFFFFFFF)
        lam = torch.as_tensor(gen.gamma(GAMMA_SHAPE, 1.0 / GAMMA_SHAPE, size=(k, V)), device=dev)
        tau0, kappa, frac = self.getLearningOffset(), self.getLearningDecay(), self.getSubsamplingRate()
        for it in range(1, self.getMaxIter() + 1):
            e_beta = torch.exp(dirichlet_expectation(lam))
            pick = R.uniform(ids, seed, 1_000_003 + it) < frac
            Xb, ib = X[pick], ids[pick]
            stat = torch.zeros((k, V), dtype=torch.float64, device=dev)
            logphat = torch.zeros(k, dtype=torch.float64, device=dev)
            for a in range(0, Xb.shape[0], _CHUNK):
                xc, ic = Xb[a:a + _CHUNK], ib[a:a + _CHUNK]
                g, ss, _, _ = e_step(xc, e_beta, alpha, _gamma_init(ic, k, seed))
                stat += ss
                logphat += dirichlet_expectation(g).sum(0)
            msg = torch.cat([stat.reshape(-1), logphat, torch.tensor([float(Xb.shape[0])], dtype=torch.float64,
                                                                     device=dev)])
            comm.allreduce_(msg)
            nb = float(msg[-1])
            if nb == 0:
                continue
            stat = msg[:k * V].reshape(k, V)
            logphat = msg[k * V:k * V + k]
            rho = (tau0 + it) ** (-kappa)
            lam = (1.0 - rho) * lam + rho * (eta + stat * e_beta * (corpus / nb))
            if self.getOptimizeDocConcentration():
                alpha = _update_alpha(alpha, logphat / nb, nb, rho)
        model = LocalLDAModel(lam.T.cpu().numpy(), alpha.cpu().numpy(), eta, V)
        self._copyValues(model)
        model._gamma_seed = seed
        return model

    def _fit_em(self, df):
        """Spark's EMLDAOptimizer (MAP EM on the document-term graph) in dense form: with
        A = N_doc + (alpha - 1) and B = (N_term + (eta - 1)) / (N_k + V (eta - 1)), the token
        responsibilities are A_jk B_wk / (A B^T)_jw, so one EM iteration is two GEMMs,
        N_doc <- A * ((X / A B^T) B) and N_term <- B * ((X / A B^T)^T A), the latter all-reduced.
        Initial counts come from a uniform random soft assignment per (document, term) token."""
        k = self.getK()
        if k < 2:
            raise ValueError("LDA: k must be > 1")
        comm = df._comm
        X = df._feature_matrix(self.getFeaturesCol()).to(torch.float64)
        n, V = X.shape
        dev = X.device
        seed = self._seed()
        a = self.getOrDefault("docConcentration") if self.isSet("docConcentration") else None
        if a is None:
            alpha = 50.0 / k + 1.0
        else:
            av = [float(v) for v in (a if isinstance(a, (list, tuple, np.ndarray)) else [a])]
            if len(set(av)) != 1:
                raise ValueError("LDA(optimizer='em') needs a symmetric docConcentration")
            alpha = av[0] if av[0] >= 0 else 50.0 / k + 1.0
        eta = self.getOrDefault("topicConcentration") if self.isSet("topicConcentration") else None
        eta = 1.1 if eta is None or eta < 0 else float(eta)
        if alpha <= 1.0 or eta <= 1.0:
            raise ValueError("LDA(optimizer='em') needs docConcentration > 1 and topicConcentration > 1")
        # random soft assignment per token: gamma_jw ~ normalised uniform(k), one per (doc, term) pair
        nz = torch.nonzero(X > 0)
        ndoc = torch.zeros((n, k), dtype=torch.float64, device=dev)
        nterm = torch.zeros((V, k), dtype=torch.float64, device=dev)
        if nz.numel():
            rows, cols = nz[:, 0], nz[:, 1]
            key_ids = df._row_ids[rows] * V + cols
            g = torch.stack([R.uniform(key_ids, seed, 500 + t) for t in range(k)], 1)
            g = g / g.sum(1, keepdim=True) * X[rows, cols][:, None]
            ndoc.index_add_(0, rows, g)
            nterm.index_add_(0, cols, g)
        comm.allreduce_(nterm)
        for _ in range(self.getMaxIter()):
            nk = nterm.sum(0)
            A = ndoc + (alpha - 1.0)
            B = (nterm + (eta - 1.0)) / (nk + V * (eta - 1.0))[None, :]
            Z = A @ B.T
            Q = torch.where(X > 0, X / Z, torch.zeros_like(X))
            ndoc = A * (Q @ B)
            nterm = B * (Q.T @ A)
            comm.allreduce_(nterm)
        model = DistributedLDAModel(nterm.cpu().numpy(), np.full(k, alpha), eta, V)
        model._train_stats = _em_training_stats(X, ndoc, nterm, alpha, eta, comm)
        self._copyValues(model)
        model._gamma_seed = seed
        return model

    def _alpha0(self, k: int) -> torch.Tensor:
        a = self.getOrDefault("docConcentration") if self.isSet("docConcentration") else None
        if a is None:
            return torch.full((k,), 1.0 / k, dtype=torch.float64)
        a = [float(v) for v in (a if isinstance(a, (list, tuple, np.ndarray)) else [a])]
        if len(a) == 1:
            a = a * k
        if len(a) != k:
            raise ValueError(f"docConcentration must have length 1 or k = {k}")
        return torch.as_tensor(a, dtype=torch.float64)


def _update_alpha(alpha: torch.Tensor, logphat: torch.Tensor, n: float, rho: float) -> torch.Tensor:
    """One damped Newton step on the Dirichlet prior (Spark's OnlineLDAOptimizer.updateAlpha)."""
    gradf = n * (-dirichlet_expectation(alpha) + logphat)
    c = n * torch.special.polygamma(1, alpha.sum())
    q = -n * torch.special.polygamma(1, alpha)
    b = (gradf / q).sum() / (1.0 / c + (1.0 / q).sum())
    dalpha = -(gradf - b) / q
    nxt = alpha + rho * dalpha
    return nxt if bool((nxt > 0).all()) else alpha


class LocalLDAModel(Model):
    _params = _LDA_PARAMS

    def __init__(self, topics=None, alpha=None, eta: float = 0.0, vocab_size: int = 0):
        super().__init__()
        self._topics = np.asarray(topics if topics is not None else np.zeros((0, 0)), dtype=np.float64)  # [V, k]
        self._alpha = np.asarray(alpha if alpha is not None else [], dtype=np.float64)
        self._eta = float(eta)
        self._V = int(vocab_size)
        self._gamma_seed = 0

    # ------------------------------------------------------------------------ model API
    def isDistributed(self) -> bool:
        return False

    def vocabSize(self) -> int:
        return self._V

    def topicsMatrix(self) -> DenseMatrix:
        """[vocabSize, k] inferred (unnormalised) topics, column-major like Spark."""
        t = self._topics
        return DenseMatrix(t.shape[0], t.shape[1], t.T.reshape(-1))

    def estimatedDocConcentration(self) -> DenseVector:
        return DenseVector(self._alpha)

    def describeTopics(self, maxTermsPerTopic: int = 10):
        from ..sql.builder import rows_round_robin
        from ..sql.session import SparkSession
        lam = self._topics.T
        norm = lam / lam.sum(1, keepdims=True)
        rows = []
        for j in range(norm.shape[0]):
            order = np.argsort(-norm[j], kind="stable")[:maxTermsPerTopic]
            rows.append([j, [int(i) for i in order], [float(norm[j, i]) for i in order]])
        schema = T.StructType([T.StructField("topic", T.IntegerType(), False),
                               T.StructField("termIndices", T.ArrayType(T.IntegerType()), True),
                               T.StructField("termWeights", T.ArrayType(T.DoubleType()), True)])
        return rows_round_robin(SparkSession.builder.getOrCreate(), schema, rows)

    def _infer(self, df):
        X = df._feature_matrix(self.getFeaturesCol()).to(torch.float64)
        dev = X.device
        lam = torch.as_tensor(self._topics.T, device=dev)
        e_beta = torch.exp(dirichlet_expectation(lam))
        alpha = torch.as_tensor(self._alpha, device=dev)
        k = lam.shape[0]
        gammas = torch.zeros((X.shape[0], k), dtype=torch.float64, device=dev)
        lse_part = torch.zeros(X.shape[0], dtype=torch.float64, device=dev)
        for a in range(0, X.shape[0], _CHUNK):
            xc = X[a:a + _CHUNK]
            g, _, _, _ = e_step(xc, e_beta, alpha, _gamma_init(df._row_ids[a:a + _CHUNK], k, self._gamma_seed))
            gammas[a:a + _CHUNK] = g
        return X, gammas, lam, alpha

    def _transform(self, df):
        X, g, _, _ = self._infer(df)
        empty = X.sum(1) == 0
        dist = g / g.sum(1, keepdim=True)
        dist = torch.where(empty[:, None], torch.zeros_like(dist), dist)
        return _replace_col(df, self.getTopicDistributionCol(), ColumnData(dist.contiguous(), None, T.VectorUDT()))

    def logLikelihood(self, dataset) -> float:
        """Variational lower bound on log p(corpus) (Spark's LDAModel.logLikelihood)."""
        X, g, lam, alpha = self._infer(dataset)
        nonempty = X.sum(1) > 0
        X, g = X[nonempty], g[nonempty]
        elog_theta = dirichlet_expectation(g)
        elog_beta = dirichlet_expectation(lam)
        # Σ_w c_w log Σ_k exp(E[log θ_k] + E[log β_kw]), via a stable logsumexp over k
        doc = torch.zeros((), dtype=torch.float64, device=X.device)
        step = max(1, (1 << 24) // max(1, lam.shape[0] * lam.shape[1]))  # bound the [B, k, V] temporary
        for a in range(0, X.shape[0], step):
            t = torch.logsumexp(elog_theta[a:a + step, :, None] + elog_beta[None, :, :], 1)
            doc = doc + (X[a:a + step] * t).sum()
        doc = doc + ((alpha[None, :] - g) * elog_theta).sum() + (torch.lgamma(g) - torch.lgamma(alpha)[None, :]).sum()
        doc = doc + (torch.lgamma(alpha.sum()) - torch.lgamma(g.sum(1))).sum()
        msg = doc.reshape(1).clone()
        dataset._comm.allreduce_(msg)
        eta = self._eta
        V = lam.shape[1]
        topics = ((eta - lam) * elog_beta).sum() + (torch.lgamma(lam) - math.lgamma(eta)).sum()
        topics = topics + (math.lgamma(eta * V) - torch.lgamma(lam.sum(1))).sum()
        return float(msg[0] + topics)

    def logPerplexity(self, dataset) -> float:
        X = dataset._feature_matrix(self.getFeaturesCol()).to(torch.float64)
        tok = X.sum().reshape(1).clone()
        dataset._comm.allreduce_(tok)
        return -self.logLikelihood(dataset) / float(tok[0])

    # ------------------------------------------------------------------------ persistence
    def _save_impl(self, path):
        import pyarrow as pa
        U.write_metadata(self, path)
        U.write_parquet(path, "data", pa.Table.from_pylist(
            [{"vocabSize": self._V, "topicsMatrix": U.matrix_struct(self._topics),
              "docConcentration": U.vector_struct(self._alpha), "topicConcentration": self._eta,
              "gammaShape": GAMMA_SHAPE}],
            schema=pa.schema([pa.field("vocabSize", pa.int32(), False), ("topicsMatrix", U.matrix_arrow_type()),
                              ("docConcentration", U.vector_arrow_type()),
                              pa.field("topicConcentration", pa.float64(), False),
                              pa.field("gammaShape", pa.float64(), False)])))

    @classmethod
    def _load_impl(cls, path, md):
        r = U.read_parquet(path, "data").to_pylist()[0]
        m = cls(U.matrix_from_struct(r["topicsMatrix"]), U.vector_from_struct(r["docConcentration"]),
                r["topicConcentration"], r["vocabSize"])
        U.apply_params(m, md)
        seed = md.get("paramMap", {}).get("seed")
        m._gamma_seed = int(seed) if seed is not None else 0
        return m


def _em_training_stats(X, ndoc, nterm, alpha: float, eta: float, comm):
    """(trainingLogLikelihood, logPrior) of an EM fit, as Spark's DistributedLDAModel defines them."""
    k = ndoc.shape[1]
    V = nterm.shape[0]
    nk = nterm.sum(0)
    phi = (nterm + (eta - 1.0)) / (nk + V * (eta - 1.0))[None, :]            # [V, k]
    nj = ndoc.sum(1, keepdim=True)
    theta = (ndoc + (alpha - 1.0)) / (nj + k * (alpha - 1.0))                 # [n, k]
    p = theta @ phi.T                                                          # [n, V]
    ll = torch.where(X > 0, X * torch.log(p.clamp(min=1e-300)), torch.zeros_like(X)).sum()
    doc_prior = ((alpha - 1.0) * torch.log(theta.clamp(min=1e-300))).sum()
    msg = torch.stack([ll, doc_prior]).clone()
    comm.allreduce_(msg)
    term_prior = ((eta - 1.0) * torch.log(phi.clamp(min=1e-300))).sum()
    return float(msg[0]), float(msg[1] + term_prior)


class DistributedLDAModel(LocalLDAModel):
    """The EM optimizer's model: term-topic counts N_wk as ``topicsMatrix`` plus the training
    statistics; inference on new documents uses the same variational E-step as ``toLocal()``."""

    def __init__(self, topics=None, alpha=None, eta: float = 0.0, vocab_size: int = 0):
        super().__init__(topics, alpha, eta, vocab_size)
        self._train_stats = (float("nan"), float("nan"))

    def isDistributed(self) -> bool:
        return True

    def toLocal(self) -> LocalLDAModel:
        m = LocalLDAModel(self._topics, self._alpha, self._eta, self._V)
        self._copyValues(m)
        m._gamma_seed = self._gamma_seed
        return m

    @property
    def trainingLogLikelihood(self) -> float:
        return self._train_stats[0]

    def logPrior(self) -> float:
        return self._train_stats[1]

    def getCheckpointFiles(self) -> List[str]:
        return []

    def deleteCheckpointFiles(self) -> None:
        return None

    def _save_impl(self, path):
        import pyarrow as pa
        super()._save_impl(path)
        U.write_parquet(path, "training", pa.table({"trainingLogLikelihood": [self._train_stats[0]],
                                                    "logPrior": [self._train_stats[1]]}))

    @classmethod
    def _load_impl(cls, path, md):
        m = super()._load_impl(path, md)
        try:
            r = U.read_parquet(path, "training").to_pylist()[0]
            m._train_stats = (r["trainingLogLikelihood"], r["logPrior"])
        except (OSError, FileNotFoundError, IndexError):
            pass
        return m


__all__: List[str] = ["LDA", "LocalLDAModel", "DistributedLDAModel", "dirichlet_expectation", "e_step"]
