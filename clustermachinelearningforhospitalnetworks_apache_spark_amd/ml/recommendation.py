"""ALS collaborative filtering (pyspark.ml.recommendation): e.g. hospital x service utilisation
matrices, patient x procedure affinities.

Alternating least squares with Spark's semantics (explicit: weighted-λ regularisation, λ·n_u on
the diagonal; implicit: Hu-Koren-Volinsky confidence 1 + α|r|), designed for the device: one half
iteration forms ALL per-user normal equations at once — the rank x rank outer products of the
rated items' factors are scattered into a [users, rank, rank] tensor with one ``index_add_`` — and
solves them with one batched Cholesky (``torch.linalg.cholesky`` / ``cholesky_solve``). Ratings
stay sharded across ranks; the per-user (or per-item) Gram blocks and right-hand sides are summed
with one all-reduce per half iteration, so every rank holds identical factors.
"""
from __future__ import annotations

from typing import List

import numpy as np
import torch

from ..sql import types as T
from ..sql.column import ColumnData
from . import util as U
from .base import Estimator, Model
from .feature import _replace_col

_ALS_PARAMS = {
    "rank": (10, "rank of the factorization", int),
    "maxIter": (10, "max number of iterations (>= 0)", int),
    "regParam": (0.1, "regularization parameter (>= 0)", float),
    "numUserBlocks": (10, "number of user blocks", int),
    "numItemBlocks": (10, "number of item blocks", int),
    "implicitPrefs": (False, "whether to use implicit preference", bool),
    "alpha": (1.0, "alpha for implicit preference", float),
    "userCol": ("user", "column name for user ids; ids must be integers", str),
    "itemCol": ("item", "column name for item ids; ids must be integers", str),
    "ratingCol": ("rating", "column name for ratings", str),
    "nonnegative": (False, "whether to use nonnegative constraint for least squares", bool),
    "checkpointInterval": (10, "checkpoint interval (>= 1) or -1 to disable", int),
    "intermediateStorageLevel": ("MEMORY_AND_DISK", "StorageLevel for intermediate datasets", str),
    "finalStorageLevel": ("MEMORY_AND_DISK", "StorageLevel for ALS model factors", str),
    "coldStartStrategy": ("nan", "strategy for unknown or unseen ids at prediction time: 'nan' or 'drop'", str),
    "blockSize": (4096, "block size for stacking input data in matrices", int),
    "predictionCol": ("prediction", "prediction column name", str),
    "seed": (None, "random seed", None),
}


def _ids(df, col: str) -> torch.Tensor:
    cd = df._column_data(col)
    v = cd.values
    if v.is_floating_point():
        if bool((v != torch.floor(v)).any()):
            raise ValueError(f"ALS: {col} ids must be integers")
    return v.to(torch.int64)


def _solve_side(fixed: torch.Tensor, idx_solve: torch.Tensor, idx_fixed: torch.Tensor, r: torch.Tensor, n_solve: int,
                lam: float, implicit: bool, alpha: float, nonneg: bool, comm) -> torch.Tensor:
    """New factors of the solved side (users or items) given the fixed side's factors."""
    k = fixed.shape[1]
    dev = fixed.device
    Y = fixed[idx_fixed]                         # [nnz, k]
    if implicit:
        c = 1.0 + alpha * r.abs()                # confidence
        p = (r > 0).to(torch.float64)            # preference
        w_outer = (c - 1.0)                      # Yᵀ(C-I)Y term
        rhs_w = c * p
    else:
        w_outer = torch.ones_like(r)
        rhs_w = r
    A = torch.zeros((n_solve, k, k), dtype=torch.float64, device=dev)
    A.index_add_(0, idx_solve, (Y * w_outer[:, None])[:, :, None] * Y[:, None, :])
    b = torch.zeros((n_solve, k), dtype=torch.float64, device=dev)
    b.index_add_(0, idx_solve, Y * rhs_w[:, None])
    cnt = torch.zeros(n_solve, dtype=torch.float64, device=dev)
    cnt.index_add_(0, idx_solve, torch.ones_like(r))
    msg = torch.cat([A.reshape(-1), b.reshape(-1), cnt])
    comm.allreduce_(msg)
    A = msg[: n_solve * k * k].reshape(n_solve, k, k)
    b = msg[n_solve * k * k: n_solve * k * k + n_solve * k].reshape(n_solve, k)
    cnt = msg[n_solve * k * k + n_solve * k:]
    eye = torch.eye(k, dtype=torch.float64, device=dev)
    if implicit:
        A = A + (fixed.T @ fixed)[None] + lam * cnt[:, None, None] * eye
    else:
        A = A + lam * cnt[:, None, None] * eye
    has = cnt > 0
    A = torch.where(has[:, None, None], A, eye.expand_as(A))
    if nonneg:
        x = _nnls_batched(A, b)
    else:
        L = torch.linalg.cholesky(A)
        x = torch.cholesky_solve(b[:, :, None], L)[:, :, 0]
    return torch.where(has[:, None], x, torch.zeros_like(x))


def _nnls_batched(A: torch.Tensor, b: torch.Tensor, iters: int = 200) -> torch.Tensor:
    """min ½xᵀAx − bᵀx s.t. x >= 0 for a batch of small SPD systems: projected gradient with a
    per-system step 1/λ_max (converges for SPD A; Spark uses an active-set NNLS)."""
    lmax = torch.linalg.eigvalsh(A)[:, -1].clamp(min=1e-12)
    x = torch.zeros_like(b)
    for _ in range(iters):
        g = (A @ x[:, :, None])[:, :, 0] - b
        x = (x - g / lmax[:, None]).clamp(min=0.0)
    return x


class ALS(Estimator):
    _params = _ALS_PARAMS

    def __init__(self, **kwargs):
        super().__init__(**kwargs)
        self._defaultParamMap.pop("seed", None)

    def _fit(self, df):
        from .tree_models import _default_seed
        u = _ids(df, self.getUserCol())
        i = _ids(df, self.getItemCol())
        r = df._column_data(self.getRatingCol()).values.to(torch.float64)
        comm = df._comm
        nu = int(comm.max_scalar(float(u.max().item()) if u.numel() else -1.0)) + 1
        ni = int(comm.max_scalar(float(i.max().item()) if i.numel() else -1.0)) + 1
        lo = comm.max_scalar(-float(min(u.min().item(), i.min().item())) if u.numel() else 0.0)
        if lo > 0:
            raise ValueError("ALS: user and item ids must be non-negative")
        k = self.getRank()
        seed = int(self.getOrDefault("seed")) if self.isSet("seed") else _default_seed(U.jvm_class(self))
        g = np.random.default_rng(seed & 0xFFFFFFFF)
        # Spark initialises factors with |N(0,1)| / sqrt(rank)-scaled rows (nonnegative-safe)
        U0 = np.abs(g.normal(size=(nu, k))) / np.sqrt(k)
        V0 = np.abs(g.normal(size=(ni, k))) / np.sqrt(k)
        dev = df._device
        Uf = torch.as_tensor(U0, device=dev)
        Vf = torch.as_tensor(V0, device=dev)
        lam, alpha = self.getRegParam(), self.getAlpha()
        imp, nn = self.getImplicitPrefs(), self.getNonnegative()
        for _ in range(self.getMaxIter()):
            Vf = _solve_side(Uf, i, u, r, ni, lam, imp, alpha, nn, comm)
            Uf = _solve_side(Vf, u, i, r, nu, lam, imp, alpha, nn, comm)
        uid = torch.unique(comm.allgather_cat(torch.unique(u))).cpu().numpy()
        iid = torch.unique(comm.allgather_cat(torch.unique(i))).cpu().numpy()
        model = ALSModel(k, uid, Uf.cpu().numpy()[uid], iid, Vf.cpu().numpy()[iid])
        self._copyValues(model)
        return model


class ALSModel(Model):
    _params = _ALS_PARAMS

    def __init__(self, rank: int = 0, userIds=None, userF=None, itemIds=None, itemF=None):
        super().__init__()
        self._rank = int(rank)
        self._uid = np.asarray(userIds if userIds is not None else [], dtype=np.int64)
        self._uf = np.asarray(userF if userF is not None else np.zeros((0, rank)), dtype=np.float64)
        self._iid = np.asarray(itemIds if itemIds is not None else [], dtype=np.int64)
        self._if = np.asarray(itemF if itemF is not None else np.zeros((0, rank)), dtype=np.float64)

    @property
    def rank(self) -> int:
        return self._rank

    def _session(self):
        from ..sql.session import SparkSession
        return SparkSession.builder.getOrCreate()

    def _factors_df(self, ids, F):
        from ..sql.builder import rows_round_robin
        schema = T.StructType([T.StructField("id", T.IntegerType(), False),
                               T.StructField("features", T.ArrayType(T.FloatType()), True)])
        return rows_round_robin(self._session(), schema, [[int(a), [float(v) for v in f]] for a, f in zip(ids, F)])

    @property
    def userFactors(self):
        return self._factors_df(self._uid, self._uf)

    @property
    def itemFactors(self):
        return self._factors_df(self._iid, self._if)

    def _lookup(self, ids: torch.Tensor, known: np.ndarray, F: np.ndarray):
        dev = ids.device
        kt = torch.as_tensor(known, device=dev)
        pos = torch.searchsorted(kt, ids).clamp(max=max(len(known) - 1, 0))
        hit = (kt[pos] == ids) if len(known) else torch.zeros_like(ids, dtype=torch.bool)
        Ft = torch.as_tensor(F, device=dev)
        return (Ft[pos] if len(known) else torch.zeros((ids.numel(), self._rank), dtype=torch.float64,
                                                       device=dev)), hit

    def _transform(self, df):
        u = _ids(df, self.getUserCol())
        i = _ids(df, self.getItemCol())
        Uu, hu = self._lookup(u, self._uid, self._uf)
        Vi, hi = self._lookup(i, self._iid, self._if)
        pred = (Uu * Vi).sum(1).to(torch.float32)
        ok = hu & hi
        pred = torch.where(ok, pred, torch.full_like(pred, float("nan")))
        out = _replace_col(df, self.getPredictionCol(), ColumnData(pred, None, T.FloatType()))
        if self.getColdStartStrategy() == "drop":
            out = out._mask_rows(ok)
        return out

    def _recommend(self, src_ids, src_F, dst_ids, dst_F, n: int, src_name: str, dst_name: str):
        from ..sql.builder import rows_round_robin
        S = torch.as_tensor(src_F)
        D = torch.as_tensor(dst_F)
        scores = S @ D.T  # hipBLASLt on a device session would be the same GEMM; factors are small
        k = min(n, len(dst_ids))
        top = torch.topk(scores, k, dim=1) if k else None
        rows = []
        for a in range(len(src_ids)):
            recs = [] if top is None else [(int(dst_ids[j]), float(s)) for s, j in
                                          zip(top.values[a].tolist(), top.indices[a].tolist())]
            rows.append([int(src_ids[a]), recs])
        schema = T.StructType([T.StructField(src_name, T.IntegerType(), False),
                               T.StructField("recommendations", T.ArrayType(T.StructType([
                                   T.StructField(dst_name, T.IntegerType()), T.StructField("rating", T.FloatType())])))])
        from ..sql.types import Row
        rows = [[r[0], [Row(**{dst_name: a, "rating": b}) for a, b in r[1]]] for r in rows]
        return rows_round_robin(self._session(), schema, rows)

    def recommendForAllUsers(self, numItems: int):
        return self._recommend(self._uid, self._uf, self._iid, self._if, numItems, self.getUserCol(),
                               self.getItemCol())

    def recommendForAllItems(self, numUsers: int):
        return self._recommend(self._iid, self._if, self._uid, self._uf, numUsers, self.getItemCol(),
                               self.getUserCol())

    def _subset(self, df, col, ids, F):
        from ..sql.dataframe import column_to_python
        want = set()
        for part in df._comm.allgather_object([int(v) for v in column_to_python(df._column_data(col))]):
            want |= set(part)
        m = np.isin(ids, np.array(sorted(want), dtype=np.int64))
        return ids[m], F[m]

    def recommendForUserSubset(self, dataset, numItems: int):
        ids, F = self._subset(dataset, self.getUserCol(), self._uid, self._uf)
        return self._recommend(ids, F, self._iid, self._if, numItems, self.getUserCol(), self.getItemCol())

    def recommendForItemSubset(self, dataset, numUsers: int):
        ids, F = self._subset(dataset, self.getItemCol(), self._iid, self._if)
        return self._recommend(ids, F, self._uid, self._uf, numUsers, self.getItemCol(), self.getUserCol())

    def _save_impl(self, path):
        import pyarrow as pa
        U.write_metadata(self, path, extra={"rank": self._rank})
        sch = pa.schema([pa.field("id", pa.int32(), False), ("features", pa.list_(pa.float32()))])
        for sub, ids, F in (("userFactors", self._uid, self._uf), ("itemFactors", self._iid, self._if)):
            U.write_parquet(path, sub, pa.Table.from_pylist(
                [{"id": int(a), "features": [float(v) for v in f]} for a, f in zip(ids, F)], schema=sch))

    @classmethod
    def _load_impl(cls, path, md):
        uf = U.read_parquet(path, "userFactors").to_pylist()
        itf = U.read_parquet(path, "itemFactors").to_pylist()
        rank = int(md.get("rank", len(uf[0]["features"]) if uf else 0))
        m = cls(rank, [r["id"] for r in uf], np.array([r["features"] for r in uf]).reshape(len(uf), rank),
                [r["id"] for r in itf], np.array([r["features"] for r in itf]).reshape(len(itf), rank))
        U.apply_params(m, md)
        return m


__all__: List[str] = ["ALS", "ALSModel"]
