"""Locality-sensitive hashing (pyspark.ml.feature): BucketedRandomProjectionLSH (euclidean) and
MinHashLSH (Jaccard), with ``approxNearestNeighbors`` and ``approxSimilarityJoin`` — e.g. "hospitals
with a similar load profile", "admissions with similar diagnosis sets".

Device design: hashing a shard is one [n, d] x [d, L] GEMM (random projections) or one masked
min-reduction over the non-zero positions (min-hash), and candidate distances are one more GEMM /
masked reduction — the candidate filter and distance computation never leave the device. Random
coefficients come from ``java.util.Random(seed)`` exactly as Spark draws them
(``nextGaussian`` unit vectors; ``nextInt`` min-hash coefficients), so saved models match.
"""
from __future__ import annotations

from typing import List

import numpy as np
import torch

from ..sql import types as T
from ..sql.column import ColumnData
from . import util as U
from .util import JavaRandom
from .base import Estimator, Model
from .colutil import _auto_output, _replace_col
from .linalg import DenseVector, as_array
from .param import NO_DEFAULT

HASH_PRIME = 2038074743

_LSH_COMMON = {
    "inputCol": (NO_DEFAULT, "input column name", str),
    "outputCol": ("__auto__", "output column name", str),
    "numHashTables": (1, "number of hash tables, where increasing number of hash tables lowers the false "
                         "negative rate, and decreasing it improves the running performance", int),
    "seed": (None, "random seed", None),
}


def _seed(est) -> int:
    from .tree_models import _default_seed
    return int(est.getOrDefault("seed")) if est.isSet("seed") else _default_seed(U.jvm_class(est))


class _LSHModel(Model):
    """Shared query logic; subclasses define ``_hash`` ([n, L] float64 hash values) and
    ``_dist_to`` (distances of rows to one key)."""

    def _hash_col(self, x: torch.Tensor):
        h = self._hash(x)
        out = np.empty(h.shape[0], dtype=object)
        hc = h.cpu().numpy()
        for i in range(h.shape[0]):
            out[i] = [DenseVector([v]) for v in hc[i]]
        return out

    def _transform(self, df):
        x = df._feature_matrix(self.getInputCol())
        return _replace_col(df, self.getOutputCol(), ColumnData(self._hash_col(x), None,
                                                                T.ArrayType(T.VectorUDT())))

    def approxNearestNeighbors(self, dataset, key, numNearestNeighbors: int, distCol: str = "distCol"):
        """Rows sharing at least one bucket with ``key`` (single probe), the ``numNearestNeighbors``
        closest by the exact key distance, with the distance in ``distCol``."""
        x = dataset._feature_matrix(self.getInputCol())
        kv = torch.as_tensor(np.asarray(as_array(key), dtype=np.float64), device=x.device)
        hx = self._hash(x)
        hk = self._hash(kv[None, :])[0]
        cand = (hx == hk[None, :]).any(1)
        dist = self._dist_to(x, kv)
        sub = dataset if self.getOutputCol() in dataset.columns else self.transform(dataset)
        sub = _replace_col(sub, distCol, ColumnData(dist, None, T.DoubleType()))
        sub = sub._mask_rows(cand)
        return sub.orderBy(distCol).limit(int(numNearestNeighbors))

    def approxSimilarityJoin(self, datasetA, datasetB, threshold: float, distCol: str = "distCol"):
        """Pairs (a, b) that share a bucket in some hash table and whose key distance is below
        ``threshold``; output columns ``datasetA`` / ``datasetB`` (row structs) and ``distCol``."""
        from ..sql.builder import rows_round_robin
        from ..sql.types import Row
        ta = datasetA if self.getOutputCol() in datasetA.columns else self.transform(datasetA)
        tb = datasetB if self.getOutputCol() in datasetB.columns else self.transform(datasetB)
        na, ra, _ = ta._gather_host()
        nb, rb, _ = tb._gather_host()
        ia, ib = na.index(self.getInputCol()), nb.index(self.getInputCol())
        dev = datasetA._device
        xa = torch.as_tensor(np.stack([np.asarray(as_array(r[ia]), dtype=np.float64) for r in ra]), device=dev) \
            if ra else None
        xb = torch.as_tensor(np.stack([np.asarray(as_array(r[ib]), dtype=np.float64) for r in rb]), device=dev) \
            if rb else None
        rows = []
        if xa is not None and xb is not None:
            ha, hb = self._hash(xa), self._hash(xb)
            same = torch.zeros((xa.shape[0], xb.shape[0]), dtype=torch.bool, device=dev)
            for t in range(ha.shape[1]):
                same |= ha[:, t:t + 1] == hb[None, :, t]
            D = self._pair_dist(xa, xb)
            ok = same & (D < threshold)
            for i, j in torch.nonzero(ok).cpu().tolist():
                rows.append([Row(**dict(zip(na, ra[i]))), Row(**dict(zip(nb, rb[j]))), float(D[i, j])])
        schema = T.StructType([T.StructField("datasetA", T.StructType([T.StructField(n, f.dataType) for n, f in
                                                                       zip(na, ta.schema.fields)])),
                               T.StructField("datasetB", T.StructType([T.StructField(n, f.dataType) for n, f in
                                                                       zip(nb, tb.schema.fields)])),
                               T.StructField(distCol, T.DoubleType())])
        return rows_round_robin(datasetA._session, schema, rows)


# ------------------------------------------------------------------------- BucketedRandomProjectionLSH

_BRP_PARAMS = dict(_LSH_COMMON, bucketLength=(NO_DEFAULT, "the length of each hash bucket, a larger bucket "
                                                          "lowers the false negative rate", float))


class BucketedRandomProjectionLSH(Estimator):
    """h_j(x) = floor(x · u_j / bucketLength) for unit vectors u_j drawn with nextGaussian."""
    _params = _BRP_PARAMS

    def __init__(self, inputCol=None, outputCol=None, seed=None, numHashTables=None, bucketLength=None):
        super().__init__(inputCol=inputCol, outputCol=outputCol, seed=seed, numHashTables=numHashTables,
                         bucketLength=bucketLength)
        self._defaultParamMap.pop("seed", None)
        _auto_output(self)

    def _fit(self, df):
        d = df._feature_matrix(self.getInputCol()).shape[1]
        rnd = JavaRandom(_seed(self))
        vs = []
        for _ in range(self.getNumHashTables()):
            v = np.array([rnd.next_gaussian() for _ in range(d)])
            vs.append(v / np.linalg.norm(v))
        m = BucketedRandomProjectionLSHModel(np.stack(vs) if vs else np.zeros((0, d)))
        self._copyValues(m)
        return m


class BucketedRandomProjectionLSHModel(_LSHModel):
    _params = _BRP_PARAMS

    def __init__(self, randUnitVectors=None):
        super().__init__()
        self._R = np.asarray(randUnitVectors if randUnitVectors is not None else np.zeros((0, 0)), dtype=np.float64)

    def _hash(self, x: torch.Tensor) -> torch.Tensor:
        R = torch.as_tensor(self._R, device=x.device)
        return torch.floor((x.to(torch.float64) @ R.T) / self.getBucketLength())

    def _dist_to(self, x, key):
        return torch.linalg.vector_norm(x.to(torch.float64) - key[None, :], dim=1)

    def _pair_dist(self, a, b):
        return torch.cdist(a, b)

    def _save_impl(self, path):
        import pyarrow as pa
        U.write_metadata(self, path)
        U.write_parquet(path, "data", pa.Table.from_pylist([{"randUnitVectors": U.matrix_struct(self._R)}],
                                                           schema=pa.schema([("randUnitVectors",
                                                                              U.matrix_arrow_type())])))

    @classmethod
    def _load_impl(cls, path, md):
        r = U.read_parquet(path, "data").to_pylist()[0]
        m = cls(U.matrix_from_struct(r["randUnitVectors"]))
        U.apply_params(m, md)
        return m


# ----------------------------------------------------------------------------------------- MinHashLSH

class MinHashLSH(Estimator):
    """h_j(x) = min over non-zero positions i of ((1 + i)·a_j + b_j) mod 2038074743 (Spark's
    MinHashLSH); Jaccard distance on the sets of non-zero positions."""
    _params = dict(_LSH_COMMON)

    def __init__(self, inputCol=None, outputCol=None, seed=None, numHashTables=None):
        super().__init__(inputCol=inputCol, outputCol=outputCol, seed=seed, numHashTables=numHashTables)
        self._defaultParamMap.pop("seed", None)
        _auto_output(self)

    def _fit(self, df):
        rnd = JavaRandom(_seed(self))
        coefs = []
        for _ in range(self.getNumHashTables()):
            a = 1 + rnd.next_int(HASH_PRIME - 1)
            b = rnd.next_int(HASH_PRIME - 1)
            coefs.append((a, b))
        m = MinHashLSHModel(coefs)
        self._copyValues(m)
        return m


class MinHashLSHModel(_LSHModel):
    _params = MinHashLSH._params

    def __init__(self, randCoefficients=None):
        super().__init__()
        self._coefs = [(int(a), int(b)) for a, b in (randCoefficients or [])]

    def _hash(self, x: torch.Tensor) -> torch.Tensor:
        nz = x != 0
        if bool((~nz.any(1)).any()):
            raise ValueError("MinHashLSH: must have at least 1 non zero entry")
        idx = torch.arange(1, x.shape[1] + 1, dtype=torch.int64, device=x.device)
        outs = []
        big = torch.iinfo(torch.int64).max
        for a, b in self._coefs:
            hv = (idx * a + b) % HASH_PRIME  # < 2^31 * 2^31: fits int64
            outs.append(torch.where(nz, hv[None, :], torch.full_like(hv[None, :], big)).amin(1))
        return torch.stack(outs, 1).to(torch.float64) if outs else torch.zeros((x.shape[0], 0), dtype=torch.float64,
                                                                                device=x.device)

    def _dist_to(self, x, key):
        a = x != 0
        k = (key != 0)[None, :]
        inter = (a & k).sum(1).to(torch.float64)
        union = (a | k).sum(1).to(torch.float64)
        return 1.0 - inter / union.clamp(min=1.0)

    def _pair_dist(self, a, b):
        A = (a != 0).to(torch.float64)
        B = (b != 0).to(torch.float64)
        inter = A @ B.T
        union = A.sum(1)[:, None] + B.sum(1)[None, :] - inter
        return 1.0 - inter / union.clamp(min=1.0)

    def _save_impl(self, path):
        import pyarrow as pa
        U.write_metadata(self, path)
        flat = [v for ab in self._coefs for v in ab]
        U.write_parquet(path, "data", pa.table({"randCoefficients": pa.array([flat], type=pa.list_(pa.int32()))}))

    @classmethod
    def _load_impl(cls, path, md):
        flat = U.read_parquet(path, "data").to_pylist()[0]["randCoefficients"]
        m = cls(list(zip(flat[0::2], flat[1::2])))
        U.apply_params(m, md)
        return m


__all__: List[str] = ["BucketedRandomProjectionLSH", "BucketedRandomProjectionLSHModel", "MinHashLSH",
                      "MinHashLSHModel"]
