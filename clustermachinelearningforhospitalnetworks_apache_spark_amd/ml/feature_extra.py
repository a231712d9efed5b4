"""More pyspark.ml.feature transformers for tabular hospital data: Bucketizer,
QuantileDiscretizer, Normalizer and PCA.

The reference (ref.py:134-136) only assembles raw numeric columns; these are the
standard MLlib steps a user of that pipeline reaches for next (binning occupancy,
decorrelating the feature vector).  Design, MI355X-first:

* Bucketizer: one device ``searchsorted`` against the split array (left-closed
  buckets, last bucket closed on the right, Spark's NaN policy via handleInvalid).
* QuantileDiscretizer.fit: exact order statistics of the global column (shards
  gathered once, sorted on the device), splits = distinct quantiles at
  ``[0, 1/B, ..., 1]`` with ±inf at the ends, as Spark's ``approxQuantile`` at
  relativeError 0 would give; returns a Bucketizer (as Spark does).
* PCA.fit: covariance from the K15 Gram kernel (``[X 1 0]ᵀ[X 1 0]`` in float64,
  one all-reduce of (d+2)² doubles), eigen-decomposition on the host; ``transform``
  projects without centring (Spark's ``PCAModel.transform``).
"""
from __future__ import annotations

from typing import List

import numpy as np
import torch

from ..ops import glm_ops
from ..sql import types as T
from ..sql.column import ColumnData
from . import util as U
from .base import Estimator, Model, Transformer
from .colutil import _auto_output, _replace_col
from .linalg import DenseMatrix, DenseVector
from .param import NO_DEFAULT


class Bucketizer(Transformer):
    """Maps a continuous column to bucket indices: bucket j holds splits[j] <= x < splits[j+1],
    the last bucket also holds x == splits[-1].  handleInvalid: 'error' (NaN or out of range
    raises), 'skip' (drop those rows), 'keep' (NaN -> extra bucket len(splits) - 1)."""
    _params = {
        "splits": (NO_DEFAULT, "split points for mapping continuous features into buckets", None),
        "inputCol": (NO_DEFAULT, "input column name", str),
        "outputCol": ("__auto__", "output column name", str),
        "handleInvalid": ("error", "how to handle invalid entries: 'error', 'skip' or 'keep'", str),
    }

    def __init__(self, splits=None, inputCol=None, outputCol=None, handleInvalid=None):
        super().__init__(splits=splits, inputCol=inputCol, outputCol=outputCol, handleInvalid=handleInvalid)
        _auto_output(self)

    def _check_splits(self) -> np.ndarray:
        s = np.asarray(self.getSplits(), dtype=np.float64)
        if s.size < 3 or np.any(np.diff(s) <= 0):
            raise ValueError("Bucketizer splits must hold at least 3 strictly increasing values")
        return s

    def _transform(self, df):
        s = self._check_splits()
        cd = df._column_data(self.getInputCol())
        v = cd.values.to(torch.float64)
        st = torch.as_tensor(s, device=v.device)
        nb = s.size - 1
        idx = torch.searchsorted(st, v.contiguous(), right=True) - 1
        idx = torch.where(v == st[-1], torch.full_like(idx, nb - 1), idx)
        nan = torch.isnan(v)
        bad = (~nan) & ((idx < 0) | (idx >= nb))
        if cd.valid is not None:
            nan = nan | ~cd.valid
        mode = self.getHandleInvalid()
        if bool(bad.any()):
            raise ValueError(f"Bucketizer: value outside the splits [{s[0]}, {s[-1]}] in {self.getInputCol()!r}")
        if mode == "error" and bool(nan.any()):
            raise ValueError("Bucketizer: NaN/null values; set handleInvalid to 'skip' or 'keep'")
        out = torch.where(nan, torch.full_like(idx, nb), idx).to(torch.float64)
        res = _replace_col(df, self.getOutputCol(), ColumnData(out, None, T.DoubleType()))
        if mode == "skip" and bool(nan.any()):
            res = res._take_rows(torch.nonzero(~nan).flatten())
        return res


class QuantileDiscretizer(Estimator):
    """Fits a Bucketizer whose splits are the column's quantiles (numBuckets buckets, fewer when
    quantiles coincide).  NaN/null values are ignored by the fit."""
    _params = {
        "numBuckets": (2, "number of buckets (quantiles, or categories) into which data points are grouped", int),
        "inputCol": (NO_DEFAULT, "input column name", str),
        "outputCol": ("__auto__", "output column name", str),
        "relativeError": (0.001, "the relative target precision for the approximate quantile algorithm", float),
        "handleInvalid": ("error", "how to handle invalid entries: 'error', 'skip' or 'keep'", str),
    }

    def __init__(self, numBuckets=None, inputCol=None, outputCol=None, relativeError=None, handleInvalid=None):
        super().__init__(numBuckets=numBuckets, inputCol=inputCol, outputCol=outputCol, relativeError=relativeError,
                         handleInvalid=handleInvalid)
        _auto_output(self)

    def _fit(self, df):
        nb = self.getNumBuckets()
        if nb < 2:
            raise ValueError("numBuckets must be >= 2")
        cd = df._column_data(self.getInputCol())
        v = cd.values.to(torch.float64)
        ok = ~torch.isnan(v)
        if cd.valid is not None:
            ok = ok & cd.valid
        allv = df._comm.allgather_cat(v[ok].contiguous())
        srt = torch.sort(allv).values.cpu().numpy()
        n = srt.size
        if n == 0:
            raise ValueError("QuantileDiscretizer: no valid values to fit")
        probs = np.arange(nb + 1) / nb
        ranks = np.clip(np.ceil(probs * n).astype(np.int64) - 1, 0, n - 1)
        qs = srt[ranks].astype(np.float64)
        qs[0], qs[-1] = -np.inf, np.inf  # Spark: ends replaced by ±inf, then distinct
        splits = np.unique(qs)
        b = Bucketizer(splits=splits.tolist(), inputCol=self.getInputCol(), outputCol=self.getOutputCol(),
                       handleInvalid=self.getHandleInvalid())
        return b


class Normalizer(Transformer):
    """Scales every vector to unit p-norm (p >= 1, inf allowed); zero vectors stay zero."""
    _params = {
        "p": (2.0, "the p norm value", float),
        "inputCol": (NO_DEFAULT, "input column name", str),
        "outputCol": ("__auto__", "output column name", str),
    }

    def __init__(self, p=None, inputCol=None, outputCol=None):
        super().__init__(p=p, inputCol=inputCol, outputCol=outputCol)
        _auto_output(self)

    def _transform(self, df):
        x = df._feature_matrix(self.getInputCol()).to(torch.float64)
        p = float(self.getP())
        if p < 1:
            raise ValueError("Normalizer: p must be >= 1")
        nrm = torch.linalg.vector_norm(x, ord=p, dim=1, keepdim=True)
        out = torch.where(nrm > 0, x / nrm.clamp(min=1e-300), torch.zeros_like(x))
        return _replace_col(df, self.getOutputCol(), ColumnData(out, None, T.VectorUDT()))


class PCA(Estimator):
    _params = {
        "k": (NO_DEFAULT, "the number of principal components (> 0)", int),
        "inputCol": (NO_DEFAULT, "input column name", str),
        "outputCol": ("__auto__", "output column name", str),
    }

    def __init__(self, k=None, inputCol=None, outputCol=None):
        super().__init__(k=k, inputCol=inputCol, outputCol=outputCol)
        _auto_output(self)

    def _fit(self, df):
        x = df._feature_matrix(self.getInputCol())
        d = x.shape[1]
        k = self.getK()
        if not 0 < k <= d:
            raise ValueError(f"PCA: k={k} must be in [1, {d}]")
        zero = torch.zeros(x.shape[0], dtype=torch.float64, device=x.device)
        G = glm_ops.gram(x, d, zero)  # K15: [X 1 0]ᵀ[X 1 0]
        df._comm.allreduce_(G)
        g = G.cpu().numpy()
        n = g[d, d]
        if n < 2:
            raise ValueError("PCA needs at least 2 rows")
        s = g[:d, d]
        cov = (g[:d, :d] - np.outer(s, s) / n) / (n - 1)
        cov = 0.5 * (cov + cov.T)
        w, v = np.linalg.eigh(cov)
        order = np.argsort(w)[::-1]
        w, v = np.clip(w[order], 0.0, None), v[:, order]
        # deterministic orientation: the largest-magnitude entry of each component is positive
        sign = np.sign(v[np.argmax(np.abs(v), axis=0), np.arange(d)])
        v = v * np.where(sign == 0, 1.0, sign)
        tot = w.sum()
        ev = w[:k] / tot if tot > 0 else np.zeros(k)
        m = PCAModel(v[:, :k], ev)
        self._copyValues(m)
        return m


class PCAModel(Model):
    _params = PCA._params

    def __init__(self, pc=None, explainedVariance=None):
        super().__init__()
        self._pc = np.asarray(pc if pc is not None else np.zeros((0, 0)), dtype=np.float64)
        self._ev = np.asarray(explainedVariance if explainedVariance is not None else [], dtype=np.float64)

    @property
    def pc(self) -> DenseMatrix:
        return DenseMatrix(self._pc.shape[0], self._pc.shape[1], self._pc.T.reshape(-1).tolist())

    @property
    def explainedVariance(self) -> DenseVector:
        return DenseVector(self._ev)

    def _transform(self, df):
        x = df._feature_matrix(self.getInputCol()).to(torch.float64)
        out = x @ torch.as_tensor(self._pc, device=x.device)
        return _replace_col(df, self.getOutputCol(), ColumnData(out.contiguous(), None, T.VectorUDT()))

    def _save_impl(self, path):
        import pyarrow as pa
        U.write_metadata(self, path)
        U.write_parquet(path, "data", pa.Table.from_pylist(
            [{"pc": U.matrix_struct(self._pc), "explainedVariance": U.vector_struct(self._ev)}],
            schema=pa.schema([("pc", U.matrix_arrow_type()), ("explainedVariance", U.vector_arrow_type())])))

    @classmethod
    def _load_impl(cls, path, md):
        row = U.read_parquet(path, "data").to_pylist()[0]
        m = cls(U.matrix_from_struct(row["pc"]), U.vector_from_struct(row["explainedVariance"]))
        U.apply_params(m, md)
        return m


__all__: List[str] = ["Bucketizer", "QuantileDiscretizer", "Normalizer", "PCA", "PCAModel"]
