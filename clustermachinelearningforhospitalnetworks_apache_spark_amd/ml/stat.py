"""pyspark.ml.stat: Correlation (pearson / spearman) and ChiSquareTest.

The reference only prints model metrics (ref.py:160-198); these are the MLlib
statistics a user inspects before modelling a feature table such as the
reference's (ref.py:134-136).  MI355X-first:

* Pearson: the covariance comes from the K15 Gram kernel (``[X 1 0]ᵀ[X 1 0]``
  accumulated in float64 on the device, one all-reduce of (d+2)² doubles), then a
  d×d normalisation on the host.
* Spearman: global average ranks per column (shards gathered once, ranked by a
  device sort), then Pearson on the ranks.
* ChiSquareTest: per-feature contingency tables by one device ``bincount`` over
  (feature value id, label id) pairs, summed across ranks.

Results are one-row DataFrames held by rank 0 (every rank's ``collect`` sees the
row), with the pyspark column names.
"""
from __future__ import annotations

from typing import List

import numpy as np
import torch

from ..ops import glm_ops
from ..sql import types as T
from ..sql.column import ColumnData
from .linalg import DenseMatrix, DenseVector


def _one_row(df, fields: List[T.StructField], values: List[object]):
    own = df._comm.rank == 0
    cols = {}
    for f, v in zip(fields, values):
        arr = np.empty(1 if own else 0, dtype=object)
        if own:
            arr[0] = v
        cols[f.name] = ColumnData(arr, None, f.dataType)
    row_ids = torch.arange(1 if own else 0, device=df._device)
    return df._new(T.StructType(fields), cols, 1 if own else 0, row_ids)


def _pearson_from_gram(g: np.ndarray, d: int) -> np.ndarray:
    n = g[d, d]
    s = g[:d, d]
    cov = (g[:d, :d] - np.outer(s, s) / n) / max(n - 1.0, 1.0)
    sd = np.sqrt(np.clip(np.diag(cov), 0.0, None))
    with np.errstate(divide="ignore", invalid="ignore"):
        corr = cov / np.outer(sd, sd)
    corr = np.clip(corr, -1.0, 1.0)
    nz = sd > 0
    corr[np.ix_(~nz, np.arange(d))] = np.nan
    corr[np.ix_(np.arange(d), ~nz)] = np.nan
    np.fill_diagonal(corr, 1.0)
    return corr


def _avg_ranks(col: torch.Tensor) -> torch.Tensor:
    """1-based average ranks (ties share the mean of their positions)."""
    n = col.numel()
    srt, order = torch.sort(col, stable=True)
    _, inv, counts = torch.unique_consecutive(srt, return_inverse=True, return_counts=True)
    ends = torch.cumsum(counts, 0).to(torch.float64)
    avg = ends - (counts.to(torch.float64) - 1.0) / 2.0
    r = torch.empty(n, dtype=torch.float64, device=col.device)
    r[order] = avg[inv]
    return r


class Correlation:
    @staticmethod
    def corr(dataset, column: str, method: str = "pearson"):
        method = method.lower()
        if method not in ("pearson", "spearman"):
            raise ValueError(f"unsupported correlation method {method!r}")
        x = dataset._feature_matrix(column)
        d = x.shape[1]
        comm = dataset._comm
        if method == "spearman":
            allx = comm.allgather_cat(x.to(torch.float64).contiguous())
            ranks = torch.stack([_avg_ranks(allx[:, j].contiguous()) for j in range(d)], 1)
            x = ranks if comm.rank == 0 else ranks[:0]  # every rank holds all ranks: count them once
        zero = torch.zeros(x.shape[0], dtype=torch.float64, device=x.device)
        G = glm_ops.gram(x, d, zero)
        comm.allreduce_(G)
        corr = _pearson_from_gram(G.cpu().numpy(), d)
        m = DenseMatrix(d, d, corr.T.reshape(-1))
        return _one_row(dataset, [T.StructField(f"{method}({column})", T.MatrixUDT(), False)], [m])


class ChiSquareTest:
    @staticmethod
    def test(dataset, featuresCol: str, labelCol: str, flatten: bool = False):
        """Pearson's independence test of every (categorical) feature against the label."""
        from scipy.stats import chi2
        x = dataset._feature_matrix(featuresCol).to(torch.float64)
        y = dataset._column_data(labelCol).values.to(torch.float64)
        comm = dataset._comm
        d = x.shape[1]
        labels = np.unique(comm.allgather_cat(torch.unique(y)).cpu().numpy())
        lab_t = torch.as_tensor(labels, device=y.device)
        yi = torch.searchsorted(lab_t, y.contiguous())
        pv, dof, stat = [], [], []
        for j in range(d):
            col = x[:, j].contiguous()
            vals = np.unique(comm.allgather_cat(torch.unique(col)).cpu().numpy())
            if vals.size > 10000:
                raise ValueError(f"ChiSquareTest: feature {j} has {vals.size} distinct values (> 10000)")
            vi = torch.searchsorted(torch.as_tensor(vals, device=col.device), col)
            tab = torch.bincount(vi * labels.size + yi, minlength=vals.size * labels.size).to(torch.float64)
            comm.allreduce_(tab)
            obs = tab.cpu().numpy().reshape(vals.size, labels.size)
            n = obs.sum()
            exp = np.outer(obs.sum(1), obs.sum(0)) / max(n, 1.0)
            with np.errstate(divide="ignore", invalid="ignore"):
                s = float(np.where(exp > 0, (obs - exp) ** 2 / exp, 0.0).sum())
            k = (vals.size - 1) * (labels.size - 1)
            stat.append(s)
            dof.append(int(k))
            pv.append(float(chi2.sf(s, k)) if k > 0 else 1.0)
        if flatten:
            raise NotImplementedError("flatten=True is not supported; use the vector form")
        fields = [T.StructField("pValues", T.VectorUDT(), False),
                  T.StructField("degreesOfFreedom", T.ArrayType(T.IntegerType()), False),
                  T.StructField("statistics", T.VectorUDT(), False)]
        return _one_row(dataset, fields, [DenseVector(pv), dof, DenseVector(stat)])
