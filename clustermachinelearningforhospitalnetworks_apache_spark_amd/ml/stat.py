"""pyspark.ml.stat: Correlation (pearson / spearman), ChiSquareTest, ANOVATest, FValueTest,
KolmogorovSmirnovTest and Summarizer.

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

import math
from typing import List

import numpy as np
import torch

from ..ops import glm_ops
from ..sql import types as T
from ..sql.column import AggExpr, Column, ColumnData
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


def _labels_index(comm, y: torch.Tensor):
    labels = np.unique(comm.allgather_cat(torch.unique(y)).cpu().numpy())
    lab_t = torch.as_tensor(labels, device=y.device)
    return labels, torch.searchsorted(lab_t, y.contiguous())


def _chi2_arrays(dataset, featuresCol: str, labelCol: str):
    """(pValues, degreesOfFreedom, statistics) of Pearson's independence test per feature."""
    from scipy.stats import chi2
    x = dataset._feature_matrix(featuresCol).to(torch.float64)
    y = dataset._column_data(labelCol).values.to(torch.float64)
    comm = dataset._comm
    d = x.shape[1]
    labels, yi = _labels_index(comm, y)
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
    return np.asarray(pv), dof, np.asarray(stat)


def _anova_arrays(dataset, featuresCol: str, labelCol: str):
    """One-way ANOVA F-test of every continuous feature against a categorical label. The per-class
    sums and sums of squares are two [k, n] x [n, d] products on the device plus one all-reduce."""
    from scipy.stats import f as fdist
    x = dataset._feature_matrix(featuresCol).to(torch.float64)
    y = dataset._column_data(labelCol).values.to(torch.float64)
    comm = dataset._comm
    d = x.shape[1]
    labels, yi = _labels_index(comm, y)
    k = labels.size
    Y = torch.nn.functional.one_hot(yi, k).to(torch.float64) if yi.numel() else torch.zeros(
        (0, k), dtype=torch.float64, device=x.device)
    msg = torch.cat([(Y.T @ x).reshape(-1), (Y.T @ (x * x)).reshape(-1), Y.sum(0)])
    comm.allreduce_(msg)
    o = msg.cpu().numpy()
    S, Q, nc = o[:k * d].reshape(k, d), o[k * d:2 * k * d].reshape(k, d), o[2 * k * d:]
    N = nc.sum()
    tot = S.sum(0)
    ss_tot = Q.sum(0) - tot * tot / N
    ss_b = (S * S / np.where(nc > 0, nc, 1.0)[:, None]).sum(0) - tot * tot / N
    ss_w = ss_tot - ss_b
    dfb, dfw = k - 1, N - k
    with np.errstate(divide="ignore", invalid="ignore"):
        F = (ss_b / dfb) / (ss_w / dfw)
    pv = np.array([float(fdist.sf(v, dfb, dfw)) if np.isfinite(v) else (0.0 if v == np.inf else np.nan)
                   for v in F])
    return pv, [int(dfb + dfw)] * d, F


def _fvalue_arrays(dataset, featuresCol: str, labelCol: str):
    """F-value regression test (squared Pearson correlation of every feature with a continuous
    label, F = r^2 / (1 - r^2) * (n - 2)); sums from one device pass + one all-reduce."""
    from scipy.stats import f as fdist
    x = dataset._feature_matrix(featuresCol).to(torch.float64)
    y = dataset._column_data(labelCol).values.to(torch.float64)
    comm = dataset._comm
    d = x.shape[1]
    msg = torch.cat([x.sum(0), (x * x).sum(0), (x * y[:, None]).sum(0),
                     torch.stack([y.sum(), (y * y).sum(), torch.tensor(float(y.numel()), dtype=torch.float64,
                                                                       device=y.device)])])
    comm.allreduce_(msg)
    o = msg.cpu().numpy()
    sx, sxx, sxy = o[:d], o[d:2 * d], o[2 * d:3 * d]
    sy, syy, N = o[3 * d:]
    cov = sxy - sx * sy / N
    vx = sxx - sx * sx / N
    vy = syy - sy * sy / N
    with np.errstate(divide="ignore", invalid="ignore"):
        r2 = cov * cov / (vx * vy)
        F = r2 / (1.0 - r2) * (N - 2)
    pv = np.array([float(fdist.sf(v, 1, N - 2)) if np.isfinite(v) else (0.0 if v == np.inf else np.nan)
                   for v in F])
    return pv, [int(N - 2)] * d, F


def _moments(dataset, x: torch.Tensor):
    """(N, mean, unbiased variance) per feature over all ranks: K7 shifted moments per rank, merged
    around rank 0's shift with one all-reduce."""
    d = x.shape[1]
    comm = dataset._comm
    n, s1, s2, shift = glm_ops.moments(x, d)
    common = comm.broadcast_object(shift.cpu().numpy() if n else None, 0)
    common_t = torch.as_tensor(common if common is not None else np.zeros(d), dtype=torch.float64, device=x.device)
    delta = shift - common_t
    t1 = s1 + n * delta
    t2 = s2 + 2 * delta * s1 + n * delta * delta
    msg = torch.cat([torch.tensor([float(n)], dtype=torch.float64, device=x.device), t1, t2])
    comm.allreduce_(msg)
    N = msg[0].item()
    T1, T2 = msg[1:1 + d], msg[1 + d:]
    mean = common_t + T1 / max(N, 1)
    m2 = torch.clamp(T2 - T1 * T1 / max(N, 1), min=0.0)
    var = m2 / (N - 1) if N > 1 else torch.zeros_like(m2)
    return N, mean.cpu().numpy(), var.cpu().numpy()


def _test_frame(dataset, pv, dof, stat, stat_name: str):
    fields = [T.StructField("pValues", T.VectorUDT(), False),
              T.StructField("degreesOfFreedom", T.ArrayType(T.LongType() if stat_name == "fValues"
                                                            else T.IntegerType()), False),
              T.StructField(stat_name, T.VectorUDT(), False)]
    return _one_row(dataset, fields, [DenseVector(pv), list(dof), DenseVector(stat)])


def _flat_frame(dataset, pv, dof, stat, stat_name: str):
    from ..sql.builder import rows_round_robin
    schema = T.StructType([T.StructField("featureIndex", T.IntegerType(), False),
                           T.StructField("pValue", T.DoubleType(), False),
                           T.StructField("degreesOfFreedom", T.LongType() if stat_name == "fValue"
                                         else T.IntegerType(), False),
                           T.StructField(stat_name, T.DoubleType(), False)])
    rows = [[j, float(pv[j]), int(dof[j]), float(stat[j])] for j in range(len(pv))]
    return rows_round_robin(dataset._session, schema, rows)


class ChiSquareTest:
    @staticmethod
    def test(dataset, featuresCol: str, labelCol: str, flatten: bool = False):
        """Pearson's independence test of every (categorical) feature against the label."""
        pv, dof, stat = _chi2_arrays(dataset, featuresCol, labelCol)
        if flatten:
            return _flat_frame(dataset, pv, dof, stat, "statistic")
        return _test_frame(dataset, pv, dof, stat, "statistics")


class ANOVATest:
    """pyspark.ml.stat.ANOVATest: F-test of continuous features against a categorical label."""

    @staticmethod
    def test(dataset, featuresCol: str, labelCol: str, flatten: bool = False):
        pv, dof, F = _anova_arrays(dataset, featuresCol, labelCol)
        if flatten:
            return _flat_frame(dataset, pv, dof, F, "fValue")
        return _test_frame(dataset, pv, dof, F, "fValues")


class FValueTest:
    """pyspark.ml.stat.FValueTest: F-value regression test of continuous features and label."""

    @staticmethod
    def test(dataset, featuresCol: str, labelCol: str, flatten: bool = False):
        pv, dof, F = _fvalue_arrays(dataset, featuresCol, labelCol)
        if flatten:
            return _flat_frame(dataset, pv, dof, F, "fValue")
        return _test_frame(dataset, pv, dof, F, "fValues")


class KolmogorovSmirnovTest:
    """One-sample, two-sided Kolmogorov-Smirnov test of a numeric column against a continuous
    distribution (``distName='norm'``, params mean and standard deviation, default 0 and 1).
    The sample is gathered and sorted on the device; the p-value is the exact one-sample
    distribution of D_n (scipy ``kstwo``)."""

    @staticmethod
    def test(dataset, sampleCol: str, distName: str = "norm", *params):
        from scipy.stats import kstwo
        if distName != "norm":
            raise ValueError(f"KolmogorovSmirnovTest: unsupported distribution {distName!r} (only 'norm')")
        p = list(params) + [0.0, 1.0][len(params):]
        mu, sigma = p[0], p[1]
        cd = dataset._column_data(sampleCol)
        v = cd.values.to(torch.float64)
        if cd.valid is not None:
            v = v[torch.as_tensor(cd.valid, device=v.device)]
        allv = torch.sort(dataset._comm.allgather_cat(v.contiguous())).values
        n = allv.numel()
        if n == 0:
            raise ValueError("KolmogorovSmirnovTest: empty sample")
        cdf = 0.5 * (1.0 + torch.erf((allv - float(mu)) / (float(sigma) * math.sqrt(2.0))))
        i = torch.arange(1, n + 1, dtype=torch.float64, device=allv.device)
        D = float(torch.maximum((i / n - cdf).max(), (cdf - (i - 1) / n).max()))
        pv = float(kstwo.sf(D, n))
        fields = [T.StructField("pValue", T.DoubleType(), False), T.StructField("statistic", T.DoubleType(), False)]
        return _one_row(dataset, fields, [pv, D])


# ------------------------------------------------------------------------------------------- Summarizer

_VEC_METRICS = ("mean", "sum", "variance", "std", "numNonZeros", "max", "min", "normL2", "normL1")
_ALL_METRICS = _VEC_METRICS + ("count", "weightSum")


def _metric_type(m: str) -> T.DataType:
    if m == "count":
        return T.LongType()
    if m == "weightSum":
        return T.DoubleType()
    return T.VectorUDT()


class _VectorSummary(AggExpr):
    """Aggregate of Summarizer metrics over a vector column (optionally weighted). Partials are
    device reductions over each group's rows: weighted mean and M2 (merged across ranks with
    Chan's weighted update), non-zero counts, max/min and L1 / squared-L2 sums."""
    custom = True

    def __init__(self, metrics: List[str], child, weight=None, single: bool = False):
        super().__init__("summary", child)
        bad = [m for m in metrics if m not in _ALL_METRICS]
        if bad or not metrics:
            raise ValueError(f"Summarizer: unknown metrics {bad}; choose from {list(_ALL_METRICS)}")
        self.metrics, self.weight, self.single = list(metrics), weight, single

    def refs(self):
        return self.child.refs() + (self.weight.refs() if self.weight is not None else [])

    def __str__(self):
        if self.single:
            return f"{self.metrics[0]}({self.child})"
        return f"aggregate_metrics({self.child}, {self.weight if self.weight is not None else 1.0})"

    def prepare(self, df):
        x = self.child.eval(df)
        if not isinstance(x.dtype, T.VectorUDT):
            raise TypeError(f"Summarizer: {self.child} is not a vector column")
        w = self.weight.eval(df).values.to(torch.float64) if self.weight is not None else None
        return x.values.to(torch.float64), w

    def partial(self, vals, rows):
        x, w = vals
        d = x.shape[1]
        idx = torch.as_tensor(rows, dtype=torch.int64, device=x.device)
        xs = x[idx]
        ws = w[idx] if w is not None else torch.ones(xs.shape[0], dtype=torch.float64, device=x.device)
        if bool((ws < 0).any()):
            raise ValueError("Summarizer: negative weight")
        keep = ws > 0
        xs, ws = xs[keep], ws[keep]
        if xs.shape[0] == 0:
            return ("vsum", 0, 0.0, 0.0) + tuple(np.zeros(d) for _ in range(2)) + (np.zeros(d),) + (
                np.full(d, -np.inf), np.full(d, np.inf), np.zeros(d), np.zeros(d))
        W = ws.sum()
        mean = (ws[:, None] * xs).sum(0) / W
        dx = xs - mean
        out = [(ws[:, None] * dx * dx).sum(0), (xs != 0).sum(0).to(torch.float64), xs.amax(0), xs.amin(0),
               (ws[:, None] * xs.abs()).sum(0), (ws[:, None] * xs * xs).sum(0)]
        return ("vsum", int(xs.shape[0]), float(W), float((ws * ws).sum()), mean.cpu().numpy()) + tuple(
            t.cpu().numpy() for t in out)

    def merge(self, parts):
        parts = [p for p in parts if p[1] > 0]
        if not parts:
            return None
        cnt, W, W2, mean, m2, nnz, mx, mn, l1, l2 = parts[0][1:]
        mean, m2, nnz, mx, mn, l1, l2 = (a.copy() for a in (mean, m2, nnz, mx, mn, l1, l2))
        for p in parts[1:]:
            cb, Wb, W2b, mb, m2b, nnzb, mxb, mnb, l1b, l2b = p[1:]
            delta = mb - mean
            tot = W + Wb
            mean = mean + delta * (Wb / tot)
            m2 = m2 + m2b + delta * delta * (W * Wb / tot)
            cnt, W, W2 = cnt + cb, tot, W2 + W2b
            nnz, l1, l2 = nnz + nnzb, l1 + l1b, l2 + l2b
            mx, mn = np.maximum(mx, mxb), np.minimum(mn, mnb)
        denom = W - W2 / W
        var = np.clip(m2 / denom, 0.0, None) if denom > 0 else np.zeros_like(m2)
        vals = {"mean": mean, "sum": mean * W, "variance": var, "std": np.sqrt(var), "numNonZeros": nnz,
                "max": mx, "min": mn, "normL2": np.sqrt(l2), "normL1": l1, "count": int(cnt), "weightSum": float(W)}
        out = {m: (DenseVector(vals[m]) if m in _VEC_METRICS else vals[m]) for m in self.metrics}
        if self.single:
            return out[self.metrics[0]]
        from ..sql.types import Row
        return Row(**out)

    def result_type(self):
        if self.single:
            return _metric_type(self.metrics[0])
        return T.StructType([T.StructField(m, _metric_type(m), True) for m in self.metrics])


def _cexpr(c):
    from ..sql.column import ColRef
    if c is None:
        return None
    if isinstance(c, str):
        return ColRef(c)
    return c._expr if isinstance(c, Column) else c


class SummaryBuilder:
    def __init__(self, metrics: List[str]):
        self._metrics = list(metrics)

    def summary(self, featuresCol, weightCol=None) -> "Column":
        return Column(_VectorSummary(self._metrics, _cexpr(featuresCol), _cexpr(weightCol)))


class Summarizer:
    """pyspark.ml.stat.Summarizer: vector-column statistics as aggregate Columns, usable in
    ``df.select(...)`` and ``groupBy(...).agg(...)``."""

    @staticmethod
    def metrics(*metrics) -> SummaryBuilder:
        return SummaryBuilder(list(metrics))

    @staticmethod
    def _one(metric, col, weightCol=None):
        return Column(_VectorSummary([metric], _cexpr(col), _cexpr(weightCol), single=True))

    @staticmethod
    def mean(col, weightCol=None): return Summarizer._one("mean", col, weightCol)
    @staticmethod
    def sum(col, weightCol=None): return Summarizer._one("sum", col, weightCol)
    @staticmethod
    def variance(col, weightCol=None): return Summarizer._one("variance", col, weightCol)
    @staticmethod
    def std(col, weightCol=None): return Summarizer._one("std", col, weightCol)
    @staticmethod
    def count(col, weightCol=None): return Summarizer._one("count", col, weightCol)
    @staticmethod
    def numNonZeros(col, weightCol=None): return Summarizer._one("numNonZeros", col, weightCol)
    @staticmethod
    def max(col, weightCol=None): return Summarizer._one("max", col, weightCol)
    @staticmethod
    def min(col, weightCol=None): return Summarizer._one("min", col, weightCol)
    @staticmethod
    def normL1(col, weightCol=None): return Summarizer._one("normL1", col, weightCol)
    @staticmethod
    def normL2(col, weightCol=None): return Summarizer._one("normL2", col, weightCol)
    @staticmethod
    def weightSum(col, weightCol=None): return Summarizer._one("weightSum", col, weightCol)
