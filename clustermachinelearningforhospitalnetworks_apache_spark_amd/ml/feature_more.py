"""The rest of pyspark.ml.feature for numeric hospital tables: MaxAbsScaler, RobustScaler,
ElementwiseProduct, PolynomialExpansion, Interaction, VectorSlicer, VectorIndexer,
SQLTransformer, and the feature selectors (VarianceThresholdSelector, ChiSqSelector,
UnivariateFeatureSelector).

The reference assembles raw numeric columns straight into a vector (ref.py:134-136) and
trains on it; these are the MLlib stages that sit between that assembler and a model.
Design, MI355X-first: every transform is a handful of whole-shard device tensor ops on the
[n, d] feature matrix (one gather, one multiply, one ``searchsorted``), fits reduce to one
all-reduce of per-feature statistics (max |x|, moments, contingency tables) or — for the
exact order statistics of RobustScaler — one all-gather and a device column sort.
Persistence writes Spark's data layouts (``maxAbs``; ``range``/``median``;
``selectedFeatures``; ``numFeatures``/``categoryMaps``).
"""
from __future__ import annotations

import math
from typing import Dict, List, Optional, Tuple

import numpy as np
import torch

from ..sql import types as T
from ..sql.column import ColumnData
from . import util as U
from .base import Estimator, Model, Transformer
from .colutil import _auto_output, _replace_col
from .linalg import DenseVector
from .param import NO_DEFAULT


def _vector_meta(names: List[str], categorical: Optional[Dict[int, int]] = None) -> Dict:
    """Spark's ML attribute-group metadata (``ml_attr``) for a vector column."""
    categorical = categorical or {}
    numeric = [{"idx": i, "name": n} for i, n in enumerate(names) if i not in categorical]
    nominal = [{"idx": i, "name": n, "ord": False, "vals": [str(v) for v in range(categorical[i])]}
               for i, n in enumerate(names) if i in categorical]
    attrs = {}
    if numeric:
        attrs["numeric"] = numeric
    if nominal:
        attrs["nominal"] = nominal
    return {"ml_attr": {"attrs": attrs, "num_attrs": len(names)}}


def vector_attr_names(df, col: str) -> Optional[List[str]]:
    """Feature names of a vector column from its ``ml_attr`` metadata (None when absent)."""
    md = df.schema[col].metadata.get("ml_attr") if col in df.columns else None
    if not md:
        return None
    n = md.get("num_attrs", 0)
    names = [f"{col}_{i}" for i in range(n)]
    for group in md.get("attrs", {}).values():
        for a in group:
            if "name" in a:
                names[a["idx"]] = a["name"]
    return names


def _set_vector(df, name: str, x: torch.Tensor, names: Optional[List[str]] = None, categorical=None):
    out = _replace_col(df, name, ColumnData(x.contiguous(), None, T.VectorUDT()))
    if names is not None:
        f = out.schema[name]
        f.metadata = _vector_meta(names, categorical)
    return out


def _vec_data_save(model, path: str, cols: Dict[str, np.ndarray]) -> None:
    import pyarrow as pa
    U.write_metadata(model, path)
    U.write_parquet(path, "data", pa.Table.from_pylist(
        [{k: U.vector_struct(v) for k, v in cols.items()}],
        schema=pa.schema([(k, U.vector_arrow_type()) for k in cols])))


def _vec_data_load(path: str, keys: List[str]) -> List[np.ndarray]:
    row = U.read_parquet(path, "data").to_pylist()[0]
    return [U.vector_from_struct(row[k]) for k in keys]


# ------------------------------------------------------------------------------------------ scalers

class MaxAbsScaler(Estimator):
    """Scales each feature into [-1, 1] by its maximum absolute value (no shift, keeps sparsity);
    all-zero features stay zero (Spark's MaxAbsScaler)."""
    _params = {
        "inputCol": (NO_DEFAULT, "input column name", str),
        "outputCol": ("__auto__", "output column name", str),
    }

    def __init__(self, inputCol=None, outputCol=None):
        super().__init__(inputCol=inputCol, outputCol=outputCol)
        _auto_output(self)

    def _fit(self, df):
        x = df._feature_matrix(self.getInputCol())
        d = x.shape[1]
        m = x.abs().amax(0).to(torch.float64) if x.shape[0] else torch.zeros(d, dtype=torch.float64,
                                                                             device=x.device)
        m = m.contiguous()
        df._comm.allreduce_(m, "max")
        model = MaxAbsScalerModel(m.cpu().numpy())
        self._copyValues(model)
        return model


class MaxAbsScalerModel(Model):
    _params = MaxAbsScaler._params

    def __init__(self, maxAbs=None):
        super().__init__()
        self._max_abs = np.asarray(maxAbs if maxAbs is not None else [], dtype=np.float64)

    @property
    def maxAbs(self) -> DenseVector:
        return DenseVector(self._max_abs)

    def _transform(self, df):
        x = df._feature_matrix(self.getInputCol())
        div = np.where(self._max_abs == 0, 1.0, self._max_abs)
        y = x.to(torch.float64) / torch.as_tensor(div, device=x.device)
        return _replace_col(df, self.getOutputCol(), ColumnData(y.to(x.dtype), None, T.VectorUDT()))

    def _save_impl(self, path):
        _vec_data_save(self, path, {"maxAbs": self._max_abs})

    @classmethod
    def _load_impl(cls, path, md):
        m = cls(*_vec_data_load(path, ["maxAbs"]))
        U.apply_params(m, md)
        return m


def _exact_quantiles(df, x: torch.Tensor, probs: List[float]) -> np.ndarray:
    """[len(probs), d] exact order statistics per column over all ranks: the smallest value whose
    rank reaches ceil(p * n) (the limit of Spark's approxQuantile as relativeError -> 0). NaNs are
    ignored per column."""
    allx = df._comm.allgather_cat(x.to(torch.float64).contiguous())
    d = allx.shape[1] if allx.dim() == 2 else x.shape[1]
    out = np.full((len(probs), d), np.nan)
    if allx.numel() == 0:
        return out
    srt = torch.sort(allx, dim=0).values  # NaN sorts last
    nvalid = (~torch.isnan(allx)).sum(0).cpu().numpy()
    s = srt.cpu().numpy()
    for j in range(d):
        n = int(nvalid[j])
        if n == 0:
            continue
        for i, p in enumerate(probs):
            out[i, j] = s[min(max(int(math.ceil(p * n)) - 1, 0), n - 1), j]
    return out


class RobustScaler(Estimator):
    """Removes the median and scales by the [lower, upper] quantile range (Spark's RobustScaler:
    defaults lower=0.25, upper=0.75, withCentering=False, withScaling=True; a zero range maps the
    feature to 0)."""
    _params = {
        "inputCol": (NO_DEFAULT, "input column name", str),
        "outputCol": ("__auto__", "output column name", str),
        "lower": (0.25, "lower quantile to calculate quantile range", float),
        "upper": (0.75, "upper quantile to calculate quantile range", float),
        "withCentering": (False, "whether to center data with median", bool),
        "withScaling": (True, "whether to scale the data to quantile range", bool),
        "relativeError": (0.001, "the relative target precision for the approximate quantile algorithm", float),
    }

    def __init__(self, lower=None, upper=None, withCentering=None, withScaling=None, inputCol=None,
                 outputCol=None, relativeError=None):
        super().__init__(lower=lower, upper=upper, withCentering=withCentering, withScaling=withScaling,
                         inputCol=inputCol, outputCol=outputCol, relativeError=relativeError)
        _auto_output(self)

    def _fit(self, df):
        lo, hi = self.getLower(), self.getUpper()
        if not 0.0 <= lo < hi <= 1.0:
            raise ValueError(f"RobustScaler: need 0 <= lower < upper <= 1, got {lo}, {hi}")
        x = df._feature_matrix(self.getInputCol())
        q = _exact_quantiles(df, x, [lo, 0.5, hi])
        model = RobustScalerModel(q[2] - q[0], q[1])
        self._copyValues(model)
        return model


class RobustScalerModel(Model):
    _params = RobustScaler._params

    def __init__(self, range=None, median=None):  # noqa: A002 - Spark's field name
        super().__init__()
        self._range = np.asarray(range if range is not None else [], dtype=np.float64)
        self._median = np.asarray(median if median is not None else [], dtype=np.float64)

    @property
    def range(self) -> DenseVector:
        return DenseVector(self._range)

    @property
    def median(self) -> DenseVector:
        return DenseVector(self._median)

    def _transform(self, df):
        x = df._feature_matrix(self.getInputCol())
        y = x.to(torch.float64)
        dev = x.device
        if self.getWithCentering():
            y = y - torch.as_tensor(self._median, device=dev)
        if self.getWithScaling():
            scale = np.where(self._range == 0, 0.0, 1.0 / np.where(self._range == 0, 1.0, self._range))
            y = y * torch.as_tensor(scale, device=dev)
        return _replace_col(df, self.getOutputCol(), ColumnData(y.to(x.dtype).contiguous(), None, T.VectorUDT()))

    def _save_impl(self, path):
        _vec_data_save(self, path, {"range": self._range, "median": self._median})

    @classmethod
    def _load_impl(cls, path, md):
        m = cls(*_vec_data_load(path, ["range", "median"]))
        U.apply_params(m, md)
        return m


# ------------------------------------------------------------------------------- vector transforms

class ElementwiseProduct(Transformer):
    """Hadamard product of every vector with ``scalingVec``."""
    _params = {
        "scalingVec": (NO_DEFAULT, "vector for hadamard product", None),
        "inputCol": (NO_DEFAULT, "input column name", str),
        "outputCol": ("__auto__", "output column name", str),
    }

    def __init__(self, scalingVec=None, inputCol=None, outputCol=None):
        super().__init__(scalingVec=scalingVec, inputCol=inputCol, outputCol=outputCol)
        _auto_output(self)

    def _transform(self, df):
        x = df._feature_matrix(self.getInputCol())
        v = self.getScalingVec()
        s = np.asarray(v.toArray() if hasattr(v, "toArray") else v, dtype=np.float64)
        if s.size != x.shape[1]:
            raise ValueError(f"ElementwiseProduct: scalingVec has size {s.size}, vectors have {x.shape[1]}")
        y = x.to(torch.float64) * torch.as_tensor(s, device=x.device)
        return _replace_col(df, self.getOutputCol(), ColumnData(y.contiguous(), None, T.VectorUDT()))


def poly_terms(n: int, degree: int) -> List[Tuple[Tuple[int, int], ...]]:
    """Monomials of PolynomialExpansion in Spark's output order (the order its recursive dense
    expansion writes them: the last feature's exponent is the outermost loop, lower exponents
    first), without the constant term. Each monomial is ((feature, exponent), ...)."""
    terms: List[Tuple[Tuple[int, int], ...]] = []

    def rec(last: int, deg: int, mono: Tuple[Tuple[int, int], ...]) -> None:
        if deg == 0 or last < 0:
            terms.append(mono)
            return
        for e in range(deg + 1):
            rec(last - 1, deg - e, mono + (((last, e),) if e else ()))

    rec(n - 1, degree, ())
    return terms[1:]


class PolynomialExpansion(Transformer):
    """Expands a vector into all monomials up to ``degree`` (Spark's term order). On the device the
    monomials are gathered products: each term is the product of ``degree`` gathered columns of
    [x, 1]."""
    _params = {
        "degree": (2, "the polynomial degree to expand (>= 1)", int),
        "inputCol": (NO_DEFAULT, "input column name", str),
        "outputCol": ("__auto__", "output column name", str),
    }

    def __init__(self, degree=None, inputCol=None, outputCol=None):
        super().__init__(degree=degree, inputCol=inputCol, outputCol=outputCol)
        _auto_output(self)

    def _transform(self, df):
        deg = self.getDegree()
        if deg < 1:
            raise ValueError("PolynomialExpansion: degree must be >= 1")
        x = df._feature_matrix(self.getInputCol()).to(torch.float64)
        n, d = x.shape
        terms = poly_terms(d, deg)
        idx = np.full((len(terms), deg), d, dtype=np.int64)  # column d of xp is the constant 1
        for t, mono in enumerate(terms):
            s = 0
            for f, e in mono:
                idx[t, s:s + e] = f
                s += e
        xp = torch.cat([x, torch.ones((n, 1), dtype=x.dtype, device=x.device)], 1)
        it = torch.as_tensor(idx, device=x.device)
        y = xp[:, it[:, 0]]
        for s in range(1, deg):
            y = y * xp[:, it[:, s]]
        return _replace_col(df, self.getOutputCol(), ColumnData(y.contiguous(), None, T.VectorUDT()))


class Interaction(Transformer):
    """Crosses numeric and vector columns: the output holds the product of one entry from every
    input, flattened with the first column most significant (Spark's Interaction over columns
    without nominal attributes)."""
    _params = {
        "inputCols": (NO_DEFAULT, "input column names", "liststr"),
        "outputCol": ("__auto__", "output column name", str),
    }

    def __init__(self, inputCols=None, outputCol=None):
        super().__init__(inputCols=inputCols, outputCol=outputCol)
        _auto_output(self)

    def _transform(self, df):
        cols = self.getInputCols()
        if not cols:
            raise ValueError("Interaction: inputCols is empty")
        out = None
        for c in cols:
            cd = df._column_data(c)
            if cd.is_host:
                raise TypeError(f"Interaction: column {c!r} is not numeric")
            v = cd.values.to(torch.float64)
            v = v.reshape(v.shape[0], -1)
            out = v if out is None else (out[:, :, None] * v[:, None, :]).reshape(v.shape[0], -1)
        return _replace_col(df, self.getOutputCol(), ColumnData(out.contiguous(), None, T.VectorUDT()))


class VectorSlicer(Transformer):
    """Sub-vector of selected features, by index and/or by attribute name (names need the
    ``ml_attr`` metadata that VectorAssembler writes); index selections come first."""
    _params = {
        "inputCol": (NO_DEFAULT, "input column name", str),
        "outputCol": ("__auto__", "output column name", str),
        "indices": ([], "an array of indices to select features from a vector column", None),
        "names": ([], "an array of feature names to select features from a vector column", None),
    }

    def __init__(self, inputCol=None, outputCol=None, indices=None, names=None):
        super().__init__(inputCol=inputCol, outputCol=outputCol, indices=indices, names=names)
        _auto_output(self)

    def _transform(self, df):
        x = df._feature_matrix(self.getInputCol())
        idx = [int(i) for i in self.getIndices()]
        names = list(self.getNames())
        attr = vector_attr_names(df, self.getInputCol())
        if names:
            if attr is None:
                raise ValueError("VectorSlicer: selecting by name needs feature names in the column metadata")
            for nm in names:
                if nm not in attr:
                    raise ValueError(f"VectorSlicer: no feature named {nm!r}")
                idx.append(attr.index(nm))
        if not idx:
            raise ValueError("VectorSlicer: select at least one feature")
        if len(set(idx)) != len(idx) or min(idx) < 0 or max(idx) >= x.shape[1]:
            raise ValueError(f"VectorSlicer: indices {idx} must be distinct and in [0, {x.shape[1]})")
        y = x[:, torch.as_tensor(idx, device=x.device)]
        out_names = [attr[i] for i in idx] if attr is not None else None
        return _set_vector(df, self.getOutputCol(), y, out_names)


# ----------------------------------------------------------------------------------- VectorIndexer

class VectorIndexer(Estimator):
    """Marks features with at most ``maxCategories`` distinct values as categorical and re-codes their
    values to category indices: 0.0 (when present) is category 0, the other values follow in
    ascending order (Spark's VectorIndexer). Distinct values are found per rank with a device
    ``unique`` per column and merged once across ranks."""
    _params = {
        "maxCategories": (20, "threshold for the number of values a categorical feature can take (>= 2)", int),
        "inputCol": (NO_DEFAULT, "input column name", str),
        "outputCol": ("__auto__", "output column name", str),
        "handleInvalid": ("error", "how to handle invalid data (unseen labels or NULL values): "
                                   "'error', 'skip' or 'keep'", str),
    }

    def __init__(self, maxCategories=None, inputCol=None, outputCol=None, handleInvalid=None):
        super().__init__(maxCategories=maxCategories, inputCol=inputCol, outputCol=outputCol,
                         handleInvalid=handleInvalid)
        _auto_output(self)

    def _fit(self, df):
        mc = self.getMaxCategories()
        if mc < 2:
            raise ValueError("VectorIndexer: maxCategories must be >= 2")
        x = df._feature_matrix(self.getInputCol()).to(torch.float64)
        d = x.shape[1]
        local = []
        for j in range(d):
            u = torch.unique(x[:, j]) if x.shape[0] else x[:0, j]
            local.append(None if u.numel() > mc else u.cpu().numpy())
        merged: List[Optional[set]] = [set() for _ in range(d)]
        for part in df._comm.allgather_object(local):
            for j, u in enumerate(part):
                if merged[j] is None:
                    continue
                if u is None:
                    merged[j] = None
                else:
                    merged[j].update(float(v) for v in u)
                    if len(merged[j]) > mc:
                        merged[j] = None
        maps = {}
        for j, s in enumerate(merged):
            if s is None:
                continue
            vals = sorted(v for v in s if v != 0.0)
            if 0.0 in s:
                vals = [0.0] + vals
            maps[j] = {v: i for i, v in enumerate(vals)}
        model = VectorIndexerModel(d, maps)
        self._copyValues(model)
        return model


class VectorIndexerModel(Model):
    _params = VectorIndexer._params

    def __init__(self, numFeatures: int = 0, categoryMaps: Optional[Dict[int, Dict[float, int]]] = None):
        super().__init__()
        self.numFeatures = int(numFeatures)
        self.categoryMaps = {int(k): {float(a): int(b) for a, b in v.items()}
                             for k, v in (categoryMaps or {}).items()}

    def _transform(self, df):
        x = df._feature_matrix(self.getInputCol())
        if x.shape[1] != self.numFeatures:
            raise ValueError(f"VectorIndexer: expected {self.numFeatures} features, got {x.shape[1]}")
        y = x.to(torch.float64).clone()
        bad = torch.zeros(x.shape[0], dtype=torch.bool, device=x.device)
        mode = self.getHandleInvalid()
        for j, cmap in sorted(self.categoryMaps.items()):
            keys = np.array(sorted(cmap), dtype=np.float64)
            codes = torch.as_tensor(np.array([cmap[k] for k in keys], dtype=np.float64), device=x.device)
            kt = torch.as_tensor(keys, device=x.device)
            col = y[:, j].contiguous()
            pos = torch.searchsorted(kt, col).clamp(max=max(len(keys) - 1, 0))
            hit = kt[pos] == col if len(keys) else torch.zeros_like(col, dtype=torch.bool)
            miss = ~hit
            if bool(miss.any()):
                if mode == "error":
                    v = float(col[miss][0])
                    raise ValueError(f"VectorIndexer: unseen value {v} of categorical feature {j}; "
                                     "set handleInvalid='skip' or 'keep'")
                bad |= miss
            y[:, j] = torch.where(hit, codes[pos] if len(keys) else col, torch.full_like(col, float(len(keys))))
        names = [f"{self.getInputCol()}_{i}" for i in range(self.numFeatures)]
        cat = {j: len(m) + (1 if mode == "keep" else 0) for j, m in self.categoryMaps.items()}
        out = _set_vector(df, self.getOutputCol(), y, names, cat)
        if mode == "skip" and bool(bad.any()):
            out = out._mask_rows(~bad)
        return out

    def _save_impl(self, path):
        import pyarrow as pa
        U.write_metadata(self, path)
        maps = [(int(k), [(float(a), int(b)) for a, b in sorted(v.items())]) for k, v in sorted(self.categoryMaps.items())]
        typ = pa.map_(pa.int32(), pa.map_(pa.float64(), pa.int32()))
        U.write_parquet(path, "data", pa.Table.from_pylist(
            [{"numFeatures": self.numFeatures, "categoryMaps": maps}],
            schema=pa.schema([pa.field("numFeatures", pa.int32(), nullable=False), ("categoryMaps", typ)])))

    @classmethod
    def _load_impl(cls, path, md):
        row = U.read_parquet(path, "data").to_pylist()[0]
        maps = {int(k): {float(a): int(b) for a, b in v} for k, v in row["categoryMaps"]}
        m = cls(row["numFeatures"], maps)
        U.apply_params(m, md)
        return m


# ---------------------------------------------------------------------------------- SQLTransformer

class SQLTransformer(Transformer):
    """Runs a SQL statement over the input, which the statement names ``__THIS__``."""
    _params = {"statement": (NO_DEFAULT, "SQL statement", str)}

    def __init__(self, statement=None):
        super().__init__(statement=statement)

    def _transform(self, df):
        view = "__sqltrans_" + self.uid.replace("-", "_")
        df.createOrReplaceTempView(view)
        try:
            return df._session.sql(self.getStatement().replace("__THIS__", view))
        finally:
            df._session.catalog.dropTempView(view)


# --------------------------------------------------------------------------------------- selectors

def _select(scores: np.ndarray, pvals: np.ndarray, mode: str, thr: float, what: str) -> List[int]:
    """Feature indices picked by Spark's selector modes from per-feature p-values (``scores`` is
    the test statistic, used for VarianceThreshold only through ``what``)."""
    d = pvals.size
    order = sorted(range(d), key=lambda j: (pvals[j], j))
    if mode == "numTopFeatures":
        sel = order[: int(thr)]
    elif mode == "percentile":
        sel = order[: int(d * thr)]
    elif mode == "fpr":
        sel = [j for j in range(d) if pvals[j] < thr]
    elif mode == "fdr":
        # Benjamini-Hochberg: the largest rank i with p_(i) <= thr * i / d, and everything before it
        last = -1
        for i, j in enumerate(order):
            if pvals[j] <= thr * (i + 1) / d:
                last = i
        sel = order[: last + 1]
    elif mode == "fwe":
        sel = [j for j in range(d) if pvals[j] < thr / d]
    else:
        raise ValueError(f"{what}: unknown selection mode {mode!r}")
    return sorted(int(j) for j in sel)


class _SelectorModel(Model):
    """Keeps ``selectedFeatures`` of the features vector (Spark's SelectorModel)."""

    def __init__(self, selectedFeatures: Optional[List[int]] = None):
        super().__init__()
        self._selected = [int(i) for i in (selectedFeatures or [])]

    @property
    def selectedFeatures(self) -> List[int]:
        return list(self._selected)

    def _transform(self, df):
        x = df._feature_matrix(self.getFeaturesCol())
        y = x[:, torch.as_tensor(self._selected, dtype=torch.int64, device=x.device)]
        attr = vector_attr_names(df, self.getFeaturesCol())
        return _set_vector(df, self.getOutputCol(), y, [attr[i] for i in self._selected] if attr else None)

    def _save_impl(self, path):
        import pyarrow as pa
        U.write_metadata(self, path)
        U.write_parquet(path, "data", pa.table({"selectedFeatures": pa.array([self._selected],
                                                                             type=pa.list_(pa.int32()))}))

    @classmethod
    def _load_impl(cls, path, md):
        row = U.read_parquet(path, "data").to_pylist()[0]
        m = cls(row["selectedFeatures"])
        U.apply_params(m, md)
        return m


_SEL_COMMON = {
    "featuresCol": ("features", "features column name", str),
    "outputCol": ("__auto__", "output column name", str),
}


class VarianceThresholdSelector(Estimator):
    """Drops features whose sample variance is not above ``varianceThreshold`` (default 0: drops
    constant features). Variances from one all-reduce of shifted moments."""
    _params = dict(_SEL_COMMON, varianceThreshold=(0.0, "features with a variance not greater than this "
                                                           "threshold will be removed", float))

    def __init__(self, featuresCol=None, outputCol=None, varianceThreshold=None):
        super().__init__(featuresCol=featuresCol, outputCol=outputCol, varianceThreshold=varianceThreshold)
        _auto_output(self)

    def _fit(self, df):
        from .stat import _moments
        n, mean, var = _moments(df, df._feature_matrix(self.getFeaturesCol()))
        sel = [j for j in range(var.size) if var[j] > self.getVarianceThreshold()]
        m = VarianceThresholdSelectorModel(sel)
        self._copyValues(m)
        return m


class VarianceThresholdSelectorModel(_SelectorModel):
    _params = VarianceThresholdSelector._params


_UNI_PARAMS = dict(_SEL_COMMON, **{
    "labelCol": ("label", "label column name", str),
    "featureType": (NO_DEFAULT, "the feature type: 'categorical' or 'continuous'", str),
    "labelType": (NO_DEFAULT, "the label type: 'categorical' or 'continuous'", str),
    "selectionMode": ("numTopFeatures", "numTopFeatures | percentile | fpr | fdr | fwe", str),
    "selectionThreshold": (NO_DEFAULT, "the upper bound of the features that selector will select", float),
})


class UnivariateFeatureSelector(Estimator):
    """Univariate tests per feature vs the label, picked by type: categorical/categorical -> chi-squared,
    continuous/categorical -> ANOVA F, continuous/continuous -> F-value regression test. Default
    thresholds: 50 features (numTopFeatures), 0.1 (percentile), 0.05 (fpr / fdr / fwe)."""
    _params = _UNI_PARAMS

    def __init__(self, featuresCol=None, outputCol=None, labelCol=None, selectionMode=None, featureType=None,
                 labelType=None, selectionThreshold=None):
        super().__init__(featuresCol=featuresCol, outputCol=outputCol, labelCol=labelCol,
                         selectionMode=selectionMode, featureType=featureType, labelType=labelType,
                         selectionThreshold=selectionThreshold)
        _auto_output(self)

    def _threshold(self) -> float:
        if self.isSet("selectionThreshold"):
            return float(self.getOrDefault("selectionThreshold"))
        return {"numTopFeatures": 50, "percentile": 0.1}.get(self.getSelectionMode(), 0.05)

    def _fit(self, df):
        from . import stat
        ft, lt = self.getFeatureType(), self.getLabelType()
        fc, lc = self.getFeaturesCol(), self.getLabelCol()
        if (ft, lt) == ("categorical", "categorical"):
            p, _, s = stat._chi2_arrays(df, fc, lc)
        elif (ft, lt) == ("continuous", "categorical"):
            p, _, s = stat._anova_arrays(df, fc, lc)
        elif (ft, lt) == ("continuous", "continuous"):
            p, _, s = stat._fvalue_arrays(df, fc, lc)
        else:
            raise ValueError(f"UnivariateFeatureSelector: unsupported featureType/labelType {ft}/{lt}")
        m = UnivariateFeatureSelectorModel(_select(s, p, self.getSelectionMode(), self._threshold(),
                                                  "UnivariateFeatureSelector"))
        self._copyValues(m)
        return m


class UnivariateFeatureSelectorModel(_SelectorModel):
    _params = _UNI_PARAMS


_CHISQ_PARAMS = dict(_SEL_COMMON, **{
    "labelCol": ("label", "label column name", str),
    "numTopFeatures": (50, "number of features that selector will select, ordered by ascending p-value", int),
    "percentile": (0.1, "percentile of features that selector will select, ordered by ascending p-value", float),
    "fpr": (0.05, "the highest p-value for features to be kept", float),
    "fdr": (0.05, "the upper bound of the expected false discovery rate", float),
    "fwe": (0.05, "the upper bound of the expected family-wise error rate", float),
    "selectorType": ("numTopFeatures", "numTopFeatures | percentile | fpr | fdr | fwe", str),
})


class ChiSqSelector(Estimator):
    """Chi-squared feature selection on categorical features against a categorical label."""
    _params = _CHISQ_PARAMS

    def __init__(self, numTopFeatures=None, featuresCol=None, outputCol=None, labelCol=None, selectorType=None,
                 percentile=None, fpr=None, fdr=None, fwe=None):
        super().__init__(numTopFeatures=numTopFeatures, featuresCol=featuresCol, outputCol=outputCol,
                         labelCol=labelCol, selectorType=selectorType, percentile=percentile, fpr=fpr, fdr=fdr,
                         fwe=fwe)
        _auto_output(self)

    def _fit(self, df):
        from . import stat
        p, _, s = stat._chi2_arrays(df, self.getFeaturesCol(), self.getLabelCol())
        mode = self.getSelectorType()
        thr = {"numTopFeatures": self.getNumTopFeatures(), "percentile": self.getPercentile(), "fpr": self.getFpr(),
               "fdr": self.getFdr(), "fwe": self.getFwe()}.get(mode)
        m = ChiSqSelectorModel(_select(s, p, mode, thr, "ChiSqSelector"))
        self._copyValues(m)
        return m


class ChiSqSelectorModel(_SelectorModel):
    _params = _CHISQ_PARAMS


# ------------------------------------------------------------------------------------------ RFormula

def parse_formula(formula: str, schema) -> Tuple[str, List[List[str]], bool]:
    """Resolves an R model formula against a schema into (label, terms, hasIntercept).

    Supported: ``y ~ a + b``, ``.`` (every column but the label, in schema order), ``a:b``
    interactions, ``- term`` deletions (applied to the terms included so far, as Spark's
    resolver does), and the intercept switches ``+ 0`` / ``- 1`` (off) and ``+ 1`` / ``- 0`` (on)."""
    import re
    if "~" not in formula:
        raise ValueError(f"RFormula: {formula!r} has no '~'")
    lhs, rhs = formula.split("~", 1)
    label = lhs.strip()
    toks = re.findall(r"[+\-:]|[^\s+\-:]+", rhs)
    if not toks:
        raise ValueError(f"RFormula: {formula!r} has no terms")
    dot = [f.name for f in schema.fields if f.name != label]
    terms: List[List[str]] = []
    has_icpt = True
    sign, cur, expect_atom = "+", [], True
    items = []
    for t in toks + ["+"]:
        if t in "+-" and len(t) == 1:
            if cur:
                items.append((sign, cur))
            sign, cur, expect_atom = t, [], True
        elif t == ":":
            expect_atom = True
        else:
            if not expect_atom:
                raise ValueError(f"RFormula: unexpected token {t!r} in {formula!r}")
            cur.append(t)
            expect_atom = False
    for sign, atoms in items:
        if len(atoms) == 1 and atoms[0] in ("0", "1"):
            on = atoms[0] == "1"
            has_icpt = on if sign == "+" else not on
            continue
        if atoms == ["."]:
            expanded = [[c] for c in dot]
        elif "." in atoms:
            raise NotImplementedError("RFormula: '.' inside an interaction is not supported")
        else:
            for a in atoms:
                if a not in schema.names:
                    raise ValueError(f"RFormula: column {a!r} not found")
            expanded = [list(atoms)]
        if sign == "+":
            for t in expanded:
                if not any(sorted(t) == sorted(u) for u in terms):
                    terms.append(t)
        else:
            terms = [u for u in terms if not any(sorted(t) == sorted(u) for t in expanded)]
    return label, terms, has_icpt


_RFORMULA_PARAMS = {
    "formula": (NO_DEFAULT, "R model formula", str),
    "featuresCol": ("features", "features column name", str),
    "labelCol": ("label", "label column name", str),
    "forceIndexLabel": (False, "force to index the label whether it is numeric or string", bool),
    "handleInvalid": ("error", "how to handle invalid data (unseen or NULL values) in features and label column "
                               "of string type: 'error', 'skip' or 'keep'", str),
    "stringIndexerOrderType": ("frequencyDesc", "how to order categories of a string feature column: "
                                                "frequencyDesc|frequencyAsc|alphabetDesc|alphabetAsc", str),
}


class RFormula(Estimator):
    """R-style model formulas (``los ~ age + ward + age:ward``) over a DataFrame: string terms are
    indexed (``stringIndexerOrderType``) and one-hot encoded with the last category dropped (all
    categories kept for the first string term of a formula without intercept, and inside
    interactions), numeric and vector terms pass through, interactions cross their encoded terms,
    and a string label is indexed (a numeric one is cast to double). The fitted stages run as
    device transforms; the features column carries ``name_value`` attribute names."""
    _params = _RFORMULA_PARAMS

    def __init__(self, formula=None, featuresCol=None, labelCol=None, forceIndexLabel=None, handleInvalid=None,
                 stringIndexerOrderType=None):
        super().__init__(formula=formula, featuresCol=featuresCol, labelCol=labelCol,
                         forceIndexLabel=forceIndexLabel, handleInvalid=handleInvalid,
                         stringIndexerOrderType=stringIndexerOrderType)

    def _fit(self, df):
        from .feature import OneHotEncoder, StringIndexer, VectorAssembler
        label, terms, has_icpt = parse_formula(self.getFormula(), df.schema)
        hi = self.getHandleInvalid()
        tag = self.uid.replace("-", "_")
        stages, tmp = [], []
        cur = df
        labels_of: Dict[str, List[str]] = {}
        indexed: Dict[str, str] = {}

        def is_str(c):
            return isinstance(df.schema[c].dataType, T.StringType)

        for c in dict.fromkeys(a for t in terms for a in t):
            if is_str(c):
                oc = f"{tag}_stridx_{c}"
                m = StringIndexer(inputCol=c, outputCol=oc, handleInvalid=hi,
                                  stringOrderType=self.getStringIndexerOrderType()).fit(cur)
                stages.append(m)
                cur = m.transform(cur)
                tmp.append(oc)
                indexed[c], labels_of[c] = oc, m.labels

        def one_hot(c, drop):
            nonlocal cur
            oc = f"{tag}_onehot{len(tmp)}_{c}"
            m = OneHotEncoder(inputCols=[indexed[c]], outputCols=[oc], dropLast=drop,
                              handleInvalid="keep" if hi == "keep" else "error").fit(cur)
            stages.append(m)
            cur = m.transform(cur)
            tmp.append(oc)
            labs = list(labels_of[c]) + (["__unknown"] if hi == "keep" else [])
            return oc, [f"{c}_{v}" for v in (labs[:-1] if drop else labs)]

        def plain_names(c):
            if isinstance(df.schema[c].dataType, T.VectorUDT):
                names = vector_attr_names(cur, c)
                return names or [f"{c}_{i}" for i in range(cur._feature_matrix(c).shape[1])]
            return [c]

        encoded, names = [], []
        keep_ref = False
        for t in terms:
            if len(t) == 1 and is_str(t[0]):
                drop = True
                if not has_icpt and not keep_ref:
                    drop, keep_ref = False, True
                oc, nm = one_hot(t[0], drop)
                encoded.append(oc)
                names += nm
            elif len(t) == 1:
                encoded.append(t[0])
                names += plain_names(t[0])
            else:
                parts, pnames = [], []
                for c in t:
                    if is_str(c):
                        oc, nm = one_hot(c, False)
                    else:
                        oc, nm = c, plain_names(c)
                    parts.append(oc)
                    pnames.append(nm)
                oc = f"{tag}_interaction{len(tmp)}"
                it = Interaction(inputCols=parts, outputCol=oc)
                stages.append(it)
                cur = it.transform(cur)
                tmp.append(oc)
                encoded.append(oc)
                acc = [""]
                for nm in pnames:
                    acc = [a + (":" if a else "") + b for a in acc for b in nm]
                names += acc
        stages.append(VectorAssembler(inputCols=encoded, outputCol=self.getFeaturesCol(),
                                      handleInvalid="keep" if hi == "keep" else hi))
        label_model = None
        if label in df.columns and (is_str(label) or self.getForceIndexLabel()):
            label_model = StringIndexer(inputCol=label, outputCol=self.getLabelCol(), handleInvalid=hi).fit(df)
        model = RFormulaModel(label, terms, has_icpt, stages, label_model, tmp, names)
        self._copyValues(model)
        return model


class RFormulaModel(Model):
    _params = _RFORMULA_PARAMS

    def __init__(self, label: str = "", terms=None, hasIntercept: bool = True, stages=None, labelModel=None,
                 tempCols=None, featureNames=None):
        super().__init__()
        self._label, self._terms, self._has_icpt = label, [list(t) for t in (terms or [])], bool(hasIntercept)
        self._stages = list(stages or [])
        self._label_model = labelModel
        self._tmp = list(tempCols or [])
        self._names = list(featureNames or [])

    @property
    def resolvedFormula(self) -> str:
        return f"ResolvedRFormula(label={self._label}, terms=[{','.join('{' + ','.join(t) + '}' for t in self._terms)}]" \
               f", hasIntercept={str(self._has_icpt).lower()})"

    def __str__(self):
        return f"RFormulaModel({self.resolvedFormula}) (uid={self.uid})"

    def _transform(self, df):
        cur = df
        for st in self._stages:
            cur = st.transform(cur)
        fc = self.getFeaturesCol()
        if self._names and len(self._names) == cur._feature_matrix(fc).shape[1]:
            cur.schema[fc].metadata = _vector_meta(self._names)
        lc = self.getLabelCol()
        if self._label in cur.columns:
            if self._label_model is not None:
                cur = self._label_model.transform(cur)
            elif lc not in cur.columns:
                cd = cur._column_data(self._label)
                cur = _replace_col(cur, lc, ColumnData(cd.values.to(torch.float64), cd.valid, T.DoubleType()))
        keep = [c for c in cur.columns if c not in self._tmp]
        return cur.select(*keep) if len(keep) != len(cur.columns) else cur

    def _save_impl(self, path):
        import os
        import pyarrow as pa
        from .pipeline import PipelineModel
        U.write_metadata(self, path, extra={"cmlTempCols": self._tmp, "cmlFeatureNames": self._names,
                                            "cmlHasLabelModel": self._label_model is not None})
        U.write_parquet(path, "data", pa.Table.from_pylist(
            [{"label": self._label, "terms": self._terms, "hasIntercept": self._has_icpt}],
            schema=pa.schema([("label", pa.string()), ("terms", pa.list_(pa.list_(pa.string()))),
                              pa.field("hasIntercept", pa.bool_(), nullable=False)])))
        stages = self._stages + ([self._label_model] if self._label_model is not None else [])
        pm = PipelineModel(stages)
        pm.uid = self.uid + "_pipeline"
        d = os.path.join(path, "pipelineModel")
        os.makedirs(d, exist_ok=True)
        pm._save_impl(d)

    @classmethod
    def _load_impl(cls, path, md):
        import os
        row = U.read_parquet(path, "data").to_pylist()[0]
        pm = U.load(os.path.join(path, "pipelineModel"))
        stages = list(pm.stages)
        label_model = stages.pop() if md.get("cmlHasLabelModel") else None
        m = cls(row["label"], row["terms"], row["hasIntercept"], stages, label_model, md.get("cmlTempCols", []),
                md.get("cmlFeatureNames", []))
        U.apply_params(m, md)
        return m


__all__: List[str] = ["MaxAbsScaler", "MaxAbsScalerModel", "RobustScaler", "RobustScalerModel", "ElementwiseProduct",
                      "PolynomialExpansion", "Interaction", "VectorSlicer", "VectorIndexer", "VectorIndexerModel",
                      "SQLTransformer", "VarianceThresholdSelector", "VarianceThresholdSelectorModel",
                      "UnivariateFeatureSelector", "UnivariateFeatureSelectorModel", "ChiSqSelector",
                      "ChiSqSelectorModel", "RFormula", "RFormulaModel", "parse_formula", "poly_terms",
                      "vector_attr_names"]
