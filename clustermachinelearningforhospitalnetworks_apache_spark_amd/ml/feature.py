"""Feature transformers: VectorAssembler (ref.py:134-136, ref.py:179), StringIndexer
(imported by the reference, ref.py:29), StandardScaler ([NS]), Binarizer (the
reference's ``when(LOS > 5.0, 1).otherwise(0)`` label, ref.py:176-177, as a
transformer), MinMaxScaler.

A vector column is one dense [n, d] tensor on the rank's device.  The assembler
packs columns with a single device concat (K2); the scaler computes per-feature
moments with the K7 kernel + one all-reduce and applies K8.
"""
from __future__ import annotations

import math
from typing import Dict, List, Optional

import numpy as np
import torch

from ..ops import glm_ops
from ..sql import types as T
from ..sql.column import ColumnData, NanCheckedColumnData
from .base import Estimator, Model, Transformer
from .linalg import DenseVector
from .param import NO_DEFAULT
from . import util as U
from .colutil import _auto_output, _replace_col  # noqa: F401 (re-exported)


def features_dtype(session) -> torch.dtype:
    name = session.conf.get("cml.ml.features.dtype", "float64")
    return {"float64": torch.float64, "double": torch.float64, "float32": torch.float32, "float": torch.float32,
            "bfloat16": torch.bfloat16, "bf16": torch.bfloat16}[str(name).lower()]


_NAN_MSG = "VectorAssembler: encountered NaN values with handleInvalid='error'"


class VectorAssembler(Transformer):
    _params = {
        "inputCols": (NO_DEFAULT, "input column names", "liststr"),
        "outputCol": ("__auto__", "output column name", str),
        "handleInvalid": ("error", "how to handle invalid data (NULL/NaN): 'error', 'skip' or 'keep'", str),
    }

    def __init__(self, inputCols=None, outputCol=None, handleInvalid=None):
        super().__init__(inputCols=inputCols, outputCol=outputCol, handleInvalid=handleInvalid)
        if self.getOutputCol() == "__auto__":
            self._defaultParamMap["outputCol"] = self.uid + "__output"

    def _transform(self, df):
        cols = self.getInputCols()
        dtype = features_dtype(df._session)
        cds = []
        for c in cols:
            cd = df._column_data(c)
            if cd.is_host:
                raise TypeError(f"VectorAssembler: column {c!r} of type {cd.dtype.simpleString()} is not numeric")
            cds.append(cd)
        hi = self.getHandleInvalid()
        if (len(cds) == 1 and isinstance(cds[0].dtype, T.VectorUDT) and cds[0].valid is None
                and cds[0].values.dtype == dtype and cds[0].values.is_contiguous() and hi != "skip"):
            # one dense vector input already in the target dtype: the assembled matrix IS the input
            # (no 2x HBM footprint for 100+ GB shards); only the invalid-value check reads it
            # (an input whose own deferred check is pending hands it on under "error"; "keep" reads it)
            x = cds[0]._vals() if hi == "error" else cds[0].values
            out = ColumnData(x, None, T.VectorUDT())
            if hi == "error" and df._nrows and x.is_floating_point():
                # Spark raises handleInvalid="error" when the assembled rows are consumed (its transform
                # is lazy); the check is deferred to the first consumer (DataFrame._feature_matrix), and
                # a consumer whose own pass over the rows already exposes a NaN takes it over for free
                # (StandardScaler.fit: the moments) — no extra read of a 100+ GB matrix here
                out = NanCheckedColumnData(x, None, T.VectorUDT(), getattr(cds[0], "nan_pending", None) or _NAN_MSG,
                                           df._comm)
            return self._named(df, _replace_col(df, self.getOutputCol(), out))
        if df._device.type == "cuda" and cds and df._nrows:
            # K2: one fused pass gathers the typed columns into the row-major matrix + invalid flags
            from ..ops import frame_ops
            x, bad = frame_ops.assemble([(cd.values, cd.valid) for cd in cds], out_dtype=dtype)
        else:
            x, bad = self._assemble_torch(df, cds)
            x = x.to(dtype)
        if df._nrows and cds:
            if hi == "error":
                if bool(bad.any().item()):
                    raise ValueError("VectorAssembler: encountered NULL or NaN values with handleInvalid='error'; "
                                     "drop them first (df.na.drop()) or set handleInvalid='skip'/'keep'")
            elif hi == "skip":
                keep = ~bad
                idx = df._mask_index(keep)
                df = df._take_rows(idx)
                x = x[idx]
        return self._named(df, _replace_col(df, self.getOutputCol(), ColumnData(x.contiguous(), None, T.VectorUDT())))

    def _named(self, src, out):
        """Attach Spark's ``ml_attr`` feature names: scalar columns by name, vector columns by their
        own attribute names or ``<col>_<i>``."""
        from .feature_more import _vector_meta, vector_attr_names
        names = []
        for c in self.getInputCols():
            cd = src._column_data(c)
            if isinstance(cd.dtype, T.VectorUDT):
                sub = vector_attr_names(src, c)
                names += sub if sub is not None else [f"{c}_{i}" for i in range(cd.values.shape[1])]
            else:
                names.append(c)
        out.schema[self.getOutputCol()].metadata = _vector_meta(names)
        return out

    @staticmethod
    def _assemble_torch(df, cds):
        """CPU path (and the oracle of the K2 kernel test)."""
        parts, bad = [], torch.zeros(df._nrows, dtype=torch.bool, device=df._device)
        for cd in cds:
            v = cd.values
            if v.dim() == 1:
                v = v.reshape(-1, 1)
            v = v.to(torch.float64)
            invalid = ~cd.valid_mask().reshape(-1) if cd.valid is not None else None
            nan = torch.isnan(v).any(1)
            bad = bad | (nan if invalid is None else (nan | invalid))
            if invalid is not None:
                v = torch.where(invalid.reshape(-1, 1), torch.full_like(v, float("nan")), v)
            parts.append(v)
        x = torch.cat(parts, 1) if parts else torch.zeros((df._nrows, 0), dtype=torch.float64, device=df._device)
        return x, bad

    def _save_impl(self, path):
        U.write_metadata(self, path)


class StandardScaler(Estimator):
    """Spark defaults: withMean=False, withStd=True, unbiased (n-1) standard deviation."""
    _params = {
        "inputCol": (NO_DEFAULT, "input column name", str),
        "outputCol": ("__auto__", "output column name", str),
        "withMean": (False, "whether to center data with mean", bool),
        "withStd": (True, "whether to scale the data to unit standard deviation", bool),
        "outputDtype": ("auto", "cml extension: dtype of the scaled vectors (auto/float64/float32/bfloat16/fp8); "
                                "fp8 = OCP e4m3fn, saturated at +-448 (standardized values fit it)", str),
    }

    def __init__(self, withMean=None, withStd=None, inputCol=None, outputCol=None, outputDtype=None):
        super().__init__(withMean=withMean, withStd=withStd, inputCol=inputCol, outputCol=outputCol,
                         outputDtype=outputDtype)
        if self.getOutputCol() == "__auto__":
            self._defaultParamMap["outputCol"] = self.uid + "__output"

    def _fit(self, df):
        col = self.getInputCol()
        pending = df._pending_nan_check(col)
        x = df._feature_matrix(col, defer_nan_check=True)
        d = x.shape[1]
        n, s1, s2, shift = glm_ops.moments(x, d)
        comm = df._comm
        # merge shifted moments across ranks exactly: use a common shift (rank 0's first row)
        common = comm.broadcast_object(shift.cpu().numpy() if n else None, 0)
        if common is None:
            common = np.zeros(d)
        common_t = torch.as_tensor(common, dtype=torch.float64, device=x.device)
        delta = shift - common_t
        # Σ(x-c) = Σ(x-s) + n(s-c); Σ(x-c)² = Σ(x-s)² + 2(s-c)Σ(x-s) + n(s-c)²
        t1 = s1 + n * delta
        t2 = s2 + 2 * delta * s1 + n * delta * delta
        msg = torch.cat([torch.tensor([float(n)], dtype=torch.float64, device=x.device), t1, t2])
        comm.allreduce_(msg)
        if pending is not None:
            # the moments carry any NaN of the rows (every rank sees the all-reduced sums): only then the
            # exact check runs (a NaN sum can also come from +inf and -inf in one column)
            if bool(torch.isnan(msg).any().item()):
                df._run_nan_check(col)
            df._clear_nan_check(col)
        N = msg[0].item()
        T1, T2 = msg[1:1 + d], msg[1 + d:]
        mean = common_t + T1 / max(N, 1)
        m2 = torch.clamp(T2 - T1 * T1 / max(N, 1), min=0.0)
        var = m2 / (N - 1) if N > 1 else torch.zeros_like(m2)
        std = torch.sqrt(var)
        model = StandardScalerModel(mean.cpu().numpy(), std.cpu().numpy())
        self._copyValues(model)
        return model


class StandardScalerModel(Model):
    _params = StandardScaler._params

    def __init__(self, mean=None, std=None):
        super().__init__()
        self._mean = np.asarray(mean if mean is not None else [], dtype=np.float64)
        self._std = np.asarray(std if std is not None else [], dtype=np.float64)

    @property
    def mean(self) -> DenseVector:
        return DenseVector(self._mean)

    @property
    def std(self) -> DenseVector:
        return DenseVector(self._std)

    def _transform(self, df):
        x = df._feature_matrix(self.getInputCol())
        d = x.shape[1]
        with_std = self.getWithStd()
        inv = np.where(self._std > 0, 1.0 / np.where(self._std > 0, self._std, 1.0), 0.0) if with_std \
            else np.ones(d)
        dev = x.device
        od = self.getOutputDtype()
        out_dtype = x.dtype if od == "auto" else {"float64": torch.float64, "float32": torch.float32,
                                                 "bfloat16": torch.bfloat16, "fp8": torch.float8_e4m3fn,
                                                 "float8_e4m3fn": torch.float8_e4m3fn}[od]
        y = glm_ops.scale_apply(x, d, torch.as_tensor(self._mean, device=dev), torch.as_tensor(inv, device=dev),
                                self.getWithMean(), out_dtype=out_dtype)
        return _replace_col(df, self.getOutputCol(), ColumnData(y, None, T.VectorUDT()))

    def _save_impl(self, path):
        import pyarrow as pa
        U.write_metadata(self, path)
        table = pa.Table.from_pylist([{"std": U.vector_struct(self._std), "mean": U.vector_struct(self._mean)}],
                                     schema=pa.schema([("std", U.vector_arrow_type()), ("mean", U.vector_arrow_type())]))
        U.write_parquet(path, "data", table)

    @classmethod
    def _load_impl(cls, path, md):
        row = U.read_parquet(path, "data").to_pylist()[0]
        m = cls(U.vector_from_struct(row["mean"]), U.vector_from_struct(row["std"]))
        U.apply_params(m, md)
        return m


class MinMaxScaler(Estimator):
    _params = {
        "inputCol": (NO_DEFAULT, "input column name", str),
        "outputCol": ("__auto__", "output column name", str),
        "min": (0.0, "lower bound of the output feature range", float),
        "max": (1.0, "upper bound of the output feature range", float),
    }

    def __init__(self, min=None, max=None, inputCol=None, outputCol=None):  # noqa: A002
        super().__init__(min=min, max=max, inputCol=inputCol, outputCol=outputCol)
        if self.getOutputCol() == "__auto__":
            self._defaultParamMap["outputCol"] = self.uid + "__output"

    def _fit(self, df):
        x = df._feature_matrix(self.getInputCol()).to(torch.float64)
        d = x.shape[1]
        comm = df._comm
        lo = x.min(0).values if x.shape[0] else torch.full((d,), float("inf"), device=x.device, dtype=torch.float64)
        hi = x.max(0).values if x.shape[0] else torch.full((d,), float("-inf"), device=x.device, dtype=torch.float64)
        lo, hi = lo.clone(), hi.clone()
        comm.allreduce_(lo, "min")
        comm.allreduce_(hi, "max")
        m = MinMaxScalerModel(lo.cpu().numpy(), hi.cpu().numpy())
        self._copyValues(m)
        return m


class MinMaxScalerModel(Model):
    _params = MinMaxScaler._params

    def __init__(self, originalMin=None, originalMax=None):
        super().__init__()
        self._omin = np.asarray(originalMin if originalMin is not None else [], dtype=np.float64)
        self._omax = np.asarray(originalMax if originalMax is not None else [], dtype=np.float64)

    @property
    def originalMin(self):
        return DenseVector(self._omin)

    @property
    def originalMax(self):
        return DenseVector(self._omax)

    def _transform(self, df):
        x = df._feature_matrix(self.getInputCol())
        dev = x.device
        rng = self._omax - self._omin
        lo, hi = self.getMin(), self.getMax()
        scale = np.where(rng != 0, (hi - lo) / np.where(rng != 0, rng, 1.0), 0.0)
        # y = (x - omin) * scale + lo   (constant features map to (lo+hi)/2 as in Spark)
        y = glm_ops.scale_apply(x, x.shape[1], torch.as_tensor(self._omin, device=dev),
                                torch.as_tensor(scale, device=dev), True, out_dtype=x.dtype).to(torch.float64)
        const = torch.as_tensor(rng == 0, device=dev)
        y = torch.where(const, torch.full_like(y, 0.5 * (lo + hi)), y + lo).to(x.dtype)
        return _replace_col(df, self.getOutputCol(), ColumnData(y, None, T.VectorUDT()))

    def _save_impl(self, path):
        import pyarrow as pa
        U.write_metadata(self, path)
        table = pa.Table.from_pylist([{"originalMin": U.vector_struct(self._omin),
                                       "originalMax": U.vector_struct(self._omax)}],
                                     schema=pa.schema([("originalMin", U.vector_arrow_type()),
                                                       ("originalMax", U.vector_arrow_type())]))
        U.write_parquet(path, "data", table)

    @classmethod
    def _load_impl(cls, path, md):
        row = U.read_parquet(path, "data").to_pylist()[0]
        m = cls(U.vector_from_struct(row["originalMin"]), U.vector_from_struct(row["originalMax"]))
        U.apply_params(m, md)
        return m


class Binarizer(Transformer):
    """x > threshold -> 1.0 else 0.0 (the reference's LOS_binary label, ref.py:176-177)."""
    _params = {
        "threshold": (0.0, "threshold used to binarize continuous features", float),
        "inputCol": (NO_DEFAULT, "input column name", str),
        "outputCol": ("__auto__", "output column name", str),
    }

    def __init__(self, threshold=None, inputCol=None, outputCol=None):
        super().__init__(threshold=threshold, inputCol=inputCol, outputCol=outputCol)
        if self.getOutputCol() == "__auto__":
            self._defaultParamMap["outputCol"] = self.uid + "__output"

    def _transform(self, df):
        cd = df._column_data(self.getInputCol())
        v = cd.values
        if v.is_cuda and v.numel():
            from ..ops import frame_ops  # K6
            out = frame_ops.binarize(v, self.getThreshold())
        else:
            out = (v.to(torch.float64) > self.getThreshold()).to(torch.float64)
        dt = T.VectorUDT() if isinstance(cd.dtype, T.VectorUDT) else T.DoubleType()
        return _replace_col(df, self.getOutputCol(), ColumnData(out, cd.valid, dt))


class StringIndexer(Estimator):
    _params = {
        "inputCol": (NO_DEFAULT, "input column name", str),
        "outputCol": ("__auto__", "output column name", str),
        "handleInvalid": ("error", "how to handle unseen labels: 'error', 'skip' or 'keep'", str),
        "stringOrderType": ("frequencyDesc", "frequencyDesc|frequencyAsc|alphabetDesc|alphabetAsc", str),
    }

    def __init__(self, inputCol=None, outputCol=None, handleInvalid=None, stringOrderType=None):
        super().__init__(inputCol=inputCol, outputCol=outputCol, handleInvalid=handleInvalid,
                         stringOrderType=stringOrderType)
        if self.getOutputCol() == "__auto__":
            self._defaultParamMap["outputCol"] = self.uid + "__output"

    def _fit(self, df):
        from ..sql.dataframe import column_to_python
        vals = column_to_python(df._column_data(self.getInputCol()))
        counts: Dict[str, int] = {}
        for v in vals:
            if v is None:
                continue
            k = _fmt_label(v)
            counts[k] = counts.get(k, 0) + 1
        merged: Dict[str, int] = {}
        for part in df._comm.allgather_object(counts):
            for k, c in part.items():
                merged[k] = merged.get(k, 0) + c
        order = self.getStringOrderType()
        items = list(merged.items())
        if order == "frequencyDesc":
            items.sort(key=lambda kv: (-kv[1], kv[0]))
        elif order == "frequencyAsc":
            items.sort(key=lambda kv: (kv[1], kv[0]))
        elif order == "alphabetDesc":
            items.sort(key=lambda kv: kv[0], reverse=True)
        else:
            items.sort(key=lambda kv: kv[0])
        m = StringIndexerModel([k for k, _ in items])
        self._copyValues(m)
        return m


def _fmt_label(v) -> str:
    if isinstance(v, float) and v.is_integer():
        return repr(v)
    return str(v)


class StringIndexerModel(Model):
    _params = StringIndexer._params

    def __init__(self, labels: Optional[List[str]] = None):
        super().__init__()
        self._labels = list(labels or [])

    @property
    def labels(self) -> List[str]:
        return list(self._labels)

    @property
    def labelsArray(self) -> List[List[str]]:
        return [list(self._labels)]

    def _transform(self, df):
        from ..sql.dataframe import column_to_python
        vals = column_to_python(df._column_data(self.getInputCol()))
        idx = {l: i for i, l in enumerate(self._labels)}
        hi = self.getHandleInvalid()
        out = np.zeros(len(vals), dtype=np.float64)
        keep = np.ones(len(vals), dtype=bool)
        for i, v in enumerate(vals):
            k = None if v is None else idx.get(_fmt_label(v))
            if k is None:
                if hi == "error":
                    raise ValueError(f"StringIndexer: unseen label {v!r}; set handleInvalid='skip' or 'keep'")
                if hi == "skip":
                    keep[i] = False
                else:
                    out[i] = len(self._labels)
            else:
                out[i] = k
        res = _replace_col(df, self.getOutputCol(),
                           ColumnData(torch.as_tensor(out, device=df._device), None, T.DoubleType()))
        if not keep.all():
            res = res._mask_rows(torch.as_tensor(keep, device=df._device))
        return res

    def _save_impl(self, path):
        import pyarrow as pa
        U.write_metadata(self, path)
        U.write_parquet(path, "data", pa.table({"labelsArray": pa.array([[self._labels]],
                                                                        type=pa.list_(pa.list_(pa.string())))}))

    @classmethod
    def _load_impl(cls, path, md):
        row = U.read_parquet(path, "data").to_pylist()[0]
        m = cls(row["labelsArray"][0])
        U.apply_params(m, md)
        return m


class IndexToString(Transformer):
    _params = {
        "inputCol": (NO_DEFAULT, "input column name", str),
        "outputCol": ("__auto__", "output column name", str),
        "labels": (NO_DEFAULT, "ordered list of labels", "liststr"),
    }

    def __init__(self, inputCol=None, outputCol=None, labels=None):
        super().__init__(inputCol=inputCol, outputCol=outputCol, labels=labels)
        if self.getOutputCol() == "__auto__":
            self._defaultParamMap["outputCol"] = self.uid + "__output"

    def _transform(self, df):
        cd = df._column_data(self.getInputCol())
        labels = self.getLabels()
        vals = cd.values.cpu().numpy()
        out = np.array([labels[int(v)] if 0 <= int(v) < len(labels) else None for v in vals], dtype=object)
        return _replace_col(df, self.getOutputCol(), ColumnData(out, None, T.StringType()))


def _in_out_cols(inst) -> tuple:
    """(inputCols, outputCols) from either the single- or the multi-column params."""
    if inst.isSet("inputCols"):
        ins = list(inst.getInputCols())
        outs = list(inst.getOrDefault("outputCols")) if inst.isSet("outputCols") else [c + "_out" for c in ins]
    else:
        ins = [inst.getInputCol()]
        outs = [inst.getOutputCol()]
    if len(ins) != len(outs):
        raise ValueError(f"{type(inst).__name__}: inputCols and outputCols differ in length")
    return ins, outs


class OneHotEncoder(Estimator):
    """Category indices (e.g. StringIndexer output for ``hospital_id``, the column the reference
    imports StringIndexer for but never encodes, ref.py:29) -> one-hot vectors. Spark semantics:
    ``dropLast`` drops the last category's slot (it becomes all-zero), ``handleInvalid='keep'`` adds a
    slot for indices outside [0, numCategories). The vector column is a dense [n, size] device tensor
    (Spark emits sparse vectors; the values are the same). numCategories = max index + 1 over all
    ranks (one all-reduce)."""
    _params = {
        "inputCol": (NO_DEFAULT, "input column name", str),
        "outputCol": ("__auto__", "output column name", str),
        "inputCols": (NO_DEFAULT, "input column names", "liststr"),
        "outputCols": (NO_DEFAULT, "output column names", "liststr"),
        "dropLast": (True, "whether to drop the last category", bool),
        "handleInvalid": ("error", "how to handle invalid data: 'error' or 'keep'", str),
    }

    def __init__(self, inputCols=None, outputCols=None, handleInvalid=None, dropLast=None, inputCol=None,
                 outputCol=None):
        super().__init__(inputCols=inputCols, outputCols=outputCols, handleInvalid=handleInvalid, dropLast=dropLast,
                         inputCol=inputCol, outputCol=outputCol)
        if self.getOutputCol() == "__auto__":
            self._defaultParamMap["outputCol"] = self.uid + "__output"

    def _fit(self, df):
        ins, _ = _in_out_cols(self)
        maxes = []
        for c in ins:
            cd = df._column_data(c)
            v = torch.as_tensor(cd.values).to(torch.float64)
            vm = torch.as_tensor(cd.valid_mask(), device=v.device)
            v = v[vm & ~torch.isnan(v)] if v.numel() else v
            if v.numel() and (bool((v < 0).any()) or bool((v != torch.floor(v)).any())) \
                    and self.getHandleInvalid() == "error":
                raise ValueError(f"OneHotEncoder: column {c} holds values that are not category indices")
            maxes.append(float(v.max()) if v.numel() else -1.0)
        t = torch.as_tensor(maxes, dtype=torch.float64, device=df._device)
        df._comm.allreduce_(t, "max")
        m = OneHotEncoderModel([int(x) + 1 for x in t.cpu().tolist()])
        self._copyValues(m)
        return m


class OneHotEncoderModel(Model):
    _params = OneHotEncoder._params

    def __init__(self, categorySizes: Optional[List[int]] = None):
        super().__init__()
        self.categorySizes = list(categorySizes or [])

    def _transform(self, df):
        ins, outs = _in_out_cols(self)
        keep = self.getHandleInvalid() == "keep"
        drop = bool(self.getDropLast())
        for c, o, nc in zip(ins, outs, self.categorySizes):
            cd = df._column_data(c)
            v = torch.as_tensor(cd.values).to(torch.float64)
            valid = torch.as_tensor(cd.valid_mask(), device=v.device)
            size = nc + (1 if keep else 0) - (1 if drop else 0)
            bad = ~valid | torch.isnan(v) | (v < 0) | (v >= nc) | (v != torch.floor(v))
            if bool(bad.any()) and not keep:
                raise ValueError(f"OneHotEncoder: invalid category index in column {c} "
                                 "(set handleInvalid='keep' to map it to an extra slot)")
            idx = torch.where(bad, torch.full_like(v, nc), v).to(torch.int64)  # 'keep' slot = nc
            out = torch.zeros((v.shape[0], max(size, 0)), dtype=torch.float64, device=v.device)
            hit = idx < size  # the dropped last slot leaves the row all-zero
            if size > 0 and bool(hit.any()):
                rows = torch.nonzero(hit).squeeze(1)
                out[rows, idx[rows]] = 1.0
            df = _replace_col(df, o, ColumnData(out, None, T.VectorUDT()))
        return df

    def _save_impl(self, path):
        import pyarrow as pa
        U.write_metadata(self, path)
        U.write_parquet(path, "data", pa.table({"categorySizes": pa.array([self.categorySizes],
                                                                          type=pa.list_(pa.int32()))}))

    @classmethod
    def _load_impl(cls, path, md):
        row = U.read_parquet(path, "data").to_pylist()[0]
        m = cls(row["categorySizes"])
        U.apply_params(m, md)
        return m


class Imputer(Estimator):
    """Fills missing values (null, and ``missingValue`` — NaN by default) per column with the
    column's mean, median or mode over all ranks (Spark's Imputer). The reference drops every
    row with a null instead (``na.drop``, ref.py:128); this keeps them. mean: one f64 all-reduce
    of (sum, count); median / mode: exact, from the all-gathered non-missing values (Spark's median
    is approxQuantile with relativeError 0.001 — exact is within that bound)."""
    _params = {
        "inputCol": (NO_DEFAULT, "input column name", str),
        "outputCol": ("__auto__", "output column name", str),
        "inputCols": (NO_DEFAULT, "input column names", "liststr"),
        "outputCols": (NO_DEFAULT, "output column names", "liststr"),
        "strategy": ("mean", "strategy for imputation: mean, median or mode", str),
        "missingValue": (float("nan"), "placeholder for the missing values", float),
        "relativeError": (0.001, "relative error for approximate quantile computation", float),
    }

    def __init__(self, strategy=None, missingValue=None, inputCols=None, outputCols=None, inputCol=None,
                 outputCol=None, relativeError=None):
        super().__init__(strategy=strategy, missingValue=missingValue, inputCols=inputCols, outputCols=outputCols,
                         inputCol=inputCol, outputCol=outputCol, relativeError=relativeError)
        if self.getOutputCol() == "__auto__":
            self._defaultParamMap["outputCol"] = self.uid + "__output"

    def _present(self, cd) -> torch.Tensor:
        v = torch.as_tensor(cd.values).to(torch.float64)
        ok = torch.as_tensor(cd.valid_mask(), device=v.device) & ~torch.isnan(v)
        mv = float(self.getMissingValue())
        if not math.isnan(mv):
            ok &= v != mv
        return v[ok]

    def _fit(self, df):
        ins, _ = _in_out_cols(self)
        strat = self.getStrategy()
        if strat not in ("mean", "median", "mode"):
            raise ValueError(f"Imputer: unknown strategy {strat!r}")
        comm = df._comm
        surrogates = []
        for c in ins:
            v = self._present(df._column_data(c))
            if strat == "mean":
                t = torch.as_tensor([float(v.sum()), float(v.numel())], dtype=torch.float64, device=df._device)
                comm.allreduce_(t)
                s, n = t.cpu().tolist()
                if n == 0:
                    raise ValueError(f"Imputer: surrogate cannot be computed, all values of {c} are missing")
                surrogates.append(s / n)
                continue
            allv = comm.allgather_cat(v.to(df._device)).cpu().numpy()
            if allv.size == 0:
                raise ValueError(f"Imputer: surrogate cannot be computed, all values of {c} are missing")
            if strat == "median":
                srt = np.sort(allv)
                surrogates.append(float(srt[(srt.size - 1) // 2]))  # lower median, as approxQuantile(0.5)
            else:
                vals, cnt = np.unique(allv, return_counts=True)
                surrogates.append(float(vals[np.argmax(cnt)]))  # ties -> smallest value (Spark)
        m = ImputerModel(surrogates)
        self._copyValues(m)
        return m


class ImputerModel(Model):
    _params = Imputer._params

    def __init__(self, surrogates: Optional[List[float]] = None):
        super().__init__()
        self.surrogates = list(surrogates or [])

    @property
    def surrogateDF(self):
        import pandas as pd
        ins, _ = _in_out_cols(self)
        return pd.DataFrame({c: [s] for c, s in zip(ins, self.surrogates)})

    def _transform(self, df):
        ins, outs = _in_out_cols(self)
        mv = float(self.getMissingValue())
        for c, o, s in zip(ins, outs, self.surrogates):
            cd = df._column_data(c)
            v = torch.as_tensor(cd.values)
            vf = v.to(torch.float64)
            miss = ~torch.as_tensor(cd.valid_mask(), device=v.device) | torch.isnan(vf)
            if not math.isnan(mv):
                miss |= vf == mv
            if T.is_integral(cd.dtype):
                out = torch.where(miss, torch.full_like(v, int(s)), v)
            else:
                out = torch.where(miss, torch.full_like(vf, s), vf)
            dt = cd.dtype if T.is_integral(cd.dtype) else T.DoubleType()
            df = _replace_col(df, o, ColumnData(out, None, dt))
        return df

    def _save_impl(self, path):
        import pyarrow as pa
        ins, _ = _in_out_cols(self)
        U.write_metadata(self, path)
        U.write_parquet(path, "data", pa.table({c: pa.array([s], type=pa.float64())
                                                for c, s in zip(ins, self.surrogates)}))

    @classmethod
    def _load_impl(cls, path, md):
        m = cls()
        U.apply_params(m, md)
        ins, _ = _in_out_cols(m)
        row = U.read_parquet(path, "data").to_pylist()[0]
        m.surrogates = [float(row[c]) for c in ins]
        return m


from .feature_extra import Bucketizer, Normalizer, PCA, PCAModel, QuantileDiscretizer  # noqa: E402,F401
from .feature_more import (ChiSqSelector, ChiSqSelectorModel, ElementwiseProduct, Interaction,  # noqa: E402,F401
                           MaxAbsScaler, MaxAbsScalerModel, PolynomialExpansion, RFormula, RFormulaModel,
                           RobustScaler, RobustScalerModel, SQLTransformer, UnivariateFeatureSelector,
                           UnivariateFeatureSelectorModel, VarianceThresholdSelector, VarianceThresholdSelectorModel,
                           VectorIndexer, VectorIndexerModel, VectorSlicer)
from .lsh import (BucketedRandomProjectionLSH, BucketedRandomProjectionLSHModel, MinHashLSH,  # noqa: E402,F401
                  MinHashLSHModel)
from .feature_text import (CountVectorizer, CountVectorizerModel, HashingTF, IDF, IDFModel, NGram,  # noqa: E402,F401
                           RegexTokenizer, StopWordsRemover, Tokenizer)
from .feature_misc import DCT, FeatureHasher, VectorSizeHint  # noqa: E402,F401
from .word2vec import Word2Vec, Word2VecModel  # noqa: E402,F401
