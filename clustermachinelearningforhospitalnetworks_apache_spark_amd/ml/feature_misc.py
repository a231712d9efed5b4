"""Remaining pyspark.ml.feature transformers: DCT, FeatureHasher, VectorSizeHint.

The reference imports its transformers from ``pyspark.ml.feature`` (ref.py:29); these complete
that namespace. DCT is one [n, d] x [d, d] GEMM against the orthonormal DCT-II basis (Spark's
JTransforms ``forward(x, scale = true)``; the inverse is the DCT-III = transpose). FeatureHasher
hashes ``column`` (numeric) or ``column=value`` (categorical) with MurmurHash3 x86_32, seed 42,
and scatters the values into the dense device matrix with one ``index_put_`` (duplicates summed).
"""
from __future__ import annotations

import math
from typing import Dict, List

import numpy as np
import torch

from ..sql import types as T
from ..sql.column import ColumnData
from .base import Transformer
from .colutil import _auto_output, _replace_col
from .feature_text import _scatter_counts, murmur3_32
from .param import NO_DEFAULT


def dct_basis(d: int, inverse: bool = False, dtype=torch.float64, device=None) -> torch.Tensor:
    """Orthonormal DCT-II matrix C ([d, d], y = C x); the inverse transform is C^T."""
    n = torch.arange(d, dtype=torch.float64)
    k = n[:, None]
    c = torch.cos(math.pi * (2 * n[None, :] + 1) * k / (2 * d)) * math.sqrt(2.0 / d)
    c[0] /= math.sqrt(2.0)
    c = c.T.contiguous() if inverse else c
    return c.to(dtype=dtype, device=device)


class DCT(Transformer):
    """Discrete cosine transform (type II, orthonormal) of each feature vector; ``inverse=True``
    applies the type-III inverse."""
    _params = {"inputCol": (NO_DEFAULT, "input column name", str),
               "outputCol": ("__auto__", "output column name", str),
               "inverse": (False, "Set transformer to perform inverse DCT", bool)}

    def __init__(self, inverse=None, inputCol=None, outputCol=None):
        super().__init__(inverse=inverse, inputCol=inputCol, outputCol=outputCol)
        _auto_output(self)

    def _transform(self, df):
        cd = df._cols[self.getInputCol()]
        x = df._feature_matrix(self.getInputCol()).to(torch.float64)
        if x.shape[1] == 0:
            raise ValueError("DCT: input vectors must be non-empty")
        c = dct_basis(x.shape[1], self.getInverse(), device=x.device)
        y = x @ c.T
        return _replace_col(df, self.getOutputCol(), ColumnData(y, cd.valid, T.VectorUDT()))


def _hash_index(term: str, n: int) -> int:
    return murmur3_32(term.encode("utf-8"), 42) % n  # Python % is Spark's nonNegativeMod


def _value_str(v) -> str:
    if isinstance(v, bool):
        return "true" if v else "false"
    if isinstance(v, float):
        from .util import java_double_str
        return java_double_str(v)
    return str(v)


class FeatureHasher(Transformer):
    """Hashes a set of columns into one feature vector of ``numFeatures`` entries. Numeric columns
    (not listed in ``categoricalCols``) put their value at hash(name); string / boolean /
    categorical columns put 1.0 at hash(name=value). Nulls are skipped; collisions add up."""
    _params = {"inputCols": (NO_DEFAULT, "input column names", "liststr"),
               "outputCol": ("__auto__", "output column name", str),
               "numFeatures": (1 << 18, "Number of features. Should be greater than 0", int),
               "categoricalCols": ([], "numeric columns to treat as categorical", "liststr")}

    def __init__(self, numFeatures=None, inputCols=None, outputCol=None, categoricalCols=None):
        super().__init__(numFeatures=numFeatures, inputCols=inputCols, outputCol=outputCol,
                         categoricalCols=categoricalCols)
        _auto_output(self)

    def _transform(self, df):
        from ..sql.dataframe import column_to_python
        nf = self.getNumFeatures()
        if nf <= 0:
            raise ValueError("numFeatures must be > 0")
        cat = set(self.getOrDefault("categoricalCols") or [])
        n = df._nrows
        dev = df._device
        rows_i: List[torch.Tensor] = []
        cols_i: List[torch.Tensor] = []
        vals: List[torch.Tensor] = []
        for name in self.getInputCols():
            cd = df._cols[name]
            numeric = (not cd.is_host and not isinstance(cd.dtype, (T.BooleanType, T.VectorUDT))
                       and name not in cat and cd.values.dim() == 1)
            if numeric:
                vm = cd.valid_mask().to(dev)
                r = torch.nonzero(vm).flatten()
                rows_i.append(r)
                cols_i.append(torch.full_like(r, _hash_index(name, nf)))
                vals.append(cd.values.to(torch.float64)[r])
                continue
            py = column_to_python(cd)
            cache: Dict = {}
            rr, cc = [], []
            for i, v in enumerate(py):
                if v is None:
                    continue
                j = cache.get(v)
                if j is None:
                    j = cache[v] = _hash_index(f"{name}={_value_str(v)}", nf)
                rr.append(i)
                cc.append(j)
            rows_i.append(torch.as_tensor(rr, dtype=torch.int64, device=dev))
            cols_i.append(torch.as_tensor(cc, dtype=torch.int64, device=dev))
            vals.append(torch.ones(len(rr), dtype=torch.float64, device=dev))
        x = _scatter_counts(df, [[] for _ in range(n)], nf, False)
        if rows_i:
            x.index_put_((torch.cat(rows_i), torch.cat(cols_i)), torch.cat(vals), accumulate=True)
        return _replace_col(df, self.getOutputCol(), ColumnData(x, None, T.VectorUDT()))


class VectorSizeHint(Transformer):
    """Declares the size of a vector column (attached as ``ml_attr.num_attrs`` metadata). Rows whose
    vector is null or of another size raise (``handleInvalid='error'``), are dropped ('skip') or
    are passed through unchecked ('optimistic')."""
    _params = {"inputCol": (NO_DEFAULT, "input column name", str),
               "size": (NO_DEFAULT, "Size of vectors in column.", int),
               "handleInvalid": ("error", "How to handle invalid vectors in inputCol: 'error', 'skip' or "
                                          "'optimistic'", str)}

    def __init__(self, inputCol=None, size=None, handleInvalid=None):
        super().__init__(inputCol=inputCol, size=size, handleInvalid=handleInvalid)

    def _transform(self, df):
        name, size, how = self.getInputCol(), self.getSize(), self.getHandleInvalid()
        if how not in ("error", "skip", "optimistic"):
            raise ValueError(f"handleInvalid must be error/skip/optimistic, got {how!r}")
        cd = df._cols[name]
        if not isinstance(cd.dtype, T.VectorUDT):
            raise TypeError(f"VectorSizeHint: column {name!r} is not a vector column")
        d = int(cd.values.shape[1]) if cd.values.dim() == 2 else -1
        out = df
        if how != "optimistic":
            bad_size = d != size and df._nrows > 0
            if how == "error":
                if bad_size:
                    raise ValueError(f"VectorSizeHint: expected vectors of size {size} in {name!r}, got {d}")
                if cd.valid is not None and not bool(cd.valid.all()):
                    raise ValueError(f"VectorSizeHint: null vectors in {name!r} (handleInvalid='error')")
            else:
                keep = cd.valid_mask().to(df._device)
                if bad_size:
                    keep = torch.zeros_like(keep)
                out = df._mask_rows(keep)
        if d != size:
            return out
        res = _replace_col(out, name, out._cols[name])
        old = (df.schema[name].metadata or {}).get("ml_attr", {})
        res.schema[name].metadata = {"ml_attr": old if old.get("num_attrs") == size else {"num_attrs": size}}
        return res

__all__ = ["DCT", "FeatureHasher", "VectorSizeHint", "dct_basis"]
