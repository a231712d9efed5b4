"""pyspark.ml.functions: conversions between vector columns (dense [n, d] device tensors here) and
array columns (host lists)."""
from __future__ import annotations

import numpy as np
import torch

from ..sql import types as T
from ..sql.column import Column, ColumnData, Func, _to_host
from ..sql.functions import _c


def vector_to_array(col, dtype: str = "float64") -> Column:
    """Vector column -> array<double> (or array<float> with dtype='float32')."""
    if dtype not in ("float64", "float32"):
        raise ValueError("dtype must be 'float64' or 'float32'")

    def impl(frame, args):
        a = args[0]
        if not isinstance(a.dtype, T.VectorUDT):
            raise TypeError("vector_to_array needs a vector column")
        x = a.values.to(torch.float64 if dtype == "float64" else torch.float32).cpu().numpy()
        out = np.empty(x.shape[0], dtype=object)
        for i in range(x.shape[0]):
            out[i] = x[i].tolist()
        et = T.DoubleType() if dtype == "float64" else T.FloatType()
        return ColumnData(out, a.valid, T.ArrayType(et))
    return Column(Func("vector_to_array", [_c(col)], impl))


def array_to_vector(col) -> Column:
    """array<numeric> column of equal-length rows -> dense vector column on the frame's device."""
    def impl(frame, args):
        h = _to_host(args[0])
        rows = [v for v in h.values]
        if any(r is None for r in rows):
            raise ValueError("array_to_vector: null arrays are not supported")
        widths = {len(r) for r in rows}
        if len(widths) > 1:
            raise ValueError("array_to_vector: arrays must all have the same length")
        d = widths.pop() if widths else 0
        x = np.asarray(rows, dtype=np.float64).reshape(len(rows), d)
        return ColumnData(torch.as_tensor(x, device=frame._device), None, T.VectorUDT())
    return Column(Func("array_to_vector", [_c(col)], impl))


__all__ = ["vector_to_array", "array_to_vector"]
