"""Build device-resident column shards from host data (lists, numpy, pandas, arrow)."""
from __future__ import annotations

import datetime as _dt
import math
from typing import Any, Dict, List, Optional, Sequence

import numpy as np
import torch

from . import types as T
from .column import ColumnData, ts_to_micros


def _is_null(v) -> bool:
    if v is None:
        return True
    if isinstance(v, float) and math.isnan(v):
        return False  # NaN is a value in Spark, not null
    try:
        import pandas as pd
        if v is pd.NaT:
            return True
    except Exception:  # pragma: no cover
        pass
    return False


def column_from_values(values, dtype: T.DataType, device) -> ColumnData:
    """Python/numpy values -> ColumnData with a validity mask."""
    if isinstance(values, np.ndarray) and values.dtype != object and dtype.torch_dtype is not None \
            and not isinstance(dtype, (T.TimestampType, T.DateType)):
        arr = values
        valid = None
        if arr.dtype.kind == "f" and T.is_integral(dtype):
            nan = np.isnan(arr)
            valid = None if not nan.any() else torch.as_tensor(~nan, device=device)
            arr = np.where(nan, 0, arr)
        t = torch.as_tensor(np.ascontiguousarray(arr)).to(device=device, dtype=dtype.torch_dtype)
        return ColumnData(t, valid, dtype)
    if isinstance(dtype, T.TimestampType) and isinstance(values, np.ndarray) and values.dtype.kind == "M":
        nat = np.isnat(values)
        us = values.astype("datetime64[us]").astype(np.int64)
        us = np.where(nat, 0, us)
        return ColumnData(torch.as_tensor(us).to(device), None if not nat.any() else
                          torch.as_tensor(~nat, device=device), dtype)
    if isinstance(dtype, T.StringType):
        return _string_column(values, dtype)
    vals = list(values) if not isinstance(values, list) else values
    n = len(vals)
    if isinstance(dtype, T.VectorUDT):
        from ..ml.linalg import as_array
        valid = np.array([v is not None for v in vals], dtype=bool)
        d = 0
        for v in vals:
            if v is not None:
                d = len(as_array(v))
                break
        arr = np.zeros((n, d), dtype=np.float64)
        for i, v in enumerate(vals):
            if v is not None:
                arr[i] = as_array(v)
        return ColumnData(torch.as_tensor(arr, device=device), None if valid.all() else torch.as_tensor(
            valid, device=device), dtype)
    if dtype.torch_dtype is None or dtype.host_only:
        out = np.empty(n, dtype=object)
        valid = np.ones(n, dtype=bool)
        for i, v in enumerate(vals):
            if _is_null(v):
                valid[i] = False
                out[i] = None
            else:
                keep = isinstance(dtype, (T.ArrayType, T.StructType, T.MapType, T.MatrixUDT)) or (
                    isinstance(dtype, T.BinaryType) and isinstance(v, (bytes, bytearray)))
                out[i] = v if keep or isinstance(v, str) else str(v)
        return ColumnData(out, None if valid.all() else valid, dtype)
    valid = np.ones(n, dtype=bool)
    if isinstance(dtype, T.TimestampType):
        arr = np.zeros(n, dtype=np.int64)
        for i, v in enumerate(vals):
            if _is_null(v):
                valid[i] = False
            else:
                try:
                    arr[i] = ts_to_micros(v.to_pydatetime() if hasattr(v, "to_pydatetime") else v)
                except (TypeError, ValueError):
                    valid[i] = False
    elif isinstance(dtype, T.DateType):
        arr = np.zeros(n, dtype=np.int32)
        for i, v in enumerate(vals):
            if _is_null(v):
                valid[i] = False
            else:
                if isinstance(v, str):
                    v = _dt.date.fromisoformat(v[:10])
                if isinstance(v, _dt.datetime):
                    v = v.date()
                arr[i] = (v - _dt.date(1970, 1, 1)).days
    else:
        npd = {torch.bool: np.bool_, torch.int8: np.int8, torch.int16: np.int16, torch.int32: np.int32,
               torch.int64: np.int64, torch.float32: np.float32, torch.float64: np.float64}[dtype.torch_dtype]
        arr = np.zeros(n, dtype=npd)
        for i, v in enumerate(vals):
            if _is_null(v):
                valid[i] = False
            else:
                try:
                    if isinstance(dtype, T.BooleanType):
                        arr[i] = (v.lower() == "true") if isinstance(v, str) else bool(v)
                    elif T.is_integral(dtype):
                        if isinstance(v, (int, np.integer)):
                            arr[i] = int(v)  # exact: no float round trip for 64-bit values
                            continue
                        fv = float(v)
                        if math.isnan(fv):
                            valid[i] = False
                        else:
                            arr[i] = int(fv)
                    else:
                        arr[i] = float(v)
                except (TypeError, ValueError):
                    valid[i] = False
    t = torch.as_tensor(arr).to(device)
    return ColumnData(t, None if valid.all() else torch.as_tensor(valid, device=device), dtype)


def frame_from_pycolumns(session, schema: T.StructType, pycols: Dict[str, Sequence[Any]], row_ids) -> "DataFrame":
    from .dataframe import DataFrame
    dev = session._device
    cols = {}
    n = None
    for f in schema.fields:
        cd = column_from_values(pycols[f.name], f.dataType, dev)
        cols[f.name] = cd
        n = len(cd)
    if n is None:
        n = len(row_ids) if row_ids is not None else 0
    if row_ids is None:
        row_ids = torch.arange(n, dtype=torch.int64, device=dev)
    elif not isinstance(row_ids, torch.Tensor):
        row_ids = torch.as_tensor(np.asarray(row_ids, dtype=np.int64), device=dev)
    return DataFrame(session, schema, cols, n, row_ids.to(dev), dev)


DICT_MIN_ROWS = 32768  # below this a plain object array is as cheap as codes + dictionary


def _string_column(values, dtype) -> ColumnData:
    """A host string column without a per-row Python loop: nulls (None / NaN / NaT) found by
    ``pandas.isna``, non-string values stringified, and — for large columns with few distinct
    values (hospital ids, wards, regions) — dictionary encoding (``DictColumnData``: int32 codes +
    distinct strings), which the group-by, sort, join and take paths use instead of the objects."""
    import pandas as pd
    from .column import DictColumnData
    arr = values if isinstance(values, np.ndarray) and values.dtype == object else np.asarray(
        list(values) if not isinstance(values, list) else values, dtype=object)
    if arr.ndim != 1:  # e.g. a list of equal-length tuples
        out = np.empty(len(values), dtype=object)
        out[:] = list(values)
        arr = out
    n = arr.shape[0]
    null = np.asarray(pd.isna(arr), dtype=bool) if n else np.zeros(0, dtype=bool)
    if pd.api.types.infer_dtype(arr, skipna=True) not in ("string", "empty"):
        arr = arr.copy()
        for i in np.flatnonzero(~null):
            v = arr[i]
            if not isinstance(v, str):
                arr[i] = v.decode() if isinstance(v, (bytes, bytearray)) else str(v)
    valid = None if not null.any() else ~null
    if n >= DICT_MIN_ROWS:
        codes, uniq = pd.factorize(arr, use_na_sentinel=True)
        if 4 * len(uniq) <= n:
            dictionary = np.empty(len(uniq) + 1, dtype=object)
            dictionary[:-1] = np.asarray(uniq, dtype=object)
            dictionary[-1] = None
            return DictColumnData(codes.astype(np.int32), dictionary, valid, dtype)
    if valid is not None:
        arr = arr.copy() if arr is values else arr
        arr[null] = None
    return ColumnData(arr, valid, dtype)


def shard_range(n: int, rank: int, world: int):
    per = n // world
    extra = n - per * world
    start = rank * per + min(rank, extra)
    return start, start + per + (1 if rank < extra else 0)


def rows_round_robin(session, schema: T.StructType, rows: List[Sequence[Any]]):
    """Place small global results (aggregations) on ranks round-robin: row i -> rank i % W."""
    comm = session._comm
    mine = [i for i in range(len(rows)) if i % comm.world_size == comm.rank]
    pycols = {f.name: [rows[i][j] for i in mine] for j, f in enumerate(schema.fields)}
    return frame_from_pycolumns(session, schema, pycols, mine)


def rows_contiguous(session, schema: T.StructType, rows: List[Sequence[Any]], row_ids=None):
    """Place an ordered global row list on ranks in contiguous blocks (keeps global order)."""
    comm = session._comm
    a, b = shard_range(len(rows), comm.rank, comm.world_size)
    pycols = {f.name: [rows[i][j] for i in range(a, b)] for j, f in enumerate(schema.fields)}
    ids = list(range(a, b)) if row_ids is None else row_ids[a:b]
    return frame_from_pycolumns(session, schema, pycols, ids)
