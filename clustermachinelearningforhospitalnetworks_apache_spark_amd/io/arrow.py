"""Arrow / Parquet / JSON interchange for sharded frames (pyarrow, host side)."""
from __future__ import annotations

import datetime as _dt
from typing import List, Optional, Sequence

import numpy as np
import torch

from ..sql import types as T
from ..sql.column import ColumnData


def arrow_type_to_spark(at) -> T.DataType:
    import pyarrow as pa
    if pa.types.is_boolean(at):
        return T.BooleanType()
    if pa.types.is_int8(at):
        return T.ByteType()
    if pa.types.is_int16(at):
        return T.ShortType()
    if pa.types.is_int32(at) or pa.types.is_uint8(at) or pa.types.is_uint16(at):
        return T.IntegerType()
    if pa.types.is_integer(at):
        return T.LongType()
    if pa.types.is_float32(at):
        return T.FloatType()
    if pa.types.is_floating(at):
        return T.DoubleType()
    if pa.types.is_timestamp(at):
        return T.TimestampType()
    if pa.types.is_date(at):
        return T.DateType()
    if pa.types.is_list(at) or pa.types.is_large_list(at) or pa.types.is_fixed_size_list(at):
        return T.VectorUDT() if pa.types.is_floating(at.value_type) else T.ArrayType(arrow_type_to_spark(at.value_type))
    if pa.types.is_struct(at) and {f.name for f in at} >= {"type", "size", "indices", "values"}:
        return T.VectorUDT()
    return T.StringType()


def spark_type_to_arrow(dt: T.DataType):
    import pyarrow as pa
    m = {T.BooleanType: pa.bool_(), T.ByteType: pa.int8(), T.ShortType: pa.int16(), T.IntegerType: pa.int32(),
         T.LongType: pa.int64(), T.FloatType: pa.float32(), T.DoubleType: pa.float64(),
         T.TimestampType: pa.timestamp("us"), T.DateType: pa.date32(), T.StringType: pa.string(),
         T.BinaryType: pa.binary()}
    if isinstance(dt, T.VectorUDT):
        return vector_udt_arrow()
    if isinstance(dt, T.ArrayType):
        return pa.list_(spark_type_to_arrow(dt.elementType))
    return m.get(type(dt), pa.string())


def vector_udt_arrow():
    import pyarrow as pa
    return pa.struct([pa.field("type", pa.int8(), nullable=False), pa.field("size", pa.int32()),
                      pa.field("indices", pa.list_(pa.field("element", pa.int32(), nullable=False))),
                      pa.field("values", pa.list_(pa.field("element", pa.float64(), nullable=False)))])


def vectors_to_arrow(mat: np.ndarray, valid: Optional[np.ndarray] = None):
    """Dense vectors -> VectorUDT struct array (type=1 dense, size/indices null)."""
    import pyarrow as pa
    n = mat.shape[0]
    values = pa.array([row.tolist() for row in mat], type=pa.list_(pa.field("element", pa.float64(), nullable=False)))
    types = pa.array(np.ones(n, dtype=np.int8))
    sizes = pa.array([None] * n, type=pa.int32())
    idx = pa.array([None] * n, type=pa.list_(pa.field("element", pa.int32(), nullable=False)))
    mask = None if valid is None else pa.array(~valid)
    return pa.StructArray.from_arrays([types, sizes, idx, values], fields=list(vector_udt_arrow()), mask=mask)


def column_to_arrow(cd: ColumnData):
    import pyarrow as pa
    from ..sql.dataframe import column_to_python
    if isinstance(cd.dtype, T.VectorUDT):
        mat = cd.values.detach().double().cpu().numpy()
        valid = None if cd.valid is None else cd.valid_mask().cpu().numpy()
        return vectors_to_arrow(mat, valid)
    if cd.is_host and cd.codes is not None and isinstance(cd.dtype, T.StringType):
        # dictionary-encoded strings: codes + one object per distinct value, expanded by Arrow in C++
        codes = np.asarray(cd.codes, dtype=np.int32)
        dict_vals = getattr(cd, "dictionary", None)
        if dict_vals is not None:
            dictionary = pa.array(list(dict_vals[:-1]), type=pa.string())
        else:
            k = int(codes.max(initial=-1)) + 1
            first = np.full(k, -1, dtype=np.int64)
            pos = np.nonzero(codes >= 0)[0]
            first[codes[pos][::-1]] = pos[::-1]
            dictionary = pa.array(list(cd.values[first]) if k else [], type=pa.string())
        idx = pa.array(codes, mask=codes < 0)
        return pa.DictionaryArray.from_arrays(idx, dictionary).cast(pa.string())
    if cd.is_host:
        return pa.array(column_to_python(cd), type=spark_type_to_arrow(cd.dtype))
    arr = cd.values.detach().cpu().numpy()
    mask = None if cd.valid is None else ~cd.valid_mask().cpu().numpy()
    if isinstance(cd.dtype, T.TimestampType):
        return pa.array(arr.astype("datetime64[us]"), type=pa.timestamp("us"), mask=mask)
    if isinstance(cd.dtype, T.DateType):
        return pa.array(arr.astype("datetime64[D]"), type=pa.date32(), mask=mask)
    return pa.array(arr, type=spark_type_to_arrow(cd.dtype), mask=mask)


def frame_to_arrow(df):
    import pyarrow as pa
    arrays = [column_to_arrow(df._cols[f.name]) for f in df.schema.fields]
    fields = [pa.field(f.name, a.type, nullable=f.nullable) for f, a in zip(df.schema.fields, arrays)]
    return pa.Table.from_arrays(arrays, schema=pa.schema(fields))


def arrow_column_to_data(arr, dt: T.DataType, device) -> ColumnData:
    import pyarrow as pa
    if isinstance(arr, pa.ChunkedArray):
        arr = arr.combine_chunks() if arr.num_chunks != 1 else arr.chunk(0)
    n = len(arr)
    valid_np = None
    if arr.null_count:
        valid_np = ~np.asarray(arr.is_null().to_numpy(zero_copy_only=False))
    if isinstance(dt, T.VectorUDT):
        if pa.types.is_struct(arr.type):
            vals = arr.field("values").to_pylist()
            types = arr.field("type").to_pylist()
            sizes = arr.field("size").to_pylist()
            idxs = arr.field("indices").to_pylist()
            d = 0
            for t, s, v in zip(types, sizes, vals):
                if t is not None:
                    d = s if t == 0 else len(v)
                    break
            mat = np.zeros((n, d))
            for i, (t, s, ix, v) in enumerate(zip(types, sizes, idxs, vals)):
                if t is None:
                    continue
                if t == 0:
                    mat[i, ix] = v
                else:
                    mat[i] = v
        else:
            rows = arr.to_pylist()
            d = next((len(r) for r in rows if r is not None), 0)
            mat = np.array([r if r is not None else [0.0] * d for r in rows], dtype=np.float64).reshape(n, d)
        return ColumnData(torch.as_tensor(mat, device=device), None if valid_np is None else torch.as_tensor(
            valid_np, device=device), dt)
    if dt.torch_dtype is None or dt.host_only:
        if isinstance(dt, T.StringType) and pa.types.is_dictionary(arr.type):
            arr = arr.cast(arr.type.value_type)
        if isinstance(dt, T.StringType) and (pa.types.is_string(arr.type) or pa.types.is_large_string(arr.type)):
            from ..sql.builder import DICT_MIN_ROWS
            if n >= DICT_MIN_ROWS:
                # repetitive strings (ids, wards, regions) stay dictionary-encoded: Arrow's hash
                # encoder in C++, then int32 codes + the distinct strings (sql.column.DictColumnData)
                enc = arr.dictionary_encode()
                if 4 * len(enc.dictionary) <= n:
                    from ..sql.column import DictColumnData
                    codes = enc.indices.fill_null(-1).to_numpy(zero_copy_only=False).astype(np.int32)
                    dictionary = np.empty(len(enc.dictionary) + 1, dtype=object)
                    dictionary[:-1] = enc.dictionary.to_numpy(zero_copy_only=False)
                    dictionary[-1] = None
                    return DictColumnData(codes, dictionary, valid_np, dt)
            vals = arr.to_numpy(zero_copy_only=False)  # Arrow builds the str objects in C++
            if vals.dtype != object:
                vals = vals.astype(object)
        else:
            vals = np.array(arr.to_pylist(), dtype=object)
            if isinstance(dt, T.StringType):
                vals = np.array([None if v is None else str(v) for v in vals], dtype=object)
        return ColumnData(vals, valid_np, dt)
    if isinstance(dt, T.TimestampType):
        np_arr = arr.cast(pa.timestamp("us")).cast(pa.int64()).fill_null(0).to_numpy()
    elif isinstance(dt, T.DateType):
        np_arr = arr.cast(pa.int32()).fill_null(0).to_numpy()
    elif isinstance(dt, T.BooleanType):
        np_arr = arr.fill_null(False).to_numpy(zero_copy_only=False).astype(bool)
    else:
        np_arr = arr.fill_null(0).to_numpy(zero_copy_only=False)
    t = torch.as_tensor(np.array(np_arr, copy=True)).to(device=device, dtype=dt.torch_dtype)
    return ColumnData(t, None if valid_np is None else torch.as_tensor(valid_np, device=device), dt)


def frame_from_arrow(session, table, row_ids=None, schema: Optional[T.StructType] = None):
    from ..sql.dataframe import DataFrame
    dev = session._device
    if schema is None:
        schema = T.StructType([T.StructField(f.name, arrow_type_to_spark(f.type), f.nullable) for f in table.schema])
    cols = {f.name: arrow_column_to_data(table.column(f.name), f.dataType, dev) for f in schema.fields}
    n = table.num_rows
    rid = torch.arange(n, dtype=torch.int64, device=dev) if row_ids is None else torch.as_tensor(
        np.asarray(row_ids, dtype=np.int64), device=dev)
    return DataFrame(session, schema, cols, n, rid, dev)


def read_parquet_files(session, paths: Sequence[str], schema: Optional[T.StructType] = None,
                       file_ids: Optional[Sequence[int]] = None):
    """Each rank reads whole files round-robin (or row ranges of a single file)."""
    import pyarrow as pa
    import pyarrow.parquet as pq
    from ..sql.builder import shard_range
    from .csv import cap_arrow_threads
    cap_arrow_threads()
    comm = session._comm
    W, rank = comm.world_size, comm.rank
    paths = list(paths)
    fids = list(file_ids) if file_ids is not None else list(range(len(paths)))
    tables, ids = [], []
    whole = len(paths) >= W
    for i, (p, fid) in enumerate(zip(paths, fids)):
        if whole and i % W != rank:
            continue
        t = pq.read_table(p)
        a, b = (0, t.num_rows) if whole else shard_range(t.num_rows, rank, W)
        t = t.slice(a, b - a)
        tables.append(t)
        ids.append((np.int64(fid) << np.int64(40)) + np.arange(a, b, dtype=np.int64))
    if schema is None:
        if paths:
            sch = pq.read_schema(paths[0])
            schema = T.StructType([T.StructField(f.name, arrow_type_to_spark(f.type), f.nullable) for f in sch])
        else:
            schema = T.StructType()
    if tables:
        tables = [t.select(schema.names) for t in tables]
        table = pa.concat_tables(tables, promote_options="permissive") if len(tables) > 1 else tables[0]
        rid = np.concatenate(ids)
    else:
        table = pa.table({f.name: pa.array([], type=spark_type_to_arrow(f.dataType)) for f in schema.fields})
        rid = np.zeros(0, dtype=np.int64)
    return frame_from_arrow(session, table, rid, schema)
