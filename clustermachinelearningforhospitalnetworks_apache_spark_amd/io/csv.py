"""CSV source (spark.read.csv / readStream.csv, ref.py:75-78) on the native host parser.

Files are split over ranks (whole files round-robin when there are at least as many
files as ranks, otherwise record ranges of each file); every row gets the global
id ``(file_index << 40) | record_index`` so results do not depend on the rank count.
"""
from __future__ import annotations

import ctypes
import os
from typing import Dict, List, Optional, Sequence

import numpy as np
import torch

from .. import _native
from .._native import c_int, c_ll, c_vp
from ..sql import types as T
from ..sql.builder import column_from_values, shard_range
from ..sql.column import ColumnData, DictColumnData

_native.register_host_sigs({
    "cml_csv_index": (c_ll, [ctypes.c_char_p, c_ll, ctypes.c_char, c_int, c_vp, c_ll]),
    "cml_csv_index_mt": (c_ll, [ctypes.c_char_p, c_ll, ctypes.c_char, c_int, c_vp, c_ll, c_int]),
    "cml_csv_gather_strings": (c_ll, [ctypes.c_char_p, c_vp, c_vp, c_ll, ctypes.c_char, c_vp, c_vp]),
    "cml_dict_build": (c_vp, [ctypes.c_char_p, c_vp, c_vp, c_ll, ctypes.c_char, c_int]),
    "cml_dict_size": (None, [c_vp, c_vp, c_vp]),
    "cml_dict_fill": (None, [c_vp, c_vp, c_vp, c_vp]),
    "cml_dict_free": (None, [c_vp]),
    "cml_csv_parse": (c_int, [ctypes.c_char_p, c_ll, c_vp, c_ll, c_int, ctypes.c_char, ctypes.c_char, c_vp, c_vp,
                              c_vp, c_int]),
})

_TYPE_CODE = {T.StringType: 0, T.IntegerType: 1, T.LongType: 2, T.DoubleType: 3, T.TimestampType: 4,
              T.BooleanType: 5, T.FloatType: 6, T.DateType: 7, T.ShortType: 1, T.ByteType: 1}


def _code(dt: T.DataType) -> int:
    return _TYPE_CODE.get(type(dt), 0)


def _np_dtype(code: int):
    return {0: np.int64, 1: np.int32, 2: np.int64, 3: np.float64, 4: np.int64, 5: np.uint8, 6: np.float32,
            7: np.int32}[code]


def parse_csv_bytes(buf: bytes, schema: T.StructType, header: bool, sep: str = ",", quote: str = '"',
                    rows: Optional[slice] = None, nthreads: Optional[int] = None, dicts: Optional[dict] = None):
    """Parse a CSV image into host arrays: {name: (values np.ndarray, valid np.ndarray)}, nrecords.
    Low-cardinality string columns are dictionary-encoded (values share one str object per
    distinct string); with ``dicts`` given, it receives {name: (int32 codes, dictionary)} for them."""
    lib = _native.host()
    starts = record_starts(buf, header, quote, nthreads)
    if rows is not None:
        starts = starts[rows]
    n = int(starts.shape[0])
    ncols = len(schema.fields)
    codes = np.array([_code(f.dataType) for f in schema.fields], dtype=np.int32)
    # string columns get (offset, length, escaped) triples, read only for valid rows: no zero-fill
    datas = [np.empty(n * 3, dtype=np.int64) if c == 0 else np.zeros(n, dtype=_np_dtype(c)) for c in codes]
    valids = [np.zeros(max(n, 1), dtype=np.uint8) for _ in codes]
    dptr = (ctypes.c_void_p * ncols)(*[d.ctypes.data for d in datas])
    vptr = (ctypes.c_void_p * ncols)(*[v.ctypes.data for v in valids])
    if n:
        nthreads = nthreads or host_threads()
        st = lib.cml_csv_parse(buf, len(buf), starts.ctypes.data, n, ncols, sep.encode(), quote.encode(),
                               codes.ctypes.data, dptr, vptr, nthreads)
        if st != 0:
            raise RuntimeError("CSV parse failed")
    out = {}
    for f, c, d, v in zip(schema.fields, codes, datas, valids):
        valid = v[:n].view(bool)  # 0/1 bytes: a zero-copy bool view
        if c == 0:
            enc = _dictionary(lib, buf, d, v, n, quote, nthreads)
            if enc is None:
                out[f.name] = (_strings(lib, buf, d, v, n, quote), valid)
            else:
                codes, dictionary = enc
                out[f.name] = (None, valid)  # values are built lazily from the dictionary
                if dicts is not None:
                    dicts[f.name] = enc
                else:
                    out[f.name] = (np.append(dictionary, None)[codes], valid)
        elif c == 5:
            out[f.name] = (d[:n].view(bool), valid)
        else:
            out[f.name] = (d[:n], valid)
    return out, n


def record_starts(buf: bytes, header: bool, quote: str = '"', nthreads: Optional[int] = None) -> np.ndarray:
    """Byte offsets of the records (one multithreaded native pass). A record takes at least two
    bytes with its newline, so len/2 + 1 entries always suffice; the untouched tail of the
    allocation is never paged in."""
    cap = len(buf) // 2 + 2
    starts = np.empty(cap, dtype=np.int64)
    nthreads = nthreads or host_threads()
    n = _native.host().cml_csv_index_mt(buf, len(buf), quote.encode(), 1 if header else 0, starts.ctypes.data, cap,
                                         nthreads)
    return starts[:n].copy()


_DICT_SAMPLE = 16384


def host_threads() -> int:
    """Worker threads for the native parser: the CPUs this process may run on (cgroup / affinity),
    bounded by OMP_NUM_THREADS when set and by 16."""
    try:
        n = len(os.sched_getaffinity(0))
    except AttributeError:
        n = os.cpu_count() or 1
    env = os.environ.get("OMP_NUM_THREADS")
    if env and env.isdigit() and int(env) > 0:
        n = min(n, int(env))
    return max(1, min(16, n))


_ARROW_CAPPED = False


def cap_arrow_threads() -> None:
    """Size Arrow's CPU and IO thread pools to this process's CPU share (``host_threads``) once. Arrow
    sizes them from the machine's CPU count; on a GPU box that is many times the process's share, and
    a Parquet write that spreads its compression over all of them exhausts the cgroup's CPU quota
    and stalls every thread of the process, the GPU-feeding one included."""
    global _ARROW_CAPPED
    if _ARROW_CAPPED:
        return
    import pyarrow as pa
    n = host_threads()
    if pa.cpu_count() > n:
        pa.set_cpu_count(n)
    if pa.io_thread_count() > n:
        pa.set_io_thread_count(n)
    _ARROW_CAPPED = True


def _dict_run(lib, buf, trip, valid_u8, n, quote, nthreads):
    h = lib.cml_dict_build(buf, trip.ctypes.data, valid_u8.ctypes.data, n, quote.encode(), nthreads)
    try:
        cnt, nb = ctypes.c_longlong(), ctypes.c_longlong()
        lib.cml_dict_size(h, ctypes.byref(cnt), ctypes.byref(nb))
        codes = np.empty(n, dtype=np.int32)
        offsets = np.empty(cnt.value + 1, dtype=np.int64)
        data = np.empty(max(nb.value, 1), dtype=np.uint8)
        lib.cml_dict_fill(h, codes.ctypes.data, offsets.ctypes.data, data.ctypes.data)
    finally:
        lib.cml_dict_free(h)
    return codes, offsets, data, cnt.value


def _dictionary(lib, buf: bytes, trip: np.ndarray, valid_u8: np.ndarray, n: int, quote: str,
                nthreads: Optional[int]):
    """(int32 codes with -1 for null, object array of the distinct strings in first-appearance
    order) when the column looks low-cardinality on a leading sample, else None. The native
    encoder hashes row blocks on several threads and merges the block dictionaries, so only one
    Python str per distinct value is ever created."""
    import pyarrow as pa
    if n < 2 * _DICT_SAMPLE:
        return None
    nthreads = nthreads or host_threads()
    _, _, _, k = _dict_run(lib, buf, trip, valid_u8, _DICT_SAMPLE, quote, 1)
    if k > _DICT_SAMPLE // 4:
        return None
    codes, offsets, data, k = _dict_run(lib, buf, trip, valid_u8, n, quote, nthreads)
    if k > n // 4:
        return None
    arr = pa.LargeStringArray.from_buffers(k, pa.py_buffer(offsets), pa.py_buffer(data))
    return codes, arr.to_numpy(zero_copy_only=False)


def merge_dictionaries(parts):
    """Concatenate per-chunk (codes, dictionary) into one code space (first-appearance order):
    (int32 codes, object array of the distinct strings)."""
    if len(parts) == 1:
        return parts[0][0], np.asarray(parts[0][1], dtype=object)
    index: Dict[str, int] = {}
    out = []
    for codes, dictionary in parts:
        remap = np.empty(len(dictionary) + 1, dtype=np.int32)
        for i, v in enumerate(dictionary):
            remap[i] = index.setdefault(v, len(index))
        remap[-1] = -1
        out.append(remap[codes])
    merged = np.empty(len(index), dtype=object)
    for v, i in index.items():
        merged[i] = v
    return (np.concatenate(out) if out else np.zeros(0, dtype=np.int32)), merged


def _strings(lib, buf: bytes, trip: np.ndarray, valid_u8: np.ndarray, n: int, quote: str) -> np.ndarray:
    """Object array of str (None for nulls): the native gather writes one Arrow string buffer,
    Arrow's C++ builds the Python strings — no per-row Python work."""
    import pyarrow as pa
    if n == 0:
        return np.empty(0, dtype=object)
    total = lib.cml_csv_gather_strings(buf, trip.ctypes.data, valid_u8.ctypes.data, n, quote.encode(), None, None)
    offsets = np.zeros(n + 1, dtype=np.int64)
    data = np.zeros(max(total, 1), dtype=np.uint8)
    lib.cml_csv_gather_strings(buf, trip.ctypes.data, valid_u8.ctypes.data, n, quote.encode(), offsets.ctypes.data,
                               data.ctypes.data)
    mask = pa.array(valid_u8[:n].astype(bool)).buffers()[1]
    arr = pa.LargeStringArray.from_buffers(n, pa.py_buffer(offsets), pa.py_buffer(data), mask)
    return arr.to_numpy(zero_copy_only=False)


def header_names(buf: bytes, sep: str = ",", quote: str = '"') -> List[str]:
    line = buf.split(b"\n", 1)[0].decode("utf-8", "replace").rstrip("\r")
    import csv as _csv
    return [c.strip() for c in next(_csv.reader([line], delimiter=sep, quotechar=quote))]


def infer_schema(buf: bytes, header: bool, sep: str, quote: str, infer: bool, sample: int = 1000) -> T.StructType:
    names = header_names(buf, sep, quote)
    if not header:
        names = [f"_c{i}" for i in range(len(names))]
    st = T.StructType([T.StructField(n, T.StringType()) for n in names])
    if not infer:
        return st
    parsed, n = parse_csv_bytes(buf, st, header, sep, quote, rows=slice(0, sample))
    fields = []
    for name in names:
        vals, valid = parsed[name]
        fields.append(T.StructField(name, _infer_from_strings([v for v, ok in zip(vals, valid) if ok])))
    return T.StructType(fields)


def _infer_from_strings(vals: List[str]) -> T.DataType:
    from ..sql.column import ts_to_micros
    if not vals:
        return T.StringType()

    def all_ok(fn):
        try:
            for v in vals:
                fn(v)
            return True
        except (ValueError, TypeError):
            return False

    if all_ok(lambda v: int(v) if -2**31 <= int(v) < 2**31 else (_ for _ in ()).throw(ValueError())):
        return T.IntegerType()
    if all_ok(int):
        return T.LongType()
    if all_ok(float):
        return T.DoubleType()
    if all(v.lower() in ("true", "false") for v in vals):
        return T.BooleanType()
    if all_ok(ts_to_micros):
        return T.TimestampType()
    return T.StringType()


def read_csv_files(session, paths: Sequence[str], schema: Optional[T.StructType], header: bool, sep: str = ",",
                   quote: str = '"', infer: bool = False, file_index_base: int = 0,
                   file_ids: Optional[Sequence[int]] = None):
    """Read CSV files into this rank's shard. Returns a DataFrame."""
    from ..sql.builder import frame_from_pycolumns
    comm = session._comm
    W, rank = comm.world_size, comm.rank
    paths = list(paths)
    if schema is None:
        if not paths:
            raise ValueError("cannot infer a schema without input files; pass .schema(...)")
        with open(paths[0], "rb") as fh:
            schema = infer_schema(fh.read(1 << 20), header, sep, quote, infer)
    fids = list(file_ids) if file_ids is not None else [file_index_base + i for i in range(len(paths))]
    whole_files = len(paths) >= W
    cols: Dict[str, List] = {f.name: [] for f in schema.fields}
    valids: Dict[str, List] = {f.name: [] for f in schema.fields}
    encs: Dict[str, List] = {f.name: [] for f in schema.fields}
    ids: List[np.ndarray] = []
    for i, (p, fid) in enumerate(zip(paths, fids)):
        if whole_files and i % W != rank:
            continue
        with open(p, "rb") as fh:
            buf = fh.read()
        if whole_files:
            sl = None
        else:
            n_all = int(record_starts(buf, header, quote).shape[0])
            a, b = shard_range(n_all, rank, W)
            sl = slice(a, b)
        dicts: Dict[str, tuple] = {}
        parsed, n = parse_csv_bytes(buf, schema, header, sep, quote, rows=sl, dicts=dicts)
        start = 0 if sl is None else sl.start
        ids.append((np.int64(fid) << np.int64(40)) + np.arange(start, start + n, dtype=np.int64))
        for f in schema.fields:
            v, ok = parsed[f.name]
            cols[f.name].append(v)
            valids[f.name].append(ok)
            encs[f.name].append(dicts.get(f.name))
    dev = session._device
    from ..sql.dataframe import DataFrame
    out_cols = {}
    n_total = int(sum(a.shape[0] for a in ids)) if ids else 0
    for f in schema.fields:
        if encs[f.name] and all(e is not None for e in encs[f.name]):
            codes, dictionary = merge_dictionaries(encs[f.name])
            ok = np.concatenate(valids[f.name]) if len(valids[f.name]) > 1 else valids[f.name][0]
            out_cols[f.name] = DictColumnData(codes, np.append(dictionary, None), None if ok.all() else ok,
                                              f.dataType)
            continue
        if any(v is None for v in cols[f.name]):  # mixed chunks: materialise the encoded ones
            cols[f.name] = [np.append(e[1], None)[e[0]] if v is None else v
                            for v, e in zip(cols[f.name], encs[f.name])]
        if len(cols[f.name]) == 1:
            vals, ok = cols[f.name][0], valids[f.name][0]
        elif cols[f.name]:
            vals = np.concatenate(cols[f.name])
            ok = np.concatenate(valids[f.name])
        else:
            vals = np.zeros(0, dtype=object if isinstance(f.dataType, T.StringType) else np.float64)
            ok = np.zeros(0, dtype=bool)
        out_cols[f.name] = _to_column(vals, ok, f.dataType, dev)
    rid = torch.as_tensor(np.concatenate(ids) if ids else np.zeros(0, dtype=np.int64), device=dev)
    return DataFrame(session, schema, out_cols, n_total, rid, dev)


def _to_column(vals: np.ndarray, ok: np.ndarray, dt: T.DataType, dev) -> ColumnData:
    if isinstance(dt, (T.StringType, T.BinaryType)) or dt.torch_dtype is None:
        return ColumnData(vals if vals.dtype == object else vals.astype(object), None if ok.all() else ok, dt)
    t = torch.as_tensor(np.ascontiguousarray(vals)).to(device=dev, dtype=dt.torch_dtype)
    valid = None if ok.all() else torch.as_tensor(ok, device=dev)
    return ColumnData(t, valid, dt)
