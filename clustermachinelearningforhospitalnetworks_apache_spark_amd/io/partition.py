"""Hive-style directory partitioning (``col=value/``): partitioned writes for ``df.write.partitionBy``
and partition discovery on read, as Spark does (values typed int / long / double / string, the
null value spelled ``__HIVE_DEFAULT_PARTITION__``)."""
from __future__ import annotations

import os
from typing import Dict, List, Optional, Sequence, Tuple
from urllib.parse import quote, unquote

from ..sql import types as T

NULL_PART = "__HIVE_DEFAULT_PARTITION__"


def encode_value(v) -> str:
    if v is None:
        return NULL_PART
    if isinstance(v, bool):
        return "true" if v else "false"
    return quote(str(v), safe=" -_.:")


def partitions_of(path: str, base: str) -> Dict[str, str]:
    """``{col: raw value}`` from the ``col=value`` directories between ``base`` and the file."""
    rel = os.path.relpath(os.path.dirname(path), base)
    out: Dict[str, str] = {}
    if rel in (".", ""):
        return out
    for comp in rel.split(os.sep):
        if "=" in comp:
            k, v = comp.split("=", 1)
            out[k] = unquote(v)
    return out


def infer_types(values: Dict[str, List[str]]) -> Dict[str, T.DataType]:
    out = {}
    for col, vals in values.items():
        vs = [v for v in vals if v != NULL_PART]
        t: T.DataType = T.StringType()
        try:
            ints = [int(v) for v in vs]
            t = T.IntegerType() if all(-2**31 <= x < 2**31 for x in ints) else T.LongType()
        except ValueError:
            try:
                [float(v) for v in vs]
                t = T.DoubleType()
            except ValueError:
                t = T.StringType()
        out[col] = t
    return out


def typed(v: str, t: T.DataType):
    if v == NULL_PART:
        return None
    if isinstance(t, (T.IntegerType, T.LongType)):
        return int(v)
    if isinstance(t, T.DoubleType):
        return float(v)
    return v


def discover(files: Sequence[str], bases: Sequence[str]) -> Tuple[List[Dict[str, str]], Dict[str, T.DataType]]:
    """Per file its partition dict (relative to the first base that contains it) + inferred types."""
    parts = []
    for f in files:
        base = next((b for b in bases if os.path.commonpath([os.path.abspath(b), os.path.abspath(f)]) ==
                     os.path.abspath(b)), os.path.dirname(f))
        parts.append(partitions_of(f, base))
    cols: Dict[str, List[str]] = {}
    for p in parts:
        for k, v in p.items():
            cols.setdefault(k, []).append(v)
    return parts, infer_types(cols)


def read_partitioned(session, files: Sequence[str], bases: Sequence[str], reader):
    """``reader(files, file_ids)`` per group of files sharing partition values; partition columns are
    appended as literals and the groups unioned. Returns None when nothing is partitioned."""
    from ..sql import functions as F
    parts, types = discover(files, bases)
    if not types:
        return None
    groups: Dict[tuple, List[int]] = {}
    for i, p in enumerate(parts):
        groups.setdefault(tuple(sorted(p.items())), []).append(i)
    frames = []
    for key, idx in sorted(groups.items()):
        df = reader([files[i] for i in idx], idx)
        pd_ = dict(key)
        for col, t in types.items():
            v = typed(pd_[col], t) if col in pd_ else None
            df = df.withColumn(col, F.lit(v).cast(t))
        frames.append(df)
    out = frames[0]
    for fr in frames[1:]:
        out = out.unionByName(fr)
    return out


def write_partitioned(df, path: str, cols: Sequence[str], write_one) -> None:
    """Rows grouped by the partition columns' values; ``write_one(sub_frame, directory)`` writes one
    group (without the partition columns) into ``path/c1=v1/c2=v2``."""
    import torch
    from ..sql.dataframe import column_to_python
    vals = [column_to_python(df._column_data(c)) for c in cols]
    keys = list(zip(*vals)) if vals else []
    local = sorted(set(keys), key=lambda k: tuple(str(x) for x in k))
    allkeys = []
    for part in df._comm.allgather_object(local):
        for k in part:
            if k not in allkeys:
                allkeys.append(k)
    rest = [c for c in df.columns if c not in cols]
    for key in sorted(allkeys, key=lambda k: tuple(str(x) for x in k)):
        mask = torch.as_tensor([k == key for k in keys], dtype=torch.bool, device=df._device) if keys else \
            torch.zeros(0, dtype=torch.bool, device=df._device)
        sub = df._mask_rows(mask).select(*rest)
        d = os.path.join(path, *[f"{c}={encode_value(v)}" for c, v in zip(cols, key)])
        write_one(sub, d)
