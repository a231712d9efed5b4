"""Tagged JSON codec for checkpointed Python state (streaming operator state).

Checkpoint directories live on shared storage (the reference's is an HDFS path, ref.py:43), so a
state file must never be able to run code when a query restarts: no pickle. Values are written as
JSON with explicit tags for what JSON cannot hold natively, and decoding only ever builds these types:

    tuple {"$t": [...]}         Row {"$row": [fields | null, [...]]}   dict {"$d": [[k, v], ...]}
    set {"$s": [...]}           frozenset {"$fs": [...]}               float NaN/±inf {"$f": "nan"}
    datetime {"$dt": iso}       date {"$date": iso}                    timedelta {"$td": microseconds}
    Decimal {"$dec": str}       bytes {"$b": base64}                   numpy array {"$nd": [dtype, shape, data]}

Dict keys may be any encodable value (tuples of group keys). Anything else raises TypeError, so a
new kind of state fails at save time instead of silently round-tripping wrong.
"""
from __future__ import annotations

import base64
import datetime as _dt
import json
import math
from decimal import Decimal
from typing import Any

import numpy as np


def encode(obj: Any) -> Any:
    from ..sql.types import Row
    if obj is None or isinstance(obj, (bool, str)):
        return obj
    if isinstance(obj, (int, np.integer)) and not isinstance(obj, bool):
        return int(obj)
    if isinstance(obj, (float, np.floating)):
        f = float(obj)
        if math.isnan(f):
            return {"$f": "nan"}
        if math.isinf(f):
            return {"$f": "inf" if f > 0 else "-inf"}
        return f
    if isinstance(obj, np.bool_):
        return bool(obj)
    if isinstance(obj, Row):
        return {"$row": [getattr(obj, "__fields__", None), [encode(v) for v in obj]]}
    if isinstance(obj, tuple):
        return {"$t": [encode(v) for v in obj]}
    if isinstance(obj, list):
        return [encode(v) for v in obj]
    if isinstance(obj, dict):
        return {"$d": [[encode(k), encode(v)] for k, v in obj.items()]}
    if isinstance(obj, frozenset):
        return {"$fs": [encode(v) for v in obj]}
    if isinstance(obj, set):
        return {"$s": [encode(v) for v in obj]}
    if isinstance(obj, _dt.datetime):
        return {"$dt": obj.isoformat()}
    if isinstance(obj, _dt.date):
        return {"$date": obj.isoformat()}
    if isinstance(obj, _dt.timedelta):
        return {"$td": (obj.days * 86400 + obj.seconds) * 1_000_000 + obj.microseconds}
    if isinstance(obj, Decimal):
        return {"$dec": str(obj)}
    if isinstance(obj, (bytes, bytearray)):
        return {"$b": base64.b64encode(bytes(obj)).decode("ascii")}
    if isinstance(obj, np.ndarray):
        if obj.dtype == object:
            raise TypeError("object arrays are not checkpointable state")
        return {"$nd": [obj.dtype.str, list(obj.shape), [encode(v) for v in obj.ravel().tolist()]]}
    raise TypeError(f"cannot checkpoint a value of type {type(obj).__name__}")


def decode(obj: Any) -> Any:
    from ..sql.types import Row
    if isinstance(obj, list):
        return [decode(v) for v in obj]
    if not isinstance(obj, dict):
        return obj
    if len(obj) != 1:
        raise ValueError("malformed state record")
    (tag, val), = obj.items()
    if tag == "$t":
        return tuple(decode(v) for v in val)
    if tag == "$row":
        fields, vals = val
        vals = [decode(v) for v in vals]
        return Row._make(fields, vals) if fields is not None else Row(*vals)
    if tag == "$d":
        return {_hashable(decode(k)): decode(v) for k, v in val}
    if tag == "$s":
        return {_hashable(decode(v)) for v in val}
    if tag == "$fs":
        return frozenset(_hashable(decode(v)) for v in val)
    if tag == "$f":
        return {"nan": math.nan, "inf": math.inf, "-inf": -math.inf}[val]
    if tag == "$dt":
        return _dt.datetime.fromisoformat(val)
    if tag == "$date":
        return _dt.date.fromisoformat(val)
    if tag == "$td":
        return _dt.timedelta(microseconds=int(val))
    if tag == "$dec":
        return Decimal(val)
    if tag == "$b":
        return base64.b64decode(val)
    if tag == "$nd":
        dtype, shape, data = val
        return np.asarray([decode(v) for v in data], dtype=np.dtype(dtype)).reshape(shape)
    raise ValueError(f"unknown state tag {tag!r}")


def _hashable(v):
    return tuple(_hashable(x) for x in v) if isinstance(v, list) else v


def dumps(obj: Any) -> str:
    return json.dumps(encode(obj), allow_nan=False, separators=(",", ":"))


def loads(text: str) -> Any:
    return decode(json.loads(text))
