"""SQL data types (pyspark.sql.types-compatible names).

The reference declares its input schema with StructType/StructField over
StringType, TimestampType, IntegerType and DoubleType (ref.py:27, ref.py:64-72).
Each type here also names its *physical* column storage in the sharded frame:
numeric/timestamp columns are torch tensors (HBM-resident on GPU ranks), strings
are host numpy object arrays (dictionary-encodable), vectors are dense 2-D tensors.
"""
from __future__ import annotations

import datetime as _dt
import json
from typing import Any, Dict, Iterable, List, Optional

import numpy as np
import torch


class DataType:
    torch_dtype: Optional[torch.dtype] = None
    host_only = False

    def simpleString(self) -> str:
        return self.typeName()

    @classmethod
    def typeName(cls) -> str:
        return cls.__name__[:-4].lower()

    def jsonValue(self):
        return self.typeName()

    def json(self) -> str:
        return json.dumps(self.jsonValue(), separators=(",", ":"), sort_keys=True)

    def __repr__(self) -> str:
        return f"{type(self).__name__}()"

    def __eq__(self, other) -> bool:
        return type(self) is type(other)

    def __hash__(self) -> int:
        return hash(type(self).__name__)


class NullType(DataType):
    @classmethod
    def typeName(cls):
        return "void"


class StringType(DataType):
    host_only = True


class BinaryType(DataType):
    host_only = True


class BooleanType(DataType):
    torch_dtype = torch.bool


class ByteType(DataType):
    torch_dtype = torch.int8

    def simpleString(self):
        return "tinyint"


class ShortType(DataType):
    torch_dtype = torch.int16

    def simpleString(self):
        return "smallint"


class IntegerType(DataType):
    torch_dtype = torch.int32

    def simpleString(self):
        return "int"


class LongType(DataType):
    torch_dtype = torch.int64

    def simpleString(self):
        return "bigint"


class FloatType(DataType):
    torch_dtype = torch.float32


class DoubleType(DataType):
    torch_dtype = torch.float64


class TimestampType(DataType):
    """Microseconds since the Unix epoch (UTC), int64 — Spark's physical representation."""
    torch_dtype = torch.int64


class DateType(DataType):
    """Days since the Unix epoch, int32."""
    torch_dtype = torch.int32


class VectorUDT(DataType):
    """pyspark.ml.linalg.VectorUDT: stored as a dense [n, d] tensor column."""

    @classmethod
    def typeName(cls):
        return "vector"

    def simpleString(self):
        return "vector"

    def jsonValue(self):
        return {"type": "udt", "class": "org.apache.spark.ml.linalg.VectorUDT",
                "pyClass": "pyspark.ml.linalg.VectorUDT",
                "sqlType": {"type": "struct", "fields": [
                    {"name": "type", "type": "byte", "nullable": False, "metadata": {}},
                    {"name": "size", "type": "integer", "nullable": True, "metadata": {}},
                    {"name": "indices", "type": {"type": "array", "elementType": "integer", "containsNull": False},
                     "nullable": True, "metadata": {}},
                    {"name": "values", "type": {"type": "array", "elementType": "double", "containsNull": False},
                     "nullable": True, "metadata": {}}]}}


class MatrixUDT(DataType):
    """pyspark.ml.linalg.MatrixUDT: host column of DenseMatrix objects (statistics results)."""
    host_only = True

    @classmethod
    def typeName(cls):
        return "matrix"

    def simpleString(self):
        return "matrix"


class ArrayType(DataType):
    host_only = True

    def __init__(self, elementType: DataType, containsNull: bool = True):
        self.elementType = elementType
        self.containsNull = containsNull

    def simpleString(self):
        return f"array<{self.elementType.simpleString()}>"

    def jsonValue(self):
        return {"type": "array", "elementType": self.elementType.jsonValue(), "containsNull": self.containsNull}

    def __eq__(self, other):
        return isinstance(other, ArrayType) and other.elementType == self.elementType

    def __hash__(self):
        return hash(("array", self.elementType))


class MapType(DataType):
    host_only = True

    def __init__(self, keyType: DataType, valueType: DataType, valueContainsNull: bool = True):
        self.keyType, self.valueType, self.valueContainsNull = keyType, valueType, valueContainsNull

    def simpleString(self):
        return f"map<{self.keyType.simpleString()},{self.valueType.simpleString()}>"

    def jsonValue(self):
        return {"type": "map", "keyType": self.keyType.jsonValue(), "valueType": self.valueType.jsonValue(),
                "valueContainsNull": self.valueContainsNull}

    def __eq__(self, other):
        return isinstance(other, MapType) and (other.keyType, other.valueType) == (self.keyType, self.valueType)

    def __hash__(self):
        return hash(("map", self.keyType, self.valueType))


class DecimalType(DataType):
    """Fixed-point decimal; computed as float64 on the device (precision/scale kept for the schema)."""
    torch_dtype = torch.float64

    def __init__(self, precision: int = 10, scale: int = 0):
        self.precision, self.scale = precision, scale

    def simpleString(self):
        return f"decimal({self.precision},{self.scale})"

    def jsonValue(self):
        return self.simpleString()

    def __eq__(self, other):
        return isinstance(other, DecimalType) and (other.precision, other.scale) == (self.precision, self.scale)

    def __hash__(self):
        return hash(("decimal", self.precision, self.scale))


class StructField:
    def __init__(self, name: str, dataType: DataType, nullable: bool = True, metadata: Optional[Dict] = None):
        self.name = name
        self.dataType = dataType
        self.nullable = nullable
        self.metadata = metadata or {}

    def simpleString(self) -> str:
        return f"{self.name}:{self.dataType.simpleString()}"

    def jsonValue(self):
        return {"name": self.name, "type": self.dataType.jsonValue(), "nullable": self.nullable,
                "metadata": self.metadata}

    def __repr__(self):
        return f"StructField('{self.name}', {self.dataType!r}, {self.nullable})"

    def __eq__(self, other):
        return (isinstance(other, StructField) and self.name == other.name and self.dataType == other.dataType
                and self.nullable == other.nullable)


class StructType(DataType):
    def __init__(self, fields: Optional[Iterable[StructField]] = None):
        self.fields: List[StructField] = list(fields or [])

    def add(self, field, data_type: Optional[DataType] = None, nullable: bool = True, metadata=None):
        if isinstance(field, StructField):
            self.fields.append(field)
        else:
            self.fields.append(StructField(field, data_type, nullable, metadata))
        return self

    @property
    def names(self) -> List[str]:
        return [f.name for f in self.fields]

    def fieldNames(self) -> List[str]:
        return self.names

    def __getitem__(self, key):
        if isinstance(key, int):
            return self.fields[key]
        for f in self.fields:
            if f.name == key:
                return f
        raise KeyError(key)

    def __iter__(self):
        return iter(self.fields)

    def __len__(self):
        return len(self.fields)

    def simpleString(self):
        return "struct<" + ",".join(f.simpleString() for f in self.fields) + ">"

    def jsonValue(self):
        return {"type": "struct", "fields": [f.jsonValue() for f in self.fields]}

    def treeString(self) -> str:
        lines = ["root"]
        for f in self.fields:
            lines.append(f" |-- {f.name}: {f.dataType.simpleString()} (nullable = {str(f.nullable).lower()})")
        return "\n".join(lines) + "\n"

    def __repr__(self):
        return f"StructType([{', '.join(repr(f) for f in self.fields)}])"

    def __eq__(self, other):
        return isinstance(other, StructType) and self.fields == other.fields

    def __hash__(self):
        return hash(tuple(f.name for f in self.fields))


_SIMPLE = {
    "string": StringType, "int": IntegerType, "integer": IntegerType, "bigint": LongType, "long": LongType,
    "double": DoubleType, "float": FloatType, "boolean": BooleanType, "timestamp": TimestampType,
    "date": DateType, "smallint": ShortType, "short": ShortType, "tinyint": ByteType, "byte": ByteType,
    "binary": BinaryType, "vector": VectorUDT, "void": NullType,
}


def _split_top(s: str, sep: str = ",") -> List[str]:
    """Split on ``sep`` outside <...> / (...) nesting."""
    out, depth, cur = [], 0, []
    for ch in s:
        if ch in "<(":
            depth += 1
        elif ch in ">)":
            depth -= 1
        if ch == sep and depth == 0:
            out.append("".join(cur))
            cur = []
        else:
            cur.append(ch)
    out.append("".join(cur))
    return [p.strip() for p in out if p.strip()]


def _name_type(part: str):
    """'name TYPE' / 'name: TYPE' / '`na me` TYPE' -> (name, type string)."""
    part = part.strip()
    if part.startswith("`"):
        end = part.index("`", 1)
        name, rest = part[1:end], part[end + 1:]
    else:
        i = 0
        while i < len(part) and not part[i].isspace() and part[i] != ":":
            i += 1
        name, rest = part[:i], part[i:]
    rest = rest.strip()
    if rest.startswith(":"):
        rest = rest[1:].strip()
    # drop trailing column constraints / comments
    up = rest.upper()
    for kw in (" NOT NULL", " COMMENT "):
        j = up.find(kw)
        if j >= 0:
            rest, up = rest[:j], up[:j]
    return name, rest.strip()


def parse_type(s) -> DataType:
    """Spark SQL type strings: simple names, decimal(p,s), array<T>, map<K,V>, struct<a:T,...>."""
    if isinstance(s, DataType):
        return s
    t = str(s).strip()
    low = t.lower()
    if low.startswith("array<") and low.endswith(">"):
        return ArrayType(parse_type(t[6:-1]))
    if low.startswith("map<") and low.endswith(">"):
        kv = _split_top(t[4:-1])
        if len(kv) != 2:
            raise ValueError(f"bad map type {s!r}")
        return MapType(parse_type(kv[0]), parse_type(kv[1]))
    if low.startswith("struct<") and low.endswith(">"):
        st = StructType()
        for part in _split_top(t[7:-1]):
            name, typ = _name_type(part)
            st.add(name, parse_type(typ))
        return st
    if low.startswith("decimal") or low.startswith("numeric") or low.startswith("dec"):
        if "(" in low:
            args = [int(x) for x in low[low.index("(") + 1:low.rindex(")")].split(",")]
            return DecimalType(*args)
        return DecimalType()
    if low in _SIMPLE:
        return _SIMPLE[low]()
    if low.startswith("varchar") or low.startswith("char"):
        return StringType()
    raise ValueError(f"unknown type {s!r}")


def parse_ddl_schema(ddl: str) -> StructType:
    """'a INT, b DOUBLE, c ARRAY<STRING>, d STRUCT<x: INT, y: MAP<STRING, DOUBLE>>' -> StructType."""
    st = StructType()
    for part in _split_top(ddl):
        name, typ = _name_type(part)
        st.add(name, parse_type(typ), nullable="NOT NULL" not in part.upper())
    return st


def is_numeric(t: DataType) -> bool:
    return isinstance(t, (ByteType, ShortType, IntegerType, LongType, FloatType, DoubleType, DecimalType))


def is_integral(t: DataType) -> bool:
    return isinstance(t, (ByteType, ShortType, IntegerType, LongType))


def infer_type(values: Any) -> DataType:
    """Infer a column type from a numpy array / list of python values."""
    arr = np.asarray(values, dtype=object) if not isinstance(values, np.ndarray) else values
    if isinstance(arr, np.ndarray) and arr.dtype != object:
        k = arr.dtype.kind
        if k == "b":
            return BooleanType()
        if k in "iu":
            return LongType() if arr.dtype.itemsize >= 8 else IntegerType()
        if k == "f":
            return DoubleType() if arr.dtype.itemsize >= 8 else FloatType()
        if k == "M":
            return TimestampType()
        if k in "US":
            return StringType()
    for v in arr:
        if v is None or (isinstance(v, float) and np.isnan(v)):
            continue
        if isinstance(v, bool):
            return BooleanType()
        if isinstance(v, (int, np.integer)):
            return LongType()
        if isinstance(v, (float, np.floating)):
            return DoubleType()
        if isinstance(v, (_dt.datetime, np.datetime64)):
            return TimestampType()
        if isinstance(v, _dt.date):
            return DateType()
        if isinstance(v, str):
            return StringType()
        if hasattr(v, "toArray"):
            return VectorUDT()
        if isinstance(v, (list, tuple, np.ndarray)):
            return ArrayType(DoubleType())
        return StringType()
    return StringType()


class Row(tuple):
    """pyspark.sql.Row: a tuple with named fields."""

    def __new__(cls, *args, **kwargs):
        if kwargs and args:
            raise ValueError("Row takes positional or keyword arguments, not both")
        if kwargs:
            row = tuple.__new__(cls, list(kwargs.values()))
            row.__fields__ = list(kwargs.keys())
            return row
        row = tuple.__new__(cls, args)
        row.__fields__ = None
        return row

    @classmethod
    def _make(cls, fields, values):
        row = tuple.__new__(cls, values)
        row.__fields__ = list(fields)
        return row

    def asDict(self, recursive: bool = False) -> Dict[str, Any]:
        if self.__fields__ is None:
            raise TypeError("Row has no field names")
        return dict(zip(self.__fields__, self))

    def __getattr__(self, item):
        if item.startswith("__"):
            raise AttributeError(item)
        fields = self.__dict__.get("__fields__")
        if fields and item in fields:
            return self[fields.index(item)]
        raise AttributeError(item)

    def __getitem__(self, item):
        if isinstance(item, str):
            return tuple.__getitem__(self, self.__fields__.index(item))
        return tuple.__getitem__(self, item)

    def __contains__(self, item):
        return self.__fields__ is not None and item in self.__fields__

    def __repr__(self):
        if self.__fields__:
            return "Row(" + ", ".join(f"{k}={v!r}" for k, v in zip(self.__fields__, self)) + ")"
        return "<Row(" + ", ".join(repr(v) for v in self) + ")>"

    def __reduce__(self):
        return (Row._make, (self.__fields__ or [], tuple(self)))
