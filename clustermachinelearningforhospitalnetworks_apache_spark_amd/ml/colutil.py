"""Column helpers shared by the ml.feature* modules (kept free of feature-module imports so any of
them can be imported first)."""
from __future__ import annotations

from ..sql import types as T
from ..sql.column import ColumnData


def _replace_col(df, name: str, data: ColumnData):
    """``df`` with column ``name`` replaced (or appended) by ``data``, row ids unchanged."""
    fields = list(df.schema.fields)
    cols = dict(df._cols)
    if name in cols:
        fields[df.schema.names.index(name)] = T.StructField(name, data.dtype, True)
    else:
        fields.append(T.StructField(name, data.dtype, True))
    cols[name] = data
    return df._new(T.StructType(fields), cols, df._nrows, df._row_ids)


def _auto_output(obj) -> None:
    """Spark's default output column: ``<uid>__output``."""
    if obj.getOutputCol() == "__auto__":
        obj._defaultParamMap["outputCol"] = obj.uid + "__output"
