"""The rest of the DataFrame / GroupedData API a pyspark user reaches for after the reference's
``select`` / ``filter`` / ``na.drop`` (ref.py:123-139): set operations, ``summary`` with
percentiles, ``df.stat`` (approxQuantile, corr, cov, crosstab, freqItems, sampleBy), ``pivot``,
``rollup`` / ``cube``, ``applyInPandas`` / ``mapInPandas``, and no-op hints / checkpoints.

Placement follows the frame's rules: numeric statistics reduce on the device
and all-reduce; operations on whole rows (set operations, pivots, grouped pandas functions) gather
to the host like ``distinct`` / ``join`` do — they serve reference-scale analytics, not the hot
path.
"""
from __future__ import annotations

import math
import re
from typing import Any, Dict, List, Optional, Sequence

import numpy as np
import torch

from . import types as T


def _sstr(v) -> str:
    """Spark's string form of a value (Java toString: null, true / false)."""
    if v is None:
        return "null"
    if isinstance(v, (bool, np.bool_)):
        return "true" if v else "false"
    return str(v)


def _key(row) -> tuple:
    from .group import _hashable
    return tuple(_hashable(v) for v in row)


class DataFrameMoreMixin:
    # ------------------------------------------------------------------------------ set operations
    def _set_op(self, other, keep_fn, kind: str):
        from .builder import rows_contiguous
        from .relational_fast import device_set_op
        if len(other.columns) != len(self.columns):
            raise ValueError("set operations need the same number of columns")
        out = device_set_op(self, other, kind)
        if out is not None:
            return out
        _, left, _ = self._gather_host()
        _, right, _ = other._gather_host()
        rows = keep_fn(left, right)
        return rows_contiguous(self._session, self.schema, rows)

    def intersect(self, other):
        """Distinct rows present in both frames."""
        def f(left, right):
            rk = {_key(r) for r in right}
            seen, out = set(), []
            for r in left:
                k = _key(r)
                if k in rk and k not in seen:
                    seen.add(k)
                    out.append(r)
            return out
        return self._set_op(other, f, "intersect")

    def intersectAll(self, other):
        """Rows in both frames, with multiplicity min(count_left, count_right)."""
        def f(left, right):
            cnt: Dict[tuple, int] = {}
            for r in right:
                k = _key(r)
                cnt[k] = cnt.get(k, 0) + 1
            out = []
            for r in left:
                k = _key(r)
                if cnt.get(k, 0) > 0:
                    cnt[k] -= 1
                    out.append(r)
            return out
        return self._set_op(other, f, "intersectAll")

    def subtract(self, other):
        """Distinct rows of this frame that are not in ``other`` (SQL EXCEPT DISTINCT)."""
        def f(left, right):
            rk = {_key(r) for r in right}
            seen, out = set(), []
            for r in left:
                k = _key(r)
                if k not in rk and k not in seen:
                    seen.add(k)
                    out.append(r)
            return out
        return self._set_op(other, f, "subtract")

    def exceptAll(self, other):
        """Rows of this frame minus ``other`` with multiplicity (SQL EXCEPT ALL)."""
        def f(left, right):
            cnt: Dict[tuple, int] = {}
            for r in right:
                k = _key(r)
                cnt[k] = cnt.get(k, 0) + 1
            out = []
            for r in left:
                k = _key(r)
                if cnt.get(k, 0) > 0:
                    cnt[k] -= 1
                else:
                    out.append(r)
            return out
        return self._set_op(other, f, "exceptAll")

    # ------------------------------------------------------------------------------ statistics
    @property
    def stat(self) -> "DataFrameStatFunctions":
        return DataFrameStatFunctions(self)

    def approxQuantile(self, col, probabilities: Sequence[float], relativeError: float):
        """Exact order statistics (valid for any relativeError): for each p the smallest value whose
        rank reaches ceil(p * n); nulls and NaNs are ignored. ``col`` may be a list of columns."""
        if isinstance(col, (list, tuple)):
            return [self.approxQuantile(c, probabilities, relativeError) for c in col]
        cd = self._column_data(col)
        if cd.is_host:
            raise TypeError(f"approxQuantile: column {col!r} is not numeric")
        v = cd.values.to(torch.float64)
        ok = cd.valid_mask().to(v.device) & ~torch.isnan(v)
        allv = torch.sort(self._comm.allgather_cat(v[ok].contiguous())).values.cpu().numpy()
        if allv.size == 0:
            return []
        out = []
        for p in probabilities:
            if not 0.0 <= p <= 1.0:
                raise ValueError("approxQuantile: probabilities must be in [0, 1]")
            out.append(float(allv[min(max(int(math.ceil(p * allv.size)) - 1, 0), allv.size - 1)]))
        return out

    def corr(self, col1: str, col2: str, method: Optional[str] = None) -> float:
        if method not in (None, "pearson"):
            raise ValueError("DataFrame.corr only supports the pearson method")
        from . import functions as F
        return self.select(F.corr(col1, col2)).collect()[0][0]

    def cov(self, col1: str, col2: str) -> float:
        from . import functions as F
        return self.select(F.covar_samp(col1, col2)).collect()[0][0]

    def crosstab(self, col1: str, col2: str):
        """Contingency table: one row per distinct ``col1`` value, one count column per ``col2`` value."""
        from .builder import rows_round_robin
        from .dataframe import column_to_python
        a = column_to_python(self._column_data(col1))
        b = column_to_python(self._column_data(col2))
        local: Dict[tuple, int] = {}
        for x, y in zip(a, b):
            local[(x, y)] = local.get((x, y), 0) + 1
        tab: Dict[tuple, int] = {}
        for part in self._comm.allgather_object(local):
            for k, c in part.items():
                tab[k] = tab.get(k, 0) + c
        xs = sorted({k[0] for k in tab}, key=lambda v: (v is None, str(v)))
        ys = sorted({k[1] for k in tab}, key=lambda v: (v is None, str(v)))
        yname = [_sstr(y) for y in ys]
        schema = T.StructType([T.StructField(f"{col1}_{col2}", T.StringType(), False)]
                              + [T.StructField(n, T.LongType(), False) for n in yname])
        rows = [[_sstr(x)] + [tab.get((x, y), 0) for y in ys] for x in xs]
        return rows_round_robin(self._session, schema, rows)

    def freqItems(self, cols: Sequence[str], support: Optional[float] = None):
        """Items occurring in at least ``support`` (default 1 %) of the rows, per column (exact)."""
        from .builder import rows_round_robin
        from .dataframe import column_to_python
        support = 0.01 if support is None else float(support)
        if not 1e-4 <= support <= 1.0:
            raise ValueError("freqItems: support must be in [1e-4, 1]")
        out, fields = [], []
        n = self.count()
        for c in cols:
            local: Dict[Any, int] = {}
            for v in column_to_python(self._column_data(c)):
                local[v] = local.get(v, 0) + 1
            tot: Dict[Any, int] = {}
            for part in self._comm.allgather_object(local):
                for k, cnt in part.items():
                    tot[k] = tot.get(k, 0) + cnt
            out.append([k for k, cnt in tot.items() if cnt >= support * n])
            fields.append(T.StructField(f"{c}_freqItems", T.ArrayType(self.schema[c].dataType), True))
        return rows_round_robin(self._session, T.StructType(fields), [out])

    def sampleBy(self, col: str, fractions: Dict[Any, float], seed: Optional[int] = None):
        """Stratified sample without replacement: a row of stratum s is kept with probability
        fractions[s] (0 for strata not listed), decided by hash(seed, row id) as ``sample`` does."""
        from ..utils import rng
        from .dataframe import column_to_python
        vals = column_to_python(self._column_data(col))
        frac = torch.as_tensor([float(fractions.get(v, 0.0)) for v in vals], dtype=torch.float64,
                               device=self._device)
        u = rng.uniform(self._row_ids, 0 if seed is None else int(seed), stream=5)
        return self._mask_rows(u < frac)

    def summary(self, *statistics: str):
        """count / mean / stddev / min / percentiles ("25%") / max / count_distinct per column, as
        strings (Spark's ``summary``); percentiles use approxQuantile."""
        from . import functions as F
        from .builder import rows_round_robin
        stats = list(statistics) or ["count", "mean", "stddev", "min", "25%", "50%", "75%", "max"]
        cols = [f.name for f in self.schema.fields if T.is_numeric(f.dataType) or isinstance(f.dataType,
                                                                                              T.StringType)]
        table = {s: [] for s in stats}
        for c in cols:
            num = T.is_numeric(self.schema[c].dataType)
            for s in stats:
                if s.endswith("%"):
                    v = self.approxQuantile(c, [float(s[:-1]) / 100.0], 0.0) if num else []
                    table[s].append(str(v[0]) if v else None)
                    continue
                fn = {"count": F.count, "mean": F.avg, "stddev": F.stddev, "min": F.min, "max": F.max,
                      "count_distinct": F.countDistinct}.get(s)
                if fn is None:
                    raise ValueError(f"summary: unknown statistic {s!r}")
                if not num and s in ("mean", "stddev"):
                    table[s].append(None)
                    continue
                v = self.agg(fn(c)).collect()[0][0]
                table[s].append(None if v is None else str(v))
        schema = T.StructType([T.StructField("summary", T.StringType())] + [T.StructField(c, T.StringType())
                                                                           for c in cols])
        return rows_round_robin(self._session, schema, [[s] + table[s] for s in stats])

    # ------------------------------------------------------------------------------ pandas functions
    def mapInPandas(self, func, schema):
        """``func`` maps an iterator of pandas DataFrames (this rank's shard) to an iterator of pandas
        DataFrames with ``schema``."""
        from .builder import frame_from_pycolumns
        sch = schema if isinstance(schema, T.StructType) else T.parse_ddl_schema(schema)
        pdf = self._local_pandas()
        outs = list(func(iter([pdf])))
        import pandas as pd
        res = pd.concat(outs, ignore_index=True) if outs else pd.DataFrame(columns=sch.names)
        return _frame_from_pandas_local(self, sch, res)

    def _local_pandas(self):
        import pandas as pd
        from .dataframe import column_to_python
        return pd.DataFrame({n: column_to_python(self._cols[n]) for n in self.columns})

    # ------------------------------------------------------------------------------ misc
    def checkpoint(self, eager: bool = True):
        """Shards are materialized device tensors already: the frame is its own checkpoint."""
        return self

    localCheckpoint = checkpoint

    def hint(self, name: str, *parameters):
        return self

    def sortWithinPartitions(self, *cols, **kwargs):
        return self.orderBy(*cols, **kwargs)

    def foreach(self, f) -> None:
        for r in self._local_row_objects():
            f(r)

    def foreachPartition(self, f) -> None:
        f(iter(self._local_row_objects()))

    def _local_row_objects(self):
        from .types import Row
        loc = self._local_rows_host()
        names = self.columns
        return [Row(**{n: loc[n][i] for n in names}) for i in range(self._nrows)]

    def colRegex(self, colName: str):
        from .column import Column
        pat = colName.strip("`")
        rx = re.compile(pat)
        cols = [c for c in self.columns if rx.fullmatch(c)]
        from . import functions as F
        if len(cols) == 1:
            return F.col(cols[0])
        return [F.col(c) for c in cols]

    def withColumnsRenamed(self, colsMap: Dict[str, str]):
        df = self
        for a, b in colsMap.items():
            df = df.withColumnRenamed(a, b)
        return df

    def toJSON(self) -> List[str]:
        import json
        out = []
        for r in self.collect():
            out.append(json.dumps({k: (v.isoformat() if hasattr(v, "isoformat") else v)
                                   for k, v in r.asDict().items()}, default=str))
        return out

    # ------------------------------------------------------------------------------ reshaping / misc API
    def unpivot(self, ids, values, variableColumnName: str, valueColumnName: str):
        """Wide to long: one output row per (input row, value column), ids repeated (values cast to
        their common type)."""
        from .builder import column_from_values
        from .dataframe import column_to_python
        ids = [ids] if isinstance(ids, str) else list(ids or [])
        ids = [c if isinstance(c, str) else c._expr.name() for c in ids]
        values = [c for c in self.columns if c not in ids] if values is None else (
            [values] if isinstance(values, str) else [c if isinstance(c, str) else c._expr.name() for c in values])
        if not values:
            raise ValueError("unpivot needs at least one value column")
        types = [self.schema[c].dataType for c in values]
        vt = types[0]
        for t in types[1:]:
            if type(t) is not type(vt):
                if T.is_numeric(t) and T.is_numeric(vt):
                    vt = T.DoubleType() if not (T.is_integral(t) and T.is_integral(vt)) else T.LongType()
                else:
                    vt = T.StringType()
        n, k = self._nrows, len(values)
        rep = torch.arange(n, device=self._device).repeat_interleave(k)
        base = self._take_rows(rep)
        cols = [column_to_python(self._cols[c]) for c in values]
        var, val = [], []
        for i in range(n):
            for j, c in enumerate(values):
                var.append(c)
                v = cols[j][i]
                val.append(str(v) if (v is not None and isinstance(vt, T.StringType)) else v)
        names = ids + [variableColumnName, valueColumnName]
        datas = [base._cols[c] for c in ids] + [column_from_values(var, T.StringType(), self._device),
                                                column_from_values(val, vt, self._device)]
        out = base._from_columns(names, datas)
        counts = self._comm.allgather_object(n * k)
        off = sum(counts[:self._comm.rank])
        out._row_ids = torch.arange(off, off + n * k, dtype=torch.int64, device=self._device)
        return out

    melt = unpivot

    def offset(self, num: int):
        """Skip the first ``num`` rows (global row order)."""
        counts = self._comm.allgather_object(self._nrows)
        start = sum(counts[:self._comm.rank])
        local_skip = min(max(num - start, 0), self._nrows)
        return self._take_rows(torch.arange(local_skip, self._nrows, device=self._device))

    def dropDuplicatesWithinWatermark(self, subset=None):
        return self.dropDuplicates(subset)

    def inputFiles(self) -> List[str]:
        return list(getattr(self, "_input_files_list", []) or [])

    def isLocal(self) -> bool:
        return self._comm.world_size == 1

    def repartitionByRange(self, numPartitions, *cols):
        """Range partitioning: rows sorted by ``cols`` and cut into contiguous rank shards."""
        if isinstance(numPartitions, (str,)) or hasattr(numPartitions, "_expr"):
            cols = (numPartitions,) + cols
        return self.orderBy(*cols) if cols else self.repartition()

    def replace(self, to_replace, value=None, subset=None):
        return self.na.replace(to_replace, value, subset)

    def sameSemantics(self, other) -> bool:
        """Same schema and the very same column buffers (frames here are materialised, not plans)."""
        return (self.schema == other.schema and self._nrows == other._nrows
                and all(self._cols[n] is other._cols[n] for n in self.columns))

    def semanticHash(self) -> int:
        return hash((tuple(self.columns), tuple(id(self._cols[n]) for n in self.columns))) & 0x7FFFFFFF

    def to(self, schema):
        """Reorder / cast columns by name to ``schema`` (missing nullable columns become null)."""
        from .column import Column, Lit
        from . import functions as F
        sch = schema if isinstance(schema, T.StructType) else T.parse_ddl_schema(schema)
        sel = []
        for f in sch.fields:
            if f.name in self.columns:
                sel.append(F.col(f.name).cast(f.dataType).alias(f.name))
            elif f.nullable:
                sel.append(Column(Lit(None)).cast(f.dataType).alias(f.name))
            else:
                raise ValueError(f"column {f.name!r} is missing and not nullable")
        return self.select(*sel)

    def withMetadata(self, columnName: str, metadata: Dict[str, Any]):
        out = self.select(*self.columns)
        out.schema[columnName].metadata = dict(metadata)
        return out

    def observe(self, observation, *exprs):
        """Compute named metrics over this frame (eagerly: frames are materialised) and hand them to
        the ``Observation`` (or store them under a name); returns the frame unchanged."""
        row = self.agg(*exprs).collect()[0]
        if isinstance(observation, Observation):
            observation._set(row.asDict())
        else:
            self._session._observations = getattr(self._session, "_observations", {})
            self._session._observations[str(observation)] = row.asDict()
        return self

    def mapInArrow(self, func, schema):
        """``func`` maps an iterator of pyarrow RecordBatches (this rank's shard) to RecordBatches."""
        import pyarrow as pa
        from ..io.arrow import frame_to_arrow
        sch = schema if isinstance(schema, T.StructType) else T.parse_ddl_schema(schema)
        batches = frame_to_arrow(self).to_batches()
        outs = list(func(iter(batches)))
        tbl = pa.Table.from_batches(outs) if outs else None
        pdf = tbl.to_pandas() if tbl is not None else None
        import pandas as pd
        return _frame_from_pandas_local(self, sch, pdf if pdf is not None else pd.DataFrame(columns=sch.names))

    def writeTo(self, table: str):
        return DataFrameWriterV2(self, table)

    def pandas_api(self, index_col=None):
        """A pandas DataFrame of the whole frame (pandas-on-Spark is not part of this framework)."""
        return self.toPandas()

    def rollup(self, *cols):
        from .group import _as_key_exprs
        keys = _as_key_exprs(cols)
        return MultiGroupedData(self, keys, [keys[:i] for i in range(len(keys), -1, -1)])

    def cube(self, *cols):
        from itertools import combinations
        from .group import _as_key_exprs
        keys = _as_key_exprs(cols)
        sets = [list(c) for r in range(len(keys), -1, -1) for c in combinations(keys, r)]
        return MultiGroupedData(self, keys, sets)


class Observation:
    """``pyspark.sql.Observation``: metrics collected by ``df.observe(obs, ...)``."""

    def __init__(self, name: Optional[str] = None):
        self.name = name or "observation"
        self._vals: Optional[Dict[str, Any]] = None

    def _set(self, vals: Dict[str, Any]) -> None:
        self._vals = vals

    @property
    def get(self) -> Dict[str, Any]:
        if self._vals is None:
            raise RuntimeError("the observed DataFrame has not been evaluated")
        return dict(self._vals)


class DataFrameWriterV2:
    """``df.writeTo(table)``: create / replace / createOrReplace / append / overwritePartitions on
    the catalog's transactional tables."""

    def __init__(self, df, table: str):
        self.df, self.table = df, table
        self._using = None
        self._parts: List[str] = []
        self._props: Dict[str, str] = {}

    def using(self, provider: str):
        self._using = provider
        return self

    def option(self, key, value):
        return self

    def options(self, **kw):
        return self

    def tableProperty(self, key, value):
        self._props[key] = value
        return self

    def partitionedBy(self, *cols):
        self._parts = [c if isinstance(c, str) else c._expr.name() for c in cols]
        return self

    def _exists(self) -> bool:
        return self.df._session.catalog.tableExists(self.table)

    def create(self) -> None:
        if self._exists():
            raise ValueError(f"table {self.table} already exists")
        self.df._session.catalog._save_table(self.table, self.df, "overwrite")

    def replace(self) -> None:
        if not self._exists():
            raise ValueError(f"table {self.table} does not exist")
        self.df._session.catalog._save_table(self.table, self.df, "overwrite")

    def createOrReplace(self) -> None:
        self.df._session.catalog._save_table(self.table, self.df, "overwrite")

    def append(self) -> None:
        if not self._exists():
            raise ValueError(f"table {self.table} does not exist")
        self.df._session.catalog._save_table(self.table, self.df, "append")

    def overwrite(self, condition=None) -> None:
        """Replace the rows matching ``condition`` (all rows when None) with this frame."""
        cat = self.df._session.catalog
        if condition is None:
            cat._save_table(self.table, self.df, "overwrite")
            return
        from .column import Column
        cond = condition if isinstance(condition, Column) else Column(condition)
        keep = cat._resolve(self.table).filter(~cond)
        cat._save_table(self.table, keep.unionByName(self.df), "overwrite")

    def overwritePartitions(self) -> None:
        """Dynamic partition overwrite: replace the partitions (by ``partitionedBy`` columns) present
        in this frame, keep the others."""
        cat = self.df._session.catalog
        if not self._parts or not self._exists():
            cat._save_table(self.table, self.df, "overwrite")
            return
        from .dataframe import column_to_python
        from . import functions as F
        new_keys = set()
        for part in self.df._comm.allgather_object(list(zip(*[column_to_python(self.df._cols[c])
                                                               for c in self._parts]))):
            new_keys.update(part)
        old = cat._resolve(self.table)
        old_keys = list(zip(*[column_to_python(old._cols[c]) for c in self._parts])) if old._nrows else []
        mask = torch.as_tensor([k not in new_keys for k in old_keys], dtype=torch.bool, device=old._device)
        keep = old._mask_rows(mask) if old._nrows else old
        cat._save_table(self.table, keep.unionByName(self.df), "overwrite")


def _frame_from_pandas_local(df, schema: T.StructType, pdf):
    """A frame whose rows are this rank's pandas rows (row ids renumbered globally)."""
    from .builder import frame_from_pycolumns
    n = len(pdf)
    counts = df._comm.allgather_object(n)
    off = sum(counts[:df._comm.rank])
    pycols = {}
    for f in schema.fields:
        col = pdf[f.name]
        if (col.dtype.kind in "biuf" and not isinstance(f.dataType, (T.StringType, T.VectorUDT, T.DateType,
                                                                     T.TimestampType))) or \
                (col.dtype.kind == "M" and isinstance(f.dataType, T.TimestampType)):
            pycols[f.name] = col.to_numpy()  # numpy fast path (NaN in integral columns -> null)
        else:
            pycols[f.name] = [None if (isinstance(v, float) and v != v and not isinstance(f.dataType, (
                T.DoubleType, T.FloatType))) else v for v in col.tolist()]
    return frame_from_pycolumns(df._session, schema, pycols, list(range(off, off + n)))


class DataFrameStatFunctions:
    def __init__(self, df):
        self.df = df

    def approxQuantile(self, col, probabilities, relativeError):
        return self.df.approxQuantile(col, probabilities, relativeError)

    def corr(self, col1, col2, method=None):
        return self.df.corr(col1, col2, method)

    def cov(self, col1, col2):
        return self.df.cov(col1, col2)

    def crosstab(self, col1, col2):
        return self.df.crosstab(col1, col2)

    def freqItems(self, cols, support=None):
        return self.df.freqItems(cols, support)

    def sampleBy(self, col, fractions, seed=None):
        return self.df.sampleBy(col, fractions, seed)


class MultiGroupedData:
    """rollup / cube: one aggregation per grouping set, keys outside the set are null, results
    unioned (Spark's GROUPING SETS)."""

    def __init__(self, df, keys, sets):
        self.df, self.keys, self.sets = df, keys, sets

    def agg(self, *exprs):
        from .column import Alias, Column, Lit
        from .dataframe import _as_expr
        from .functions_extra import GroupingMarker
        from .group import GroupedData
        names = [k.name() for k in self.keys]
        if len(exprs) == 1 and isinstance(exprs[0], dict):
            from . import functions as F
            exprs = tuple(getattr(F, fn if fn != "mean" else "avg")(c).alias(f"{fn}({c})")
                          for c, fn in exprs[0].items())
        es = [_as_expr(e) for e in exprs]
        plain = [Column(e) for e in es if not isinstance(e.child if isinstance(e, Alias) else e, GroupingMarker)]
        out = None
        for s in self.sets:
            part = GroupedData(self.df, list(s)).agg(*plain)
            sn = [k.name() for k in s]
            sel = []
            for nm, k in zip(names, self.keys):
                if nm in sn:
                    sel.append(Column(_as_expr(nm)))
                else:
                    dt = k.eval(self.df).dtype
                    sel.append(Column(Lit(None)).cast(dt).alias(nm))
            agg_cols = [c for c in part.columns if c not in sn]
            it = iter(agg_cols)
            for e in es:
                inner = e.child if isinstance(e, Alias) else e
                if isinstance(inner, GroupingMarker):
                    v, dt = inner.value(names, sn)
                    sel.append(Column(Lit(v)).cast(dt).alias(e.alias if isinstance(e, Alias) else inner.name()))
                else:
                    sel.append(Column(_as_expr(next(it))))
            part = part.select(*sel)
            out = part if out is None else out.union(part)
        return out

    def count(self):
        from . import functions as F
        return self.agg(F.count("*").alias("count"))


class PivotedData:
    """``groupBy(keys).pivot(col, values).agg(...)``: one output column per (pivot value, aggregate)."""

    def __init__(self, df, keys, pivot, values):
        self.df, self.keys, self.pivot, self.values = df, keys, pivot, values

    def agg(self, *exprs):
        from .builder import rows_round_robin
        from .column import Alias
        from .dataframe import _as_expr, column_to_python
        from .group import aggregate, _agg_name
        pv_expr = _as_expr(self.pivot)
        values = self.values
        if values is None:
            vals = column_to_python(pv_expr.eval(self.df))
            allv = set()
            for part in self.df._comm.allgather_object(sorted({v for v in vals if v is not None}, key=str)):
                allv |= set(part)
            values = sorted(allv, key=lambda v: (str(type(v)), v))
            if len(values) > 10000:
                raise ValueError("pivot: more than 10000 distinct values; pass them explicitly")
        from .column import ColRef
        agg_exprs = [_as_expr(e) for e in exprs]
        key_names = [k.name() for k in self.keys]
        res = aggregate(self.df, self.keys + [pv_expr], [ColRef(n) for n in key_names] + [ColRef(pv_expr.name())]
                        + agg_exprs)
        rows = res.collect()
        nk = len(key_names)
        agg_names = [a.alias if isinstance(a, Alias) else _agg_name(a) for a in agg_exprs]
        agg_types = [res.schema.fields[nk + 1 + j].dataType for j in range(len(agg_exprs))]
        table: Dict[tuple, Dict[Any, list]] = {}
        order: List[tuple] = []
        for r in rows:
            k = tuple(r[:nk])
            if k not in table:
                table[k] = {}
                order.append(k)
            table[k][r[nk]] = list(r[nk + 1:])
        fields = [T.StructField(n, res.schema.fields[i].dataType) for i, n in enumerate(key_names)]
        for v in values:
            for j, an in enumerate(agg_names):
                nm = str(v) if len(agg_names) == 1 else f"{v}_{an}"
                fields.append(T.StructField(nm, agg_types[j]))
        out_rows = []
        for k in order:
            row = list(k)
            for v in values:
                got = table[k].get(v)
                row += got if got is not None else [None] * len(agg_names)
            out_rows.append(row)
        return rows_round_robin(self.df._session, T.StructType(fields), out_rows)

    def count(self):
        from . import functions as F
        return self.agg(F.count("*").alias("count"))

    def sum(self, *cols):
        from . import functions as F
        return self.agg(*[F.sum(c) for c in cols])

    def avg(self, *cols):
        from . import functions as F
        return self.agg(*[F.avg(c) for c in cols])

    mean = avg


def apply_in_pandas(grouped, func, schema):
    """GroupedData.applyInPandas: every group's rows become one pandas DataFrame handed to ``func``.
    Groups get global dense codes (sql/relational_fast.py); group g's rows are shuffled to rank
    g % world (one all-to-all), each rank converts its rows to pandas column-wise once and calls
    ``func`` per group, in key order. Output rows stay on that rank."""
    import pandas as pd
    from . import relational_fast as RF
    df = grouped.df
    sch = schema if isinstance(schema, T.StructType) else T.parse_ddl_schema(schema)
    comm = df._comm
    kc = [k.eval(df) for k in grouped.keys]
    ok = all(RF._key_kind(c) is not None for c in kc)
    if comm.is_distributed:
        ok = all(comm.allgather_object(ok))
    if not ok:
        return _apply_in_pandas_rows(grouped, func, sch)
    if comm.is_distributed:
        counts = RF._counts(comm, df._nrows)
        off = sum(counts[:comm.rank])
        code = RF._tuple_codes([RF._blocks(c, comm, df._device) for c in kc], df._device, null_equal=True) \
            if sum(counts) else torch.zeros(0, dtype=torch.int64, device=df._device)
        dest = code[off:off + df._nrows] % comm.world_size
        df = RF.shuffle_to(df, dest)
        kc = [k.eval(df) for k in grouped.keys]
    from .dataframe import _pandas_array, column_to_python
    names = df.columns
    pdf_all = pd.DataFrame({n: _pandas_array(df._cols[n]) for n in names}, columns=names)
    mine = []
    if df._nrows:
        code = RF._tuple_codes([[c] for c in kc], df._device, null_equal=True).cpu().numpy()
        order = np.argsort(code, kind="stable")
        bounds = np.flatnonzero(np.diff(code[order])) + 1
        groups = np.split(order, bounds)
        kv = [column_to_python(c) for c in kc]
        groups.sort(key=lambda g: tuple(str(v[g[0]]) for v in kv))
        for g in groups:
            mine.append(func(pdf_all.iloc[g].reset_index(drop=True)))
    res = pd.concat(mine, ignore_index=True) if mine else pd.DataFrame(columns=sch.names)
    return _frame_from_pandas_local(df, sch, res)


def _apply_in_pandas_rows(grouped, func, sch):
    """Row-gathering applyInPandas for keys without device codes: group g is processed by rank
    crc32(g) % world (deterministic), whose output rows stay on that rank."""
    import pandas as pd
    df = grouped.df
    names, rows, _ = df._gather_host()
    from .dataframe import column_to_python
    keyvals = [df._comm.allgather_object(column_to_python(k.eval(df))) for k in grouped.keys]
    flat = [[v for part in kv for v in part] for kv in keyvals]
    groups: Dict[tuple, List[int]] = {}
    for i in range(len(rows)):
        groups.setdefault(tuple(f[i] for f in flat), []).append(i)
    import zlib
    mine = []
    W, r = df._comm.world_size, df._comm.rank
    for key in sorted(groups, key=lambda t: tuple(str(v) for v in t)):
        if zlib.crc32(repr(key).encode()) % W != r:
            continue
        pdf = pd.DataFrame([rows[i] for i in groups[key]], columns=names)
        mine.append(func(pdf))
    res = pd.concat(mine, ignore_index=True) if mine else pd.DataFrame(columns=sch.names)
    return _frame_from_pandas_local(df, sch, res)


def _frame_from_pandas_local(df, schema: T.StructType, pdf):
    """A frame whose rows are this rank's pandas rows (row ids renumbered globally)."""
    from .builder import frame_from_pycolumns
    n = len(pdf)
    counts = df._comm.allgather_object(n)
    off = sum(counts[:df._comm.rank])
    pycols = {}
    for f in schema.fields:
        col = pdf[f.name]
        if (col.dtype.kind in "biuf" and not isinstance(f.dataType, (T.StringType, T.VectorUDT, T.DateType,
                                                                     T.TimestampType))) or \
                (col.dtype.kind == "M" and isinstance(f.dataType, T.TimestampType)):
            pycols[f.name] = col.to_numpy()  # numpy fast path (NaN in integral columns -> null)
        else:
            pycols[f.name] = [None if (isinstance(v, float) and v != v and not isinstance(f.dataType, (
                T.DoubleType, T.FloatType))) else v for v in col.tolist()]
    return frame_from_pycolumns(df._session, schema, pycols, list(range(off, off + n)))


class DataFrameStatFunctions:
    def __init__(self, df):
        self.df = df

    def approxQuantile(self, col, probabilities, relativeError):
        return self.df.approxQuantile(col, probabilities, relativeError)

    def corr(self, col1, col2, method=None):
        return self.df.corr(col1, col2, method)

    def cov(self, col1, col2):
        return self.df.cov(col1, col2)

    def crosstab(self, col1, col2):
        return self.df.crosstab(col1, col2)

    def freqItems(self, cols, support=None):
        return self.df.freqItems(cols, support)

    def sampleBy(self, col, fractions, seed=None):
        return self.df.sampleBy(col, fractions, seed)


class MultiGroupedData:
    """rollup / cube: one aggregation per grouping set, keys outside the set are null, results
    unioned (Spark's GROUPING SETS)."""

    def __init__(self, df, keys, sets):
        self.df, self.keys, self.sets = df, keys, sets

    def agg(self, *exprs):
        from .column import Alias, Column, Lit
        from .dataframe import _as_expr
        from .functions_extra import GroupingMarker
        from .group import GroupedData
        names = [k.name() for k in self.keys]
        if len(exprs) == 1 and isinstance(exprs[0], dict):
            from . import functions as F
            exprs = tuple(getattr(F, fn if fn != "mean" else "avg")(c).alias(f"{fn}({c})")
                          for c, fn in exprs[0].items())
        es = [_as_expr(e) for e in exprs]
        plain = [Column(e) for e in es if not isinstance(e.child if isinstance(e, Alias) else e, GroupingMarker)]
        out = None
        for s in self.sets:
            part = GroupedData(self.df, list(s)).agg(*plain)
            sn = [k.name() for k in s]
            sel = []
            for nm, k in zip(names, self.keys):
                if nm in sn:
                    sel.append(Column(_as_expr(nm)))
                else:
                    dt = k.eval(self.df).dtype
                    sel.append(Column(Lit(None)).cast(dt).alias(nm))
            agg_cols = [c for c in part.columns if c not in sn]
            it = iter(agg_cols)
            for e in es:
                inner = e.child if isinstance(e, Alias) else e
                if isinstance(inner, GroupingMarker):
                    v, dt = inner.value(names, sn)
                    sel.append(Column(Lit(v)).cast(dt).alias(e.alias if isinstance(e, Alias) else inner.name()))
                else:
                    sel.append(Column(_as_expr(next(it))))
            part = part.select(*sel)
            out = part if out is None else out.union(part)
        return out

    def count(self):
        from . import functions as F
        return self.agg(F.count("*").alias("count"))


class PivotedData:
    """``groupBy(keys).pivot(col, values).agg(...)``: one output column per (pivot value, aggregate)."""

    def __init__(self, df, keys, pivot, values):
        self.df, self.keys, self.pivot, self.values = df, keys, pivot, values

    def agg(self, *exprs):
        from .builder import rows_round_robin
        from .column import Alias
        from .dataframe import _as_expr, column_to_python
        from .group import aggregate, _agg_name
        pv_expr = _as_expr(self.pivot)
        values = self.values
        if values is None:
            vals = column_to_python(pv_expr.eval(self.df))
            allv = set()
            for part in self.df._comm.allgather_object(sorted({v for v in vals if v is not None}, key=str)):
                allv |= set(part)
            values = sorted(allv, key=lambda v: (str(type(v)), v))
            if len(values) > 10000:
                raise ValueError("pivot: more than 10000 distinct values; pass them explicitly")
        from .column import ColRef
        agg_exprs = [_as_expr(e) for e in exprs]
        key_names = [k.name() for k in self.keys]
        res = aggregate(self.df, self.keys + [pv_expr], [ColRef(n) for n in key_names] + [ColRef(pv_expr.name())]
                        + agg_exprs)
        rows = res.collect()
        nk = len(key_names)
        agg_names = [a.alias if isinstance(a, Alias) else _agg_name(a) for a in agg_exprs]
        agg_types = [res.schema.fields[nk + 1 + j].dataType for j in range(len(agg_exprs))]
        table: Dict[tuple, Dict[Any, list]] = {}
        order: List[tuple] = []
        for r in rows:
            k = tuple(r[:nk])
            if k not in table:
                table[k] = {}
                order.append(k)
            table[k][r[nk]] = list(r[nk + 1:])
        fields = [T.StructField(n, res.schema.fields[i].dataType) for i, n in enumerate(key_names)]
        for v in values:
            for j, an in enumerate(agg_names):
                nm = str(v) if len(agg_names) == 1 else f"{v}_{an}"
                fields.append(T.StructField(nm, agg_types[j]))
        out_rows = []
        for k in order:
            row = list(k)
            for v in values:
                got = table[k].get(v)
                row += got if got is not None else [None] * len(agg_names)
            out_rows.append(row)
        return rows_round_robin(self.df._session, T.StructType(fields), out_rows)

    def count(self):
        from . import functions as F
        return self.agg(F.count("*").alias("count"))

    def sum(self, *cols):
        from . import functions as F
        return self.agg(*[F.sum(c) for c in cols])

    def avg(self, *cols):
        from . import functions as F
        return self.agg(*[F.avg(c) for c in cols])

    mean = avg


def apply_in_pandas(grouped, func, schema):
    """GroupedData.applyInPandas: every group's rows become one pandas DataFrame handed to ``func``.
    Rows are gathered; group g is processed by rank hash(g) % world (deterministic), whose output
    rows stay on that rank."""
    import pandas as pd
    df = grouped.df
    sch = schema if isinstance(schema, T.StructType) else T.parse_ddl_schema(schema)
    names, rows, _ = df._gather_host()
    from .dataframe import column_to_python
    keyvals = [df._comm.allgather_object(column_to_python(k.eval(df))) for k in grouped.keys]
    flat = [[v for part in kv for v in part] for kv in keyvals]
    groups: Dict[tuple, List[int]] = {}
    for i in range(len(rows)):
        groups.setdefault(tuple(f[i] for f in flat), []).append(i)
    import zlib
    mine = []
    W, r = df._comm.world_size, df._comm.rank
    for key in sorted(groups, key=lambda t: tuple(str(v) for v in t)):
        if zlib.crc32(repr(key).encode()) % W != r:
            continue
        pdf = pd.DataFrame([rows[i] for i in groups[key]], columns=names)
        mine.append(func(pdf))
    res = pd.concat(mine, ignore_index=True) if mine else pd.DataFrame(columns=sch.names)
    return _frame_from_pandas_local(df, sch, res)
