"""Sharded columnar DataFrame (N3 in SURVEY.md §1.2).

Every rank holds a contiguous *shard* of rows: numeric / timestamp / boolean /
vector columns are torch tensors resident on the rank's device (HBM on MI355X
ranks), string columns are host numpy arrays.  Each row carries a stable global
row id assigned at the source (file, line) or (input index), so randomized
decisions — ``randomSplit`` (ref.py:139, ref.py:180), sampling, bagging — are
pure functions of (seed, row id) and identical on 1, 2, 4 or 8 GPUs.

Row-local operations (select, withColumn, filter, na.drop, when/otherwise,
VectorAssembler) never communicate; global ones (count, collect/toPandas,
groupBy/agg, orderBy, distinct, describe) combine shards with the session's
communicator (RCCL on GPUs, gloo on CPU).
"""
from __future__ import annotations

import datetime as _dt
import math
from typing import Any, Dict, Iterable, List, Optional, Sequence, Tuple, Union

import numpy as np
import torch

from . import types as T
from .column import (AggExpr, Alias, ColRef, Column, ColumnData, DictColumnData, Expr, Lit, SortOrder, _expr, _to_host,
                     micros_to_datetime, ts_to_micros)
from .dataframe_more import DataFrameMoreMixin


def _as_expr(c) -> Expr:
    if isinstance(c, str):
        return ColRef(c)
    if isinstance(c, Column):
        return c._expr
    if isinstance(c, Expr):
        return c
    return Lit(c)


class DataFrame(DataFrameMoreMixin):
    def __init__(self, session, schema: T.StructType, cols: Dict[str, ColumnData], nrows: int,
                 row_ids: torch.Tensor, device: torch.device, stream=None):
        self._session = session
        self._schema = schema
        self._cols = cols
        self._nrows = int(nrows)
        self._row_ids = row_ids
        self._device = device
        self._stream = stream           # StreamPlan for streaming DataFrames (lazy)
        self._batch_time_us = None

    # ------------------------------------------------------------------------------------------ basics
    @property
    def sparkSession(self):
        return self._session

    @property
    def schema(self) -> T.StructType:
        return self._schema

    @property
    def columns(self) -> List[str]:
        return self._schema.names

    @property
    def dtypes(self) -> List[Tuple[str, str]]:
        return [(f.name, f.dataType.simpleString()) for f in self._schema.fields]

    @property
    def isStreaming(self) -> bool:
        return self._stream is not None

    def printSchema(self) -> None:
        print(self._schema.treeString(), end="")

    def __getitem__(self, item) -> Column:
        if isinstance(item, str):
            if item not in self._schema.names and self._stream is None:
                raise KeyError(f"column {item!r} not in {self._schema.names}")
            return Column(ColRef(item))
        if isinstance(item, int):
            return Column(ColRef(self._schema.names[item]))
        if isinstance(item, Column):
            return self.filter(item)
        if isinstance(item, (list, tuple)):
            return self.select(*item)
        raise TypeError(item)

    def __getattr__(self, item) -> Column:
        if item.startswith("_"):
            raise AttributeError(item)
        if item in self.__dict__.get("_schema", T.StructType()).names:
            return Column(ColRef(item))
        raise AttributeError(f"DataFrame has no attribute {item!r}")

    def _column_data(self, name: str) -> ColumnData:
        if name not in self._cols:
            raise KeyError(f"cannot resolve column {name!r}; available: {self.columns}")
        return self._cols[name]

    def _new(self, schema: T.StructType, cols: Dict[str, ColumnData], nrows: int, row_ids) -> "DataFrame":
        df = DataFrame(self._session, schema, cols, nrows, row_ids, self._device)
        df._batch_time_us = self._batch_time_us
        return df

    def _lazy(self, method: str, *args, **kwargs) -> "DataFrame":
        """Streaming DataFrames record transformations and replay them per micro-batch."""
        df = DataFrame(self._session, self._schema, {}, 0, None, self._device, self._stream.extend(method, args,
                                                                                                   kwargs))
        df._schema = self._stream_schema_after(method, args, kwargs)
        return df

    def _stream_schema_after(self, method, args, kwargs) -> T.StructType:
        empty = self._session._empty_frame(self._schema)
        out = getattr(empty, method)(*args, **kwargs)
        return out._schema if isinstance(out, DataFrame) else self._schema

    @property
    def _comm(self):
        return self._session._comm

    # ------------------------------------------------------------------------------------------ projection
    def select(self, *cols) -> "DataFrame":
        if self._stream is not None:
            return self._lazy("select", *cols)
        if len(cols) == 1 and isinstance(cols[0], (list, tuple)):
            cols = tuple(cols[0])
        exprs: List[Expr] = []
        for c in cols:
            if isinstance(c, str) and c == "*":
                exprs += [ColRef(n) for n in self.columns]
            else:
                exprs.append(_as_expr(c))
        if any(e.is_aggregate() for e in exprs):
            from .group import aggregate
            return aggregate(self, [], exprs)
        from .functions_more import Generator, select_with_generator
        if any(isinstance(e.child if isinstance(e, Alias) else e, Generator) for e in exprs):
            return select_with_generator(self, exprs)
        names, datas = [], []
        for e in exprs:
            names.append(e.name())
            datas.append(e.eval(self))
        return self._from_columns(names, datas)

    def _from_columns(self, names: Sequence[str], datas: Sequence[ColumnData]) -> "DataFrame":
        fields, cols = [], {}
        for n, d in zip(names, datas):
            nullable, meta = True, None
            if n in self._schema.names:
                nullable = self._schema[n].nullable
                if self._cols.get(n) is d:  # the column itself: keep its metadata (ML attributes)
                    meta = dict(self._schema[n].metadata)
            fields.append(T.StructField(n, d.dtype, nullable, meta))
            cols[n] = d
        return self._new(T.StructType(fields), cols, self._nrows, self._row_ids)

    def selectExpr(self, *exprs: str) -> "DataFrame":
        from .sqlparse import parse_select_item
        return self.select(*[Column(parse_select_item(e)) for e in exprs])

    def withColumn(self, name: str, col: Column) -> "DataFrame":
        if self._stream is not None:
            return self._lazy("withColumn", name, col)
        e = _as_expr(col)
        from .functions_more import Generator
        if isinstance(e, Generator) or (isinstance(e, Alias) and isinstance(e.child, Generator)):
            inner = e.child if isinstance(e, Alias) else e
            keep = [ColRef(c) for c in self.columns if c != name]
            return self.select(*keep, Alias(inner, name))
        data = e.eval(self)
        fields = list(self._schema.fields)
        cols = dict(self._cols)
        if name in cols:
            idx = self._schema.names.index(name)
            fields[idx] = T.StructField(name, data.dtype, True)
        else:
            fields.append(T.StructField(name, data.dtype, True))
        cols[name] = data
        return self._new(T.StructType(fields), cols, self._nrows, self._row_ids)

    def withColumns(self, mapping: Dict[str, Column]) -> "DataFrame":
        df = self
        for k, v in mapping.items():
            df = df.withColumn(k, v)
        return df

    def withColumnRenamed(self, existing: str, new: str) -> "DataFrame":
        if self._stream is not None:
            return self._lazy("withColumnRenamed", existing, new)
        if existing not in self._cols:
            return self
        fields = [T.StructField(new if f.name == existing else f.name, f.dataType, f.nullable, f.metadata)
                  for f in self._schema.fields]
        cols = {(new if k == existing else k): v for k, v in self._cols.items()}
        return self._new(T.StructType(fields), cols, self._nrows, self._row_ids)

    def drop(self, *cols) -> "DataFrame":
        if self._stream is not None:
            return self._lazy("drop", *cols)
        names = {c if isinstance(c, str) else _as_expr(c).name() for c in cols}
        keep = [f for f in self._schema.fields if f.name not in names]
        return self._new(T.StructType(keep), {f.name: self._cols[f.name] for f in keep}, self._nrows,
                         self._row_ids)

    def alias(self, name: str) -> "DataFrame":
        return self

    def toDF(self, *names) -> "DataFrame":
        df = self
        for old, new in zip(self.columns, names):
            df = df.withColumnRenamed(old, new)
        return df

    # ------------------------------------------------------------------------------------------ row selection
    def _take_rows(self, idx: torch.Tensor) -> "DataFrame":
        from ..utils.trace import trace
        idx = idx.to(self._device)
        cols = {}
        host_idx = None
        with trace("frame.take_rows"):
            for k, v in self._cols.items():
                if v.is_host or isinstance(v, DictColumnData):
                    if host_idx is None:  # one device->host copy of the index for every host column
                        with trace("frame.take_rows.index_to_host"):
                            host_idx = idx.cpu().numpy() if isinstance(idx, torch.Tensor) else np.asarray(idx)
                    with trace("frame.take_rows.host_column"):
                        cols[k] = v.take(host_idx)
                else:
                    cols[k] = v.take(idx)
            rid = self._row_ids[idx]
        return self._new(self._schema, cols, int(idx.numel()), rid)

    def _mask_index(self, mask: torch.Tensor) -> torch.Tensor:
        """Ascending row indices of a bool mask (GPU: the K3 compaction kernel)."""
        mask = mask.to(self._device)
        if mask.is_cuda:
            from ..ops import frame_ops
            return frame_ops.compact(mask)
        return torch.nonzero(mask, as_tuple=False).flatten()

    def _mask_rows(self, mask: torch.Tensor) -> "DataFrame":
        return self._take_rows(self._mask_index(mask))

    def filter(self, condition) -> "DataFrame":
        if self._stream is not None:
            return self._lazy("filter", condition)
        if isinstance(condition, str):
            from .sqlparse import parse_expression
            condition = Column(parse_expression(condition))
        cd = _as_expr(condition).eval(self)
        vals = cd.values if not cd.is_host else torch.as_tensor(np.asarray(cd.values, dtype=bool))
        mask = vals.to(torch.bool).to(self._device)
        if cd.valid is not None:
            vm = cd.valid if not isinstance(cd.valid, np.ndarray) else torch.as_tensor(cd.valid)
            mask = mask & vm.to(self._device)
        return self._mask_rows(mask)

    where = filter

    def limit(self, num: int) -> "DataFrame":
        if self._stream is not None:
            return self._lazy("limit", num)
        counts = self._comm.allgather_object(self._nrows)
        before = sum(counts[: self._comm.rank])
        take = max(0, min(self._nrows, num - before))
        return self._take_rows(torch.arange(take, device=self._device))

    def sample(self, withReplacement=None, fraction=None, seed=None) -> "DataFrame":
        if isinstance(withReplacement, float):
            withReplacement, fraction, seed = False, withReplacement, fraction
        from ..utils import rng
        seed = 0 if seed is None else int(seed)
        if withReplacement:
            cnt = rng.poisson1(self._row_ids, seed, 3)
            idx = torch.repeat_interleave(torch.arange(self._nrows, device=self._device), cnt.to(self._device))
            return self._take_rows(idx)
        u = rng.uniform(self._row_ids, seed, stream=5)
        return self._mask_rows(u < fraction)

    def randomSplit(self, weights: Sequence[float], seed: Optional[int] = None) -> List["DataFrame"]:
        """Weighted split by a counter-based uniform per global row id (GPU-count invariant).

        Spark semantics (ref.py:139): weights are normalised, each row lands in exactly
        one split, fractions are approximate.
        """
        from ..utils import rng
        w = np.asarray(weights, dtype=np.float64)
        if (w < 0).any() or w.sum() <= 0:
            raise ValueError("weights must be non-negative with a positive sum")
        cum = np.concatenate([[0.0], np.cumsum(w / w.sum())])
        cum[-1] = 1.0 + 1e-12
        seed = np.random.randint(0, 2**31 - 1) if seed is None else int(seed)
        rows = self._row_ids.to(self._device)
        if rows.is_cuda and self._nrows and len(w) <= 16:
            # K5: one fused hash + bucket pass, then one compaction per split
            from ..ops import frame_ops
            b = frame_ops.split_buckets(rows, rng.key(seed, 2), cum)
            return [self._mask_rows(b == i) for i in range(len(w))]
        u = rng.uniform(rows, seed, stream=2) if self._nrows else torch.zeros(
            0, dtype=torch.float64, device=self._device)
        out = []
        for i in range(len(w)):
            out.append(self._mask_rows((u >= cum[i]) & (u < cum[i + 1])))
        return out

    @property
    def na(self) -> "DataFrameNaFunctions":
        return DataFrameNaFunctions(self)

    def dropna(self, how: str = "any", thresh: Optional[int] = None, subset=None) -> "DataFrame":
        if self._stream is not None:
            return self._lazy("dropna", how, thresh, subset)
        names = self.columns if subset is None else ([subset] if isinstance(subset, str) else list(subset))
        if not names or self._nrows == 0:
            return self
        from ..utils.trace import trace
        with trace("DataFrame.dropna"):
            return self._dropna(names, how, thresh)

    def _dropna(self, names, how, thresh) -> "DataFrame":
        from ..utils.trace import trace
        good = torch.zeros((self._nrows,), dtype=torch.int32, device=self._device)
        with trace("dropna.masks"):
            always = 0  # columns that cannot hold a null: no per-row work (no host mask, no copy)
            for n in names:
                cd = self._cols[n]
                if _never_null(cd):
                    always += 1
                    continue
                m = _non_null_mask(cd)
                good += m.to(self._device).to(torch.int32)
            if always:
                good += always
        if thresh is not None:
            keep = good >= thresh
        elif how == "all":
            keep = good > 0
        else:
            keep = good == len(names)
        if bool(keep.all()):
            return self  # nothing to drop: no gather, the frame is returned as is
        return self._mask_rows(keep)

    def fillna(self, value, subset=None) -> "DataFrame":
        if self._stream is not None:
            return self._lazy("fillna", value, subset)
        if isinstance(value, dict):
            items = value.items()
        else:
            names = self.columns if subset is None else ([subset] if isinstance(subset, str) else list(subset))
            items = [(n, value) for n in names]
        cols = dict(self._cols)
        for n, v in items:
            cd = cols[n]
            if cd.is_host:
                if not isinstance(v, str):
                    continue
                m = ~_non_null_mask(cd).cpu().numpy()
                vals = cd.values.copy()
                vals[m] = v
                cols[n] = ColumnData(vals, None, cd.dtype)
            else:
                if isinstance(v, str) or isinstance(cd.dtype, T.VectorUDT):
                    continue
                if isinstance(v, bool) != isinstance(cd.dtype, T.BooleanType):
                    continue
                m = _non_null_mask(cd)
                fill = torch.full_like(cd.values, v if not T.is_integral(cd.dtype) else int(v))
                cols[n] = ColumnData(torch.where(m, cd.values, fill), None, cd.dtype)
        return self._new(self._schema, cols, self._nrows, self._row_ids)

    def union(self, other: "DataFrame") -> "DataFrame":
        if len(other.columns) != len(self.columns):
            raise ValueError("union requires the same number of columns")
        renamed = other.toDF(*self.columns)
        return self._concat([self, renamed])

    unionAll = union

    def unionByName(self, other: "DataFrame", allowMissingColumns: bool = False) -> "DataFrame":
        if allowMissingColumns:
            a, b = self, other
            for f in other.schema.fields:
                if f.name not in a.columns:
                    a = a.withColumn(f.name, Column(Lit(None)).cast(f.dataType))
            for f in self.schema.fields:
                if f.name not in b.columns:
                    b = b.withColumn(f.name, Column(Lit(None)).cast(f.dataType))
            return a._concat([a, b.select(*a.columns)])
        return self._concat([self, other.select(*self.columns)])

    def _concat(self, frames: List["DataFrame"]) -> "DataFrame":
        cols = {}
        for f in self._schema.fields:
            parts = [fr._cols[f.name] for fr in frames]
            cols[f.name] = concat_column_data(parts, self._device)
        rid = torch.cat([fr._row_ids for fr in frames]) if frames else self._row_ids
        # keep ids unique across the union (second frame's ids are offset into a disjoint range)
        if len(frames) > 1:
            offs = []
            for i, fr in enumerate(frames):
                offs.append(fr._row_ids + (i << 52))
            rid = torch.cat(offs)
        schema = T.StructType([T.StructField(f.name, cols[f.name].dtype, True) for f in self._schema.fields])
        return self._new(schema, cols, sum(fr._nrows for fr in frames), rid)

    # ------------------------------------------------------------------------------------------ actions
    def count(self) -> int:
        if self._stream is not None:
            raise RuntimeError("Queries with streaming sources must be executed with writeStream.start()")
        return int(self._comm.sum_scalar(float(self._nrows)))

    def isEmpty(self) -> bool:
        return self.count() == 0

    def _local_rows_host(self) -> Dict[str, List[Any]]:
        out = {}
        for f in self._schema.fields:
            out[f.name] = column_to_python(self._cols[f.name])
        return out

    def _gather_host(self) -> Tuple[List[str], List[List[Any]], List[int]]:
        """All rows of all ranks, in rank order (collect-to-driver, ref.py:204)."""
        local = self._local_rows_host()
        ids = self._row_ids.cpu().tolist() if self._nrows else []
        parts = self._comm.allgather_object((local, ids, self._nrows))
        names = self.columns
        rows: List[List[Any]] = []
        all_ids: List[int] = []
        for loc, pid, n in parts:
            if n:
                rows.extend(map(list, zip(*[loc[nm] for nm in names])) if names else ([] for _ in range(n)))
            all_ids += pid
        return names, rows, all_ids

    def collect(self) -> List[T.Row]:
        if self._stream is not None:
            raise RuntimeError("Queries with streaming sources must be executed with writeStream.start()")
        names, rows, _ = self._gather_host()
        return [T.Row._make(names, r) for r in rows]

    def take(self, num: int) -> List[T.Row]:
        return self.limit(num).collect()

    def head(self, n: Optional[int] = None):
        rows = self.take(1 if n is None else n)
        if n is None:
            return rows[0] if rows else None
        return rows

    def first(self):
        return self.head()

    def tail(self, num: int) -> List[T.Row]:
        rows = self.collect()
        return rows[-num:] if num else []

    def toLocalIterator(self):
        return iter(self.collect())

    def toPandas(self):
        """All rows as a pandas DataFrame (collect-to-driver, ref.py:204). Numeric, boolean and
        timestamp columns move as numpy arrays (one device-to-host copy per column); other types
        go through Python values."""
        import pandas as pd
        names = self.columns
        local = {n: _pandas_array(self._cols[n]) for n in names}
        parts = self._comm.allgather_object(local) if self._comm.is_distributed else [local]
        data = {}
        for n in names:
            arrs = [p[n] for p in parts]
            data[n] = np.concatenate(arrs) if all(isinstance(a, np.ndarray) for a in arrs) else \
                [v for a in arrs for v in (a.tolist() if isinstance(a, np.ndarray) else a)]
        pdf = pd.DataFrame(data, columns=names)
        for f in self._schema.fields:
            if isinstance(f.dataType, T.TimestampType):
                pdf[f.name] = pd.to_datetime(pdf[f.name])
            elif T.is_numeric(f.dataType) and not T.is_integral(f.dataType):
                pdf[f.name] = pd.to_numeric(pdf[f.name])
        return pdf

    def toArrow(self):
        import pyarrow as pa
        return pa.Table.from_pandas(self.toPandas(), preserve_index=False)

    def show(self, n: int = 20, truncate: Union[bool, int] = True, vertical: bool = False) -> None:
        print(self._show_string(n, truncate, vertical), end="")

    def _show_string(self, n=20, truncate=True, vertical=False) -> str:
        rows = self.limit(n + 1).collect()
        more = len(rows) > n
        rows = rows[:n]
        names = self.columns
        width = 20 if truncate is True else (int(truncate) if truncate else 0)

        def fmt(v):
            if v is None:
                s = "NULL"
            elif isinstance(v, bool):
                s = "true" if v else "false"
            elif isinstance(v, float):
                s = repr(v) if not v.is_integer() or abs(v) >= 1e16 else f"{v:.1f}"
            elif isinstance(v, _dt.datetime):
                s = v.strftime("%Y-%m-%d %H:%M:%S") + (f".{v.microsecond:06d}".rstrip("0") if v.microsecond else "")
            else:
                s = str(v)
            if width and len(s) > width:
                s = s[: width - 3] + "..."
            return s

        cells = [[fmt(v) for v in r] for r in rows]
        if vertical:
            out = []
            for i, r in enumerate(cells):
                out.append(f"-RECORD {i}" + "-" * 20)
                for nm, v in zip(names, r):
                    out.append(f" {nm} | {v}")
            return "\n".join(out) + "\n"
        ws = [max([len(nm)] + [len(r[i]) for r in cells]) for i, nm in enumerate(names)]
        sep = "+" + "+".join("-" * w for w in ws) + "+"
        lines = [sep, "|" + "|".join(nm.rjust(w) for nm, w in zip(names, ws)) + "|", sep]
        for r in cells:
            lines.append("|" + "|".join(v.rjust(w) for v, w in zip(r, ws)) + "|")
        lines.append(sep)
        if more:
            lines.append(f"only showing top {n} rows")
        return "\n".join(lines) + "\n"

    def __repr__(self):
        return "DataFrame[" + ", ".join(f"{a}: {b}" for a, b in self.dtypes) + "]"

    # ------------------------------------------------------------------------------------------ global ops
    def groupBy(self, *cols) -> "GroupedData":
        from .group import GroupedData
        if len(cols) == 1 and isinstance(cols[0], (list, tuple)):
            cols = tuple(cols[0])
        return GroupedData(self, [_as_expr(c) for c in cols])

    groupby = groupBy

    def agg(self, *exprs) -> "DataFrame":
        return self.groupBy().agg(*exprs)

    def orderBy(self, *cols, ascending=True) -> "DataFrame":
        from .group import sort_frame
        if len(cols) == 1 and isinstance(cols[0], (list, tuple)):
            cols = tuple(cols[0])
        asc = ascending if isinstance(ascending, (list, tuple)) else [ascending] * len(cols)
        orders = []
        for c, a in zip(cols, asc):
            if isinstance(c, SortOrder):
                orders.append(c)
            else:
                orders.append(SortOrder(_as_expr(c), bool(a)))
        return sort_frame(self, orders)

    sort = orderBy

    def distinct(self) -> "DataFrame":
        return self.dropDuplicates()

    def dropDuplicates(self, subset: Optional[Sequence[str]] = None) -> "DataFrame":
        if self._stream is not None:
            return self._lazy("_stream_dedup", list(subset) if subset else None)
        from .group import drop_duplicates
        return drop_duplicates(self, subset)

    def _stream_dedup(self, subset) -> "DataFrame":
        """Batch semantics of a streaming dropDuplicates (used for the plan's schema)."""
        from .group import drop_duplicates
        return drop_duplicates(self, subset)

    def _stream_aggregate(self, keys, exprs) -> "DataFrame":
        """Batch semantics of a streaming groupBy().agg() (used for the plan's schema)."""
        from .group import aggregate
        return aggregate(self, keys, exprs)

    drop_duplicates = dropDuplicates

    def describe(self, *cols) -> "DataFrame":
        from .group import describe
        if len(cols) == 1 and isinstance(cols[0], (list, tuple)):
            cols = tuple(cols[0])
        return describe(self, list(cols))


    def join(self, other: "DataFrame", on=None, how: str = "inner") -> "DataFrame":
        from .group import join_frames
        return join_frames(self, other, on, how)

    def crossJoin(self, other: "DataFrame") -> "DataFrame":
        from .group import join_frames
        return join_frames(self, other, None, "cross")

    # ------------------------------------------------------------------------------------------ persistence & misc
    def cache(self) -> "DataFrame":
        """Shards already live in HBM (or host RAM in local mode): caching is the identity."""
        return self

    persist = cache

    def unpersist(self, blocking: bool = False) -> "DataFrame":
        return self

    @property
    def storageLevel(self):
        return "MEMORY_AND_HBM"

    def repartition(self, numPartitions=None, *cols) -> "DataFrame":
        """Rebalance rows evenly across ranks (row ids and order preserved)."""
        from .group import rebalance
        return rebalance(self)

    def coalesce(self, numPartitions: int) -> "DataFrame":
        return self

    def rdd(self):  # pragma: no cover - compatibility stub
        raise NotImplementedError("RDDs are not part of this engine; use DataFrame operations")

    def createOrReplaceTempView(self, name: str) -> None:
        self._session.catalog._register_view(name, self, replace=True)

    def createTempView(self, name: str) -> None:
        self._session.catalog._register_view(name, self, replace=False)

    registerTempTable = createOrReplaceTempView

    def createGlobalTempView(self, name: str) -> None:
        self._session.catalog._register_global_view(name, self, replace=False)

    def createOrReplaceGlobalTempView(self, name: str) -> None:
        self._session.catalog._register_global_view(name, self, replace=True)

    @property
    def write(self):
        from ..io.writer import DataFrameWriter
        return DataFrameWriter(self)

    @property
    def writeStream(self):
        if self._stream is None:
            raise RuntimeError("'writeStream' can be called only on streaming Dataset/DataFrame")
        from .streaming import DataStreamWriter
        return DataStreamWriter(self)

    def withWatermark(self, eventTime: str, delayThreshold: str) -> "DataFrame":
        """Event-time watermark (ref.py:81).  Batch frames: no-op, as in Spark."""
        if self._stream is None:
            return self
        df = self._lazy("withWatermark", eventTime, delayThreshold)
        df._stream.watermark = (eventTime, delayThreshold)
        return df

    def explain(self, extended: bool = False) -> None:
        kind = "Streaming" if self._stream is not None else "Resident"
        print(f"== Physical Plan ==\n{kind}Scan [{', '.join(self.columns)}] on {self._device} "
              f"(rank {self._comm.rank}/{self._comm.world_size})")

    def _apply_transformer(self, model) -> "DataFrame":
        """Used to replay ``model.transform`` on each micro-batch of a streaming frame."""
        return model.transform(self)

    def transform(self, func, *args, **kwargs) -> "DataFrame":
        return func(self, *args, **kwargs)

    # ------------------------------------------------------------------------------------------ device helpers
    def _feature_matrix(self, col: str, defer_nan_check: bool = False) -> torch.Tensor:
        """The [n, d] tensor of a vector column (row-major, device-resident). A NaN check a producer
        deferred to its consumers (VectorAssembler handleInvalid="error") runs here, once, unless the
        caller takes it over (``defer_nan_check``: it calls _run_nan_check / _clear_nan_check)."""
        cd = self._cols[col]
        if not isinstance(cd.dtype, T.VectorUDT):
            raise TypeError(f"column {col!r} is {cd.dtype.simpleString()}, expected vector")
        if not defer_nan_check and getattr(cd, "nan_pending", None):
            self._run_nan_check(col)
            cd.nan_pending = None
        return cd._vals()

    def _pending_nan_check(self, col: str):
        return getattr(self._cols[col], "nan_pending", None)

    def _run_nan_check(self, col: str) -> None:
        """Raise the deferred handleInvalid error when a row of the column holds a NaN on any rank."""
        cd = self._cols[col]
        msg = getattr(cd, "nan_pending", None)
        if not msg:
            return
        x = cd._vals()
        if not x.numel():
            bad = False
        elif x.is_cuda:
            from ..ops import frame_ops
            bad = bool(frame_ops.has_nan(x))
        else:
            bad = bool(torch.isnan(x).any().item())
        if self._comm.is_distributed:
            bad = self._comm.max_scalar(1.0 if bad else 0.0) > 0
        if bad:
            raise ValueError(msg)

    def _clear_nan_check(self, col: str) -> None:
        cd = self._cols[col]
        if getattr(cd, "nan_pending", None):
            cd.nan_pending = None

    def _numeric(self, col: str, dtype=torch.float64) -> torch.Tensor:
        cd = self._cols[col]
        if cd.is_host:
            raise TypeError(f"column {col!r} is not numeric")
        return cd.values.to(dtype)


class DataFrameNaFunctions:
    def __init__(self, df: DataFrame):
        self.df = df

    def drop(self, how: str = "any", thresh: Optional[int] = None, subset=None) -> DataFrame:
        return self.df.dropna(how, thresh, subset)

    def fill(self, value, subset=None) -> DataFrame:
        return self.df.fillna(value, subset)

    def replace(self, to_replace, value=None, subset=None) -> DataFrame:
        df = self.df
        names = df.columns if subset is None else list(subset)
        from .functions import when, col as _col
        mapping = to_replace if isinstance(to_replace, dict) else {to_replace: value}
        for n in names:
            c = _col(n)
            expr = None
            for a, b in mapping.items():
                expr = when(c == a, b) if expr is None else expr.when(c == a, b)
            if expr is not None:
                df = df.withColumn(n, expr.otherwise(c))
        return df


# ---------------------------------------------------------------------------------------------- helpers

def _never_null(cd: ColumnData) -> bool:
    """No validity mask and no value that reads as null: dictionary strings (nulls are masked rows),
    device integer/bool columns (floats can hold NaN, which na.drop treats as null)."""
    if cd.valid is not None:
        return False
    if isinstance(cd, DictColumnData):
        nn = getattr(cd, "_never_null", None)
        if nn is None:  # code -1 is a null string: one min over the codes, cached on the column
            nn = cd._never_null = bool(len(cd) == 0 or int(cd.codes.min()) >= 0)
        return nn
    return (not cd.is_host) and not cd.values.is_floating_point() and not cd.values.is_complex()


def _non_null_mask(cd: ColumnData) -> torch.Tensor:
    if cd.is_host and cd.codes is not None:
        return torch.as_tensor(np.asarray(cd.codes) >= 0)  # dictionary codes: -1 is null
    if cd.is_host:
        import pandas as pd
        m = cd.valid_mask() & ~pd.isna(cd.values)  # None / NaN test in C, not a Python loop
        return torch.as_tensor(np.asarray(m, dtype=bool))
    m = cd.valid_mask()
    if cd.values.is_floating_point():
        if cd.values.dim() == 1:
            m = m & ~torch.isnan(cd.values)
    return m


def concat_column_data(parts: List[ColumnData], device) -> ColumnData:
    dt = parts[0].dtype
    if any(p.is_host for p in parts):
        hs = [_to_host(p) for p in parts]
        vals = np.concatenate([h.values for h in hs]) if hs else np.empty(0, dtype=object)
        valid = None
        if any(h.valid is not None for h in hs):
            valid = np.concatenate([h.valid_mask() for h in hs])
        return ColumnData(vals, valid, dt)
    vals = torch.cat([p.values.to(device) for p in parts])
    valid = None
    if any(p.valid is not None for p in parts):
        valid = torch.cat([p.valid_mask().to(device) for p in parts])
    return ColumnData(vals, valid, dt)


def _pandas_array(cd: ColumnData):
    """The pandas representation of one local column: a numpy array where pandas would infer the
    same dtype from the Python values (int64 / float64 with NaN for nulls / bool / datetime64 with
    NaT), else the list of Python values."""
    dt = cd.dtype
    if cd.is_host or cd.values.dim() != 1 or not (T.is_numeric(dt) or isinstance(dt, (T.BooleanType,
                                                                                        T.TimestampType))):
        return column_to_python(cd)
    v = cd.values.detach()
    ok = None if cd.valid is None else cd.valid.detach().cpu().numpy().astype(bool)
    nulls = ok is not None and not ok.all()
    if isinstance(dt, T.TimestampType):
        a = v.to(torch.int64).cpu().numpy().astype("datetime64[us]").astype("datetime64[ns]")
        if nulls:
            a[~ok] = np.datetime64("NaT")
        return a
    if isinstance(dt, T.BooleanType):
        return column_to_python(cd) if nulls else v.cpu().numpy().astype(bool)
    if T.is_integral(dt) and not nulls:
        return v.to(torch.int64).cpu().numpy()
    a = v.to(torch.float64).cpu().numpy()
    if nulls:
        a = a.copy()
        a[~ok] = np.nan
    return a


def column_to_python(cd: ColumnData) -> List[Any]:
    """Host python values of a column (nulls -> None)."""
    from ..ml.linalg import DenseVector
    n = len(cd)
    if cd.is_host:
        if cd.valid is None:
            return cd.values.tolist() if isinstance(cd.values, np.ndarray) and cd.values.dtype == object \
                else list(cd.values)
        vals = np.asarray(cd.values, dtype=object)
        return np.where(np.asarray(cd.valid, dtype=bool), vals, None).tolist()
    vals = cd.values.detach()
    if vals.dtype in (torch.bfloat16, torch.float8_e4m3fn):
        vals = vals.float()
    arr = vals.cpu().numpy()
    vm = cd.valid_mask().cpu().numpy() if n else np.ones(0, dtype=bool)
    dt = cd.dtype
    if isinstance(dt, T.VectorUDT):
        return [DenseVector(arr[i].astype(np.float64)) if vm[i] else None for i in range(n)]
    # vectorised conversions: numpy builds the Python objects (datetime64[us] -> datetime.datetime,
    # datetime64[D] -> datetime.date), nulls are patched in with one masked select
    if isinstance(dt, T.TimestampType):
        obj = arr.astype(np.int64).astype("datetime64[us]").astype(object)
    elif isinstance(dt, T.DateType):
        obj = arr.astype(np.int64).astype("datetime64[D]").astype(object)
    elif isinstance(dt, T.BooleanType):
        obj = arr.astype(bool)
    elif T.is_integral(dt):
        obj = arr.astype(np.int64)
    elif isinstance(dt, (T.FloatType, T.DoubleType)):
        obj = arr.astype(np.float64)
    else:
        return [arr[i] if vm[i] else None for i in range(n)]
    if vm.all():
        return obj.tolist()
    return np.where(vm, obj.astype(object), None).tolist()
