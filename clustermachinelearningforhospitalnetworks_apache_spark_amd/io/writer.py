"""df.write — DataFrameWriter (parquet / csv / json / orc / text / table / saveAsTable; Hive-style
``partitionBy`` directories)."""
from __future__ import annotations

import os
import shutil
from typing import Dict, Optional

from .reader import strip_scheme


class DataFrameWriter:
    def __init__(self, df):
        self._df = df
        self._format = "parquet"
        self._mode = "errorifexists"
        self._options: Dict[str, str] = {}
        self._partition_by = None

    def format(self, source: str) -> "DataFrameWriter":
        self._format = source.lower()
        return self

    def mode(self, saveMode: str) -> "DataFrameWriter":
        m = (saveMode or "errorifexists").lower()
        if m not in ("append", "overwrite", "error", "errorifexists", "ignore"):
            raise ValueError(f"unknown save mode {saveMode}")
        self._mode = m
        return self

    def option(self, key, value) -> "DataFrameWriter":
        self._options[key.lower()] = value
        return self

    def options(self, **opts) -> "DataFrameWriter":
        for k, v in opts.items():
            self.option(k, v)
        return self

    def partitionBy(self, *cols) -> "DataFrameWriter":
        self._partition_by = cols
        return self

    def _prepare_dir(self, path: str) -> bool:
        """Apply the save mode to a plain directory output. Returns False when the write is skipped."""
        comm = self._df._comm
        exists = os.path.exists(path) and bool(os.listdir(path)) if os.path.isdir(path) else os.path.exists(path)
        if exists:
            if self._mode in ("error", "errorifexists"):
                raise FileExistsError(f"path {path} already exists")
            if self._mode == "ignore":
                return False
            if self._mode == "overwrite":
                comm.barrier()
                if comm.is_root:
                    shutil.rmtree(path) if os.path.isdir(path) else os.remove(path)
                comm.barrier()
        os.makedirs(path, exist_ok=True)
        comm.barrier()
        return True

    def save(self, path: Optional[str] = None, format: Optional[str] = None, mode: Optional[str] = None, **opts):
        if format:
            self.format(format)
        if mode:
            self.mode(mode)
        path = strip_scheme(path)
        f = self._format
        if f in ("delta", "table"):
            from . import table
            table.write_frame(self._df, path, self._mode)
            return
        if f == "parquet":
            return self.parquet(path)
        if f == "csv":
            return self.csv(path)
        if f == "json":
            return self.json(path)
        if f == "orc":
            return self.orc(path)
        if f == "text":
            return self.text(path)
        raise ValueError(f"unsupported format {f}")

    def _write(self, path: str, write_part) -> None:
        """Save mode, optional Hive partitioning (``partitionBy``), one part file per rank, _SUCCESS."""
        path = strip_scheme(path)
        if not self._prepare_dir(path):
            return
        if self._partition_by:
            from .partition import write_partitioned

            def one(sub, d):
                os.makedirs(d, exist_ok=True)
                if sub._nrows:
                    write_part(sub, d)
            write_partitioned(self._df, path, list(self._partition_by), one)
        else:
            write_part(self._df, path)
        self._success(path)

    def orc(self, path: str, mode: Optional[str] = None):
        import pyarrow.orc as orc
        from .arrow import frame_to_arrow
        if mode:
            self.mode(mode)
        self._write(path, lambda df, d: orc.write_table(frame_to_arrow(df), self._part(d, "orc", df)))

    def text(self, path: str, mode: Optional[str] = None):
        from ..sql.dataframe import column_to_python
        if mode:
            self.mode(mode)
        if len(self._df.columns) - len(self._partition_by or ()) != 1:
            raise ValueError("text data source supports only a single column")

        def w(df, d):
            with open(self._part(d, "txt", df), "w") as fh:
                for v in column_to_python(df._column_data(df.columns[0])):
                    fh.write(("" if v is None else str(v)) + "\n")
        self._write(path, w)

    def _part(self, path: str, ext: str, df=None) -> str:
        comm = self._df._comm
        import uuid
        return os.path.join(path, f"part-{comm.rank:05d}-{uuid.uuid4().hex[:8]}.{ext}")

    def _success(self, path: str):
        comm = self._df._comm
        comm.barrier()
        if comm.is_root:
            open(os.path.join(path, "_SUCCESS"), "w").close()
        comm.barrier()

    def parquet(self, path: str, mode: Optional[str] = None):
        import pyarrow.parquet as pq
        from .arrow import frame_to_arrow
        if mode:
            self.mode(mode)
        comp = self._options.get("compression", "snappy")
        self._write(path, lambda df, d: pq.write_table(frame_to_arrow(df), self._part(d, "parquet", df),
                                                      compression=None if comp in ("none", "uncompressed")
                                                      else comp))

    def csv(self, path: str, mode: Optional[str] = None, header=None, sep=None):
        if mode:
            self.mode(mode)
        if header is not None:
            self.option("header", header)
        if sep is not None:
            self.option("sep", sep)
        hdr = str(self._options.get("header", "false")).lower() == "true"
        self._write(path, lambda df, d: self._local_pandas(df, csv=True).to_csv(self._part(d, "csv", df), index=False,
                                                                     header=hdr, sep=self._options.get("sep", ",")))

    def json(self, path: str, mode: Optional[str] = None):
        if mode:
            self.mode(mode)
        self._write(path, lambda df, d: self._json_lines(df, self._part(d, "json", df)))

    @staticmethod
    def _json_lines(df, path: str) -> None:
        """JSON Lines as Spark writes them: one object per row, null fields omitted (ignoreNullFields),
        doubles with every significant digit (shortest repr round-trips; pandas' to_json keeps 10),
        NaN / ±Infinity as the quoted strings Spark writes."""
        import datetime
        import decimal
        import json
        import math
        from ..sql.dataframe import column_to_python

        def conv(v):
            if isinstance(v, float):
                # Spark writes non-finite doubles as the strings "NaN" / "Infinity" / "-Infinity" and
                # reads them back (allowNonNumericNumbers): NaN must not turn into a missing field
                if math.isnan(v):
                    return "NaN"
                if math.isinf(v):
                    return "Infinity" if v > 0 else "-Infinity"
                return v
            if isinstance(v, datetime.datetime):
                return v.isoformat(timespec="milliseconds")
            if isinstance(v, datetime.date):
                return v.isoformat()
            if isinstance(v, decimal.Decimal):
                return float(v)
            if hasattr(v, "toArray"):
                return v.toArray().tolist()
            if hasattr(v, "asDict"):
                return {k: conv(x) for k, x in v.asDict().items()}
            if isinstance(v, dict):
                return {str(k): conv(x) for k, x in v.items()}
            if isinstance(v, (list, tuple)):
                return [conv(x) for x in v]
            if isinstance(v, (bytes, bytearray)):
                import base64
                return base64.b64encode(bytes(v)).decode()
            return v

        cols = [(f.name, column_to_python(df._cols[f.name])) for f in df.schema.fields]
        n = len(cols[0][1]) if cols else 0
        with open(path, "w") as fh:
            for i in range(n):
                rec = {}
                for name, vals in cols:
                    v = conv(vals[i])
                    if v is not None:
                        rec[name] = v
                fh.write(json.dumps(rec, allow_nan=False, separators=(",", ":"), ensure_ascii=False) + "\n")

    def _local_pandas(self, df=None, csv: bool = False):
        import pandas as pd
        from ..sql.dataframe import column_to_python
        df = self._df if df is None else df
        from ..sql import types as T
        data = {}
        for f in df.schema.fields:
            vals = column_to_python(df._cols[f.name])
            vals = [v.toArray().tolist() if hasattr(v, "toArray") else v for v in vals]
            if isinstance(f.dataType, (T.ByteType, T.ShortType, T.IntegerType, T.LongType)):
                vals = pd.array(vals, dtype="Int64")  # nulls stay empty cells, integers stay integers (not 0.0)
            elif csv and isinstance(f.dataType, T.BooleanType):
                vals = [None if v is None else ("true" if v else "false") for v in vals]  # Spark's spelling
            data[f.name] = vals
        return pd.DataFrame(data, columns=df.columns)

    def saveAsTable(self, name: str, format: Optional[str] = None, mode: Optional[str] = None):
        if mode:
            self.mode(mode)
        self._df._session.catalog._save_table(name, self._df, self._mode)

    def insertInto(self, tableName: str, overwrite: bool = False):
        self.mode("overwrite" if overwrite else "append")
        self._df._session.catalog._save_table(tableName, self._df, self._mode)
