"""spark.read — DataFrameReader (csv / parquet / json / table / delta-style table paths)."""
from __future__ import annotations

import glob
import os
from typing import Dict, List, Optional, Union

from ..sql import types as T


def expand_paths(path: Union[str, List[str]], exts=None) -> List[str]:
    paths = [path] if isinstance(path, str) else list(path)
    out: List[str] = []
    for p in paths:
        p = strip_scheme(p)
        if os.path.isdir(p):
            for root, dirs, files in os.walk(p):
                dirs[:] = sorted(d for d in dirs if not d.startswith(("_", ".")))
                for f in sorted(files):
                    if f.startswith(("_", ".")):
                        continue
                    if exts and not any(f.endswith(e) for e in exts):
                        continue
                    out.append(os.path.join(root, f))
        elif any(ch in p for ch in "*?["):
            out += sorted(glob.glob(p))
        else:
            out.append(p)
    return out


def strip_scheme(p: str) -> str:
    """file:// paths are local; hdfs://host:port/x maps onto the local warehouse root (no HDFS here)."""
    if p.startswith("file://"):
        return p[len("file://"):]
    if p.startswith("hdfs://"):
        rest = p[len("hdfs://"):]
        rest = rest.split("/", 1)[1] if "/" in rest else ""
        base = os.environ.get("CML_HDFS_ROOT", os.path.join(os.getcwd(), "hdfs"))
        return os.path.join(base, rest)
    return p


class DataFrameReader:
    def __init__(self, session):
        self._session = session
        self._format = "parquet"
        self._schema: Optional[T.StructType] = None
        self._options: Dict[str, str] = {}

    def format(self, source: str) -> "DataFrameReader":
        self._format = source.lower()
        return self

    def schema(self, schema) -> "DataFrameReader":
        self._schema = T.parse_ddl_schema(schema) if isinstance(schema, str) else schema
        return self

    def option(self, key: str, value) -> "DataFrameReader":
        self._options[key.lower()] = value
        return self

    def options(self, **opts) -> "DataFrameReader":
        for k, v in opts.items():
            self.option(k, v)
        return self

    def _bool(self, key, default=False) -> bool:
        v = self._options.get(key, default)
        return v if isinstance(v, bool) else str(v).lower() == "true"

    def load(self, path=None, format=None, schema=None, **options):
        if format:
            self.format(format)
        if schema is not None:
            self.schema(schema)
        for k, v in options.items():
            self.option(k, v)
        f = self._format
        if f == "csv":
            return self.csv(path)
        if f == "parquet":
            return self.parquet(path)
        if f == "json":
            return self.json(path)
        if f == "orc":
            return self.orc(path)
        if f == "text":
            return self.text(path)
        if f in ("delta", "table"):
            from . import table
            return table.read_table(self._session, strip_scheme(path), self._options.get("versionasof"))
        raise ValueError(f"unsupported format {f}")

    def csv(self, path, schema=None, sep=None, header=None, inferSchema=None, **kw):
        from .csv import read_csv_files
        if schema is not None:
            self.schema(schema)
        if header is not None:
            self.option("header", header)
        if sep is not None:
            self.option("sep", sep)
        if inferSchema is not None:
            self.option("inferschema", inferSchema)
        files = expand_paths(path)
        sch = self._schema

        def read(fs, ids=None):
            return read_csv_files(self._session, fs, sch, self._bool("header"),
                                  sep=str(self._options.get("sep", self._options.get("delimiter", ","))),
                                  quote=str(self._options.get("quote", '"')), infer=self._bool("inferschema"),
                                  file_ids=ids)
        return self._maybe_partitioned(path, files, read)

    def _maybe_partitioned(self, path, files, read):
        """Hive partition discovery: ``col=value`` directories become typed columns."""
        from .partition import read_partitioned
        bases = [strip_scheme(p) for p in ([path] if isinstance(path, str) else list(path))]
        bases = [b for b in bases if os.path.isdir(b)]
        if bases and files:
            out = read_partitioned(self._session, files, bases, read)
            if out is not None:
                return out
        return read(files)

    def orc(self, path):
        import pyarrow as pa
        import pyarrow.orc as orc
        from .arrow import frame_from_arrow
        from ..sql.builder import shard_range
        files = expand_paths(path, exts=[".orc"])

        def read(fs, ids=None):
            tabs = [orc.read_table(f) for f in fs]
            table = pa.concat_tables(tabs) if len(tabs) > 1 else (tabs[0] if tabs else pa.table({}))
            comm = self._session._comm
            a, b = shard_range(table.num_rows, comm.rank, comm.world_size)
            base = (min(ids) << 40) if ids else 0
            return frame_from_arrow(self._session, table.slice(a, b - a), list(range(base + a, base + b)))
        return self._maybe_partitioned(path, files, read)

    def parquet(self, *paths):
        from .arrow import read_parquet_files
        from . import table
        files: List[str] = []
        for p in paths:
            sp = strip_scheme(p)
            if os.path.isdir(sp) and table.exists(sp):
                return table.read_table(self._session, sp)
            files += expand_paths(p, exts=[".parquet"])
        sch = self._schema
        return self._maybe_partitioned(list(paths), files,
                                       lambda fs, ids=None: read_parquet_files(self._session, fs, sch, file_ids=ids))

    def json(self, path, schema=None):
        import pandas as pd
        import pyarrow as pa
        from .arrow import frame_from_arrow
        from ..sql.builder import shard_range
        if schema is not None:
            self.schema(schema)
        files = expand_paths(path)
        # precise_float: exact round trip of the writer's shortest-repr doubles (the default parser rounds)
        frames = [pd.read_json(f, lines=True, precise_float=True) for f in files]
        pdf = pd.concat(frames, ignore_index=True) if frames else pd.DataFrame()
        if self._schema is not None and pdf.shape[1] == 0 and len(pdf):
            # every record is {} (Spark omits null fields): a placeholder column keeps the row count through
            # Arrow (a column-less table has no rows); the schema select below drops it
            pdf["__cml_rows"] = 0
        special = _non_numeric_numbers(pdf, files)
        comm = self._session._comm
        a, b = shard_range(len(pdf), comm.rank, comm.world_size)
        table = pa.Table.from_pandas(pdf.iloc[a:b], preserve_index=False)
        for c, vals in special.items():  # NaN is a value there, not a null: build the column directly
            i = table.schema.get_field_index(c)
            table = table.set_column(i, c, pa.array(vals[a:b], type=pa.float64(), from_pandas=False))
        df = frame_from_arrow(self._session, table, list(range(a, b)))
        if self._schema is not None:
            from ..sql import functions as F
            # a field no record carries (Spark omits null fields when writing) reads as an all-null column
            df = df.select(*[(df[f.name] if f.name in df.columns else F.lit(None)).cast(f.dataType).alias(f.name)
                             for f in self._schema.fields])
        return df

    def table(self, name: str):
        return self._session.table(name)

    def text(self, path):
        from ..sql.builder import frame_from_pycolumns, shard_range
        lines: List[str] = []
        for f in expand_paths(path):
            with open(f) as fh:
                lines += fh.read().splitlines()
        comm = self._session._comm
        a, b = shard_range(len(lines), comm.rank, comm.world_size)
        schema = T.StructType([T.StructField("value", T.StringType())])
        return frame_from_pycolumns(self._session, schema, {"value": lines[a:b]}, list(range(a, b)))


_NON_NUMERIC = {"NaN": float("nan"), "Infinity": float("inf"), "+Infinity": float("inf"), "-Infinity": float("-inf"),
                "INF": float("inf"), "+INF": float("inf"), "-INF": float("-inf")}


def _non_numeric_numbers(pdf, files) -> dict:
    """Spark's allowNonNumericNumbers (default on): non-finite doubles written as "NaN" / "Infinity" /
    "-Infinity" strings read back as those values. pandas parses them but cannot keep a NaN apart from
    a missing field (both become NaN), so when a file carries such strings the numeric columns are
    rebuilt from the records: {column: python values, None for a missing or null field}."""
    import json
    import math
    import numbers
    # only columns pandas typed float-with-NaN or object-holding-such-a-string can be affected: with none,
    # the files are not read a second time (any quoted "NaN" inside an ordinary string value
    # used to trigger a full re-parse of every record)
    cand = []
    for c in pdf.columns:
        col = pdf[c]
        if col.dtype.kind == "f":
            if bool(col.isna().any()):
                cand.append(c)
        elif col.dtype == object:
            if any((isinstance(v, str) and v in _NON_NUMERIC) or (isinstance(v, float) and math.isnan(v))
                   for v in col):
                cand.append(c)
    if not cand:
        return {}
    texts = []
    for f in files:
        with open(f, encoding="utf-8") as fh:
            texts.append(fh.read())
    if not any(any(f'"{w}"' in t for w in _NON_NUMERIC) for t in texts):
        return {}
    recs = [json.loads(line) for t in texts for line in t.splitlines() if line.strip()]
    if len(recs) != len(pdf):
        return {}
    out = {}
    for c in cand:
        vals = [r.get(c) for r in recs]
        present = [v for v in vals if v is not None]
        if not any(isinstance(v, str) and v in _NON_NUMERIC for v in present):
            continue
        if not all((isinstance(v, str) and v in _NON_NUMERIC) or
                   (isinstance(v, numbers.Number) and not isinstance(v, bool)) for v in present):
            continue
        if not any(isinstance(v, numbers.Number) for v in present):
            # only strings (no JSON number at all): Spark's inference keeps a string column
            pdf[c] = pd_object(vals)
            continue
        out[c] = [None if v is None else (_NON_NUMERIC[v] if isinstance(v, str) else float(v)) for v in vals]
        pdf[c] = [0.0 if v is None or (isinstance(v, float) and math.isnan(v)) else v for v in out[c]]
    return out


def pd_object(vals):
    """A pandas object column holding exactly ``vals`` (strings and None, no NaN coercion)."""
    import pandas as pd
    return pd.Series(vals, dtype=object)
