"""Structured-streaming micro-batch engine (N5) — the reference's ingest path
(ref.py:75-118): file source over a directory of CSV uploads, event-time watermark,
per-batch ``current_timestamp()`` ingest time, ``foreachBatch`` per-batch hook and
an append-only table sink with a checkpoint directory.

Exactly-once: each micro-batch is planned by writing ``offsets/<id>`` (the files it
covers, the batch timestamp and watermark) before it runs and ``commits/<id>`` after
its sink finished.  On restart an offsets entry without a commit is re-run with the
*same* files and timestamp; the table sink skips batches whose (queryId, batchId)
transaction is already in the table log, so a crash between the sink commit and the
checkpoint commit cannot duplicate rows.

Stateful operators: a streaming ``groupBy().agg()`` keeps per-group partial aggregates (the same
partials the batch aggregation merges across ranks) in a versioned state checkpoint
(``state/<id>``, written before the commit) and emits all groups (``complete``), the updated
groups (``update``) or the groups whose event-time window the watermark passed (``append``);
``dropDuplicates`` keeps the seen keys. Late rows (event time behind the watermark) are dropped.

Defects of the reference are not reproduced: ``foreachBatch``
calls ``fn(df, batch_id)``; ``.table(name)`` is accepted as an alias of
``toTable``; when both a foreachBatch function and a table target are given, each
batch is appended to the table first and then handed to the function.

Multi-rank (SPMD) runs: rank 0 lists the directory and plans the batch, the plan
is broadcast, every rank reads its share of the batch's files.  Micro-batches run
in the caller's thread there (``processAllAvailable`` / ``availableNow`` /
``awaitTermination``) so collectives never race with the main program; a
single-process query with a processing-time trigger runs on a background thread.
"""
from __future__ import annotations

import json
import logging

from ..utils.fault import maybe_fail
from ..utils.trace import trace
import os
import re
import threading
import time
import uuid
from typing import Any, Callable, Dict, List, Optional

from . import types as T

log = logging.getLogger("cml.streaming")


def parse_interval_ms(s) -> int:
    if isinstance(s, (int, float)):
        return int(s)
    m = re.fullmatch(r"\s*(\d+(?:\.\d+)?)\s*(ms|millisecond|milliseconds|s|sec|second|seconds|min|minute|minutes|"
                     r"h|hour|hours|d|day|days)?\s*", str(s).lower())
    if not m:
        raise ValueError(f"bad interval {s!r}")
    v = float(m.group(1))
    unit = m.group(2) or "ms"
    mult = {"ms": 1, "millisecond": 1, "milliseconds": 1, "s": 1000, "sec": 1000, "second": 1000,
            "seconds": 1000, "min": 60000, "minute": 60000, "minutes": 60000, "h": 3600000, "hour": 3600000,
            "hours": 3600000, "d": 86400000, "day": 86400000, "days": 86400000}[unit]
    return int(v * mult)


class StreamPlan:
    """Source description + recorded per-batch transformations."""

    def __init__(self, fmt: str, path: str, schema: T.StructType, options: Dict[str, Any], ops=None):
        self.fmt, self.path, self.schema, self.options = fmt, path, schema, options
        self.ops = list(ops or [])
        self.watermark = None

    def extend(self, method, args, kwargs) -> "StreamPlan":
        p = StreamPlan(self.fmt, self.path, self.schema, self.options, self.ops + [(method, args, kwargs)])
        p.watermark = self.watermark
        return p


class DataStreamReader:
    def __init__(self, session):
        self._session = session
        self._format = "parquet"
        self._schema: Optional[T.StructType] = None
        self._options: Dict[str, Any] = {}

    def format(self, source: str) -> "DataStreamReader":
        self._format = source.lower()
        return self

    def schema(self, schema) -> "DataStreamReader":
        self._schema = T.parse_ddl_schema(schema) if isinstance(schema, str) else schema
        return self

    def option(self, key, value) -> "DataStreamReader":
        self._options[key.lower()] = value
        return self

    def options(self, **opts) -> "DataStreamReader":
        for k, v in opts.items():
            self.option(k, v)
        return self

    def load(self, path: Optional[str] = None, format: Optional[str] = None, schema=None, **options):
        if format:
            self.format(format)
        if schema is not None:
            self.schema(schema)
        for k, v in options.items():
            self.option(k, v)
        return self._frame(path)

    def csv(self, path: str, schema=None, **kw):
        self.format("csv")
        return self.load(path, schema=schema, **kw)

    def parquet(self, path: str):
        self.format("parquet")
        return self.load(path)

    def json(self, path: str, schema=None):
        self.format("json")
        return self.load(path, schema=schema)

    def _frame(self, path: str):
        from ..io.reader import strip_scheme
        from .dataframe import DataFrame
        if self._schema is None:
            raise ValueError("Schema must be specified when creating a streaming source DataFrame")
        plan = StreamPlan(self._format, strip_scheme(path), self._schema, dict(self._options))
        return DataFrame(self._session, self._schema, {}, 0, None, self._session._device, plan)


class DataStreamWriter:
    def __init__(self, df):
        self._df = df
        self._format = None
        self._mode = "append"
        self._options: Dict[str, Any] = {}
        self._foreach_batch: Optional[Callable] = None
        self._trigger: Dict[str, Any] = {"processingTime": 0}
        self._name: Optional[str] = None

    def format(self, source: str) -> "DataStreamWriter":
        self._format = source.lower()
        return self

    def outputMode(self, mode: str) -> "DataStreamWriter":
        m = mode.lower()
        if m not in ("append", "update", "complete"):
            raise ValueError(f"unknown output mode {mode}")
        self._mode = m
        return self

    def option(self, key, value) -> "DataStreamWriter":
        self._options[key.lower()] = value
        return self

    def options(self, **opts) -> "DataStreamWriter":
        for k, v in opts.items():
            self.option(k, v)
        return self

    def queryName(self, name: str) -> "DataStreamWriter":
        self._name = name
        return self

    def foreachBatch(self, func: Callable) -> "DataStreamWriter":
        self._foreach_batch = func
        return self

    def trigger(self, processingTime=None, once=None, availableNow=None, continuous=None) -> "DataStreamWriter":
        if once:
            self._trigger = {"once": True}
        elif availableNow:
            self._trigger = {"availableNow": True}
        elif processingTime is not None:
            self._trigger = {"processingTime": parse_interval_ms(processingTime)}
        elif continuous is not None:
            raise NotImplementedError("continuous processing is not supported; use micro-batches")
        return self

    def partitionBy(self, *cols) -> "DataStreamWriter":
        return self

    def toTable(self, tableName: str, format=None, outputMode=None, partitionBy=None, queryName=None, **options):
        if outputMode:
            self.outputMode(outputMode)
        if queryName:
            self.queryName(queryName)
        for k, v in options.items():
            self.option(k, v)
        return self._start(table=tableName)

    # the reference calls DataStreamWriter.table(...) (ref.py:115); accept it as toTable
    table = toTable

    def start(self, path: Optional[str] = None, format=None, outputMode=None, queryName=None, **options):
        if format:
            self.format(format)
        if outputMode:
            self.outputMode(outputMode)
        if queryName:
            self.queryName(queryName)
        for k, v in options.items():
            self.option(k, v)
        return self._start(path=path or self._options.get("path"))

    def _start(self, table: Optional[str] = None, path: Optional[str] = None):
        session = self._df._session
        plan = self._df._stream
        has_agg = any(m == "_stream_aggregate" for m, _, _ in plan.ops)
        if self._mode == "complete" and not has_agg:
            raise ValueError("Complete output mode not supported when there are no streaming aggregations")
        if self._mode == "append" and has_agg and not plan.watermark:
            raise ValueError("Append output mode not supported when there are streaming aggregations without "
                             "watermark")
        if self._mode == "update" and has_agg and (table is not None or path is not None):
            raise ValueError("update output mode is not supported by table / file sinks; use foreachBatch or "
                             "the memory / console sinks")
        if table is not None and not has_agg and not session.catalog.tableExists(table):
            # like Spark's toTable: the sink table exists (empty, with the stream's schema) from the start,
            # so readers of the unbounded table do not fail before the first file arrives
            session.catalog.createTable(table, schema=self._df.schema)
        q = StreamingQuery(session, self._df._stream, self, table=table, path=path)
        session.streams._register(q)
        q._launch()
        return q


class StreamingQuery:
    def __init__(self, session, plan: StreamPlan, writer: DataStreamWriter, table=None, path=None):
        from ..io.reader import strip_scheme
        self._session = session
        self._plan = plan
        self._writer = writer
        self._table = table
        self._path = strip_scheme(path) if path else None
        self.name = writer._name
        ckpt = writer._options.get("checkpointlocation")
        if ckpt is None:
            ckpt = os.path.join(session.catalog.warehouse, "_checkpoints", table or self.name or uuid.uuid4().hex)
        self._ckpt = strip_scheme(ckpt)
        self.runId = uuid.uuid4().hex
        self._watermark_ms = 0
        self.id = self._load_or_create_id()
        self._stop = threading.Event()
        self._thread: Optional[threading.Thread] = None
        self._error: Optional[BaseException] = None
        self.recentProgress: List[dict] = []
        self._lock = threading.Lock()
        self._next_batch = None
        self._batch_wm = 0          # watermark (ms) the running batch started with
        self._wm_source = None      # frame the watermark column is read from (pre-aggregation)
        self._state = self._load_state()  # stateful operators: {op index: state}

    # ------------------------------------------------------------------ checkpoint files
    def _load_or_create_id(self) -> str:
        """Query id from ``metadata`` (created on first start); also restores the event-time
        watermark from the last commit, so a restarted query does not fall back to 0."""
        comm = self._session._comm
        state = None
        if comm.is_root:
            os.makedirs(os.path.join(self._ckpt, "offsets"), exist_ok=True)
            os.makedirs(os.path.join(self._ckpt, "commits"), exist_ok=True)
            os.makedirs(os.path.join(self._ckpt, "sources", "0"), exist_ok=True)
            meta = os.path.join(self._ckpt, "metadata")
            if os.path.exists(meta):
                with open(meta) as fh:
                    qid = json.load(fh)["id"]
            else:
                qid = uuid.uuid4().hex
                with open(meta, "w") as fh:
                    json.dump({"id": qid}, fh)
            commits = self._ids("commits")
            wm = int(self._read_json("commits", commits[-1]).get("nextBatchWatermarkMs", 0)) if commits else 0
            state = (qid, wm)
        qid, wm = comm.broadcast_object(state)
        self._watermark_ms = wm
        return qid

    def _ids(self, sub: str) -> List[int]:
        d = os.path.join(self._ckpt, sub)
        return sorted(int(f) for f in os.listdir(d) if f.isdigit()) if os.path.isdir(d) else []

    def _read_json(self, sub: str, bid: int):
        with open(os.path.join(self._ckpt, sub, str(bid))) as fh:
            return json.load(fh)

    def _write_json(self, sub: str, bid: int, obj) -> None:
        p = os.path.join(self._ckpt, sub, str(bid))
        tmp = p + ".tmp"
        with open(tmp, "w") as fh:
            json.dump(obj, fh)
        os.replace(tmp, p)

    def _load_state(self) -> Dict[int, Any]:
        """State of the stateful operators after the last committed batch (``state/<batch id>``,
        written by this engine before the commit), identical on every rank."""
        from ..utils import jsonstate
        comm = self._session._comm
        st = None
        if comm.is_root:
            commits = self._ids("commits")
            p = os.path.join(self._ckpt, "state", str(commits[-1])) if commits else None
            if p and os.path.exists(p):
                # tagged JSON (utils/jsonstate.py): a shared checkpoint directory can never run code
                with open(p, encoding="utf-8") as fh:
                    try:
                        st = jsonstate.loads(fh.read())
                    except (ValueError, UnicodeDecodeError) as e:
                        raise ValueError(f"streaming state file {p} is not a state record of this engine "
                                         f"(tagged JSON): {e}") from None
                st = {int(k): v for k, v in st.items()}
        return comm.broadcast_object(st) or {}

    def _save_state(self, bid: int) -> None:
        from ..utils import jsonstate
        if not self._state or not self._session._comm.is_root:
            return
        d = os.path.join(self._ckpt, "state")
        os.makedirs(d, exist_ok=True)
        tmp = os.path.join(d, f"{bid}.tmp")
        with open(tmp, "w", encoding="utf-8") as fh:
            fh.write(jsonstate.dumps(self._state))
            fh.flush()
            os.fsync(fh.fileno())
        os.replace(tmp, os.path.join(d, str(bid)))
        for old in self._ids("state"):
            if old < bid - 2:  # keep a short history (replays only ever need the last committed one)
                try:
                    os.remove(os.path.join(d, str(old)))
                except OSError:
                    pass

    def _seen_files(self) -> List[str]:
        """Files of every PLANNED batch, in batch order. The offsets log is the write-ahead record
        of a plan (written first), so a file counts as seen only once its batch has an offsets
        entry: a crash between the two planning writes can never hide a file."""
        seen: List[str] = []
        for bid in self._ids("offsets"):
            seen += self._read_json("offsets", bid)["files"]
        return seen

    # ------------------------------------------------------------------ planning (rank 0)
    def _list_new(self, seen: set) -> List[str]:
        d = self._plan.path
        if not os.path.isdir(d):
            return []
        ext = {"csv": (".csv", ".txt", ".csv.gz"), "json": (".json", ".jsonl"), "parquet": (".parquet",)}.get(
            self._plan.fmt)
        files = []
        for root, dirs, fs in os.walk(d):
            dirs[:] = sorted(x for x in dirs if not x.startswith(("_", ".")))
            for f in fs:
                if f.startswith(("_", ".")) or f.endswith((".tmp", ".crc")):
                    continue
                if ext and not f.endswith(ext):
                    continue
                p = os.path.join(root, f)
                if p not in seen:
                    files.append(p)
        files.sort(key=lambda p: (os.path.getmtime(p), p))
        mf = self._plan.options.get("maxfilespertrigger")
        if mf:
            files = files[: int(mf)]
        return files

    def _plan_next(self):
        """Decide the next batch on rank 0: (batch_id, files, ts_ms, watermark_ms, is_replay) or None."""
        comm = self._session._comm
        plan = None
        if comm.is_root:
            offs, commits = self._ids("offsets"), self._ids("commits")
            last_commit = commits[-1] if commits else -1
            if offs and offs[-1] > last_commit:
                bid = offs[-1]
                o = self._read_json("offsets", bid)
                plan = (bid, o["files"], o["batchTimestampMs"], o["batchWatermarkMs"], True)
                if not os.path.exists(os.path.join(self._ckpt, "sources", "0", str(bid))):
                    self._write_json(os.path.join("sources", "0"), bid, {"files": o["files"]})
            else:
                seen = set(self._seen_files())
                new = self._list_new(seen)
                if new:
                    bid = last_commit + 1
                    ts = int(time.time() * 1000)
                    plan = (bid, new, ts, self._watermark_ms, False)
                    # offsets (the WAL) first: once it exists the batch replays after any crash;
                    # sources/0 is the file-source log of the same plan (re-written on replay)
                    self._write_json("offsets", bid, {"batchId": bid, "files": new, "batchTimestampMs": ts,
                                                      "batchWatermarkMs": self._watermark_ms,
                                                      "queryId": self.id})
                    maybe_fail("stream.between_plan_writes", bid)
                    self._write_json(os.path.join("sources", "0"), bid, {"files": new})
        return comm.broadcast_object(plan)

    # ------------------------------------------------------------------ execution
    def _file_ids(self, files: List[str]) -> List[int]:
        order = {}
        for i, f in enumerate(self._seen_files_cached()):
            order.setdefault(f, i)
        return [order.get(f, hash(f) & 0xFFFFF) for f in files]

    def _seen_files_cached(self):
        comm = self._session._comm
        return comm.broadcast_object(self._seen_files() if comm.is_root else None)

    def _read_batch(self, files: List[str], ts_ms: int):
        from ..io.arrow import read_parquet_files
        from ..io.csv import read_csv_files
        s = self._session
        opts = self._plan.options
        fids = self._file_ids(files)
        if self._plan.fmt == "csv":
            hdr = opts.get("header", False)
            hdr = hdr if isinstance(hdr, bool) else str(hdr).lower() == "true"
            df = read_csv_files(s, files, self._plan.schema, hdr, sep=str(opts.get("sep", ",")),
                                quote=str(opts.get("quote", '"')), file_ids=fids)
        elif self._plan.fmt == "parquet":
            df = read_parquet_files(s, files, self._plan.schema, file_ids=fids)
        elif self._plan.fmt == "json":
            df = s.read.schema(self._plan.schema).json(files)
        else:
            raise ValueError(f"unsupported streaming source format {self._plan.fmt}")
        df._batch_time_us = int(ts_ms) * 1000
        self._wm_source = None
        for i, (method, args, kwargs) in enumerate(self._plan.ops):
            if method == "withWatermark":
                self._wm_source = df
                continue
            if method == "_stream_aggregate":
                if self._wm_source is None:
                    self._wm_source = df
                df = self._stateful_aggregate(i, df, *args)
            elif method == "_stream_dedup":
                df = self._stateful_dedup(i, df, *args)
            else:
                df = getattr(df, method)(*args, **kwargs)
            df._batch_time_us = int(ts_ms) * 1000
        return df

    # ------------------------------------------------------------------ stateful operators
    def _late_mask(self, df):
        """Rows at or after the batch's watermark (late rows are dropped by stateful operators)."""
        import torch
        wm = self._plan.watermark
        if not wm or self._batch_wm <= 0 or wm[0] not in df.columns:
            return None
        cd = df._column_data(wm[0])
        if cd.is_host:
            return None
        return cd.values.to(torch.int64) >= self._batch_wm * 1000

    def _expired(self, key: tuple, key_exprs) -> bool:
        """A group whose event time is behind the watermark: its time-window ends at or before it, or
        its key is the watermark column itself and is older."""
        from .column import ColRef, ts_to_micros
        wm = self._plan.watermark
        if not wm:
            return False
        lim = self._batch_wm * 1000
        for v, e in zip(key, key_exprs):
            end = getattr(v, "end", None) if hasattr(v, "__fields__") else None
            if end is not None:
                return ts_to_micros(end) <= lim
            if isinstance(e, ColRef) and e.col == wm[0] and v is not None:
                return ts_to_micros(v) < lim
        return False

    def _stateful_aggregate(self, idx: int, df, keys, exprs):
        """Streaming groupBy().agg(): this batch's partials are merged into the per-group state; the
        output is every group (complete), the groups this batch touched (update), or the groups whose
        event-time window the watermark has passed, which then leave the state (append)."""
        from .builder import rows_round_robin
        from .group import (combine_partials, final_row, fix_long_columns, gather_partials, local_partials,
                            result_schema)
        keep = self._late_mask(df)
        if keep is not None:
            df = df._mask_rows(keep)
        st = self._state.setdefault(idx, {})
        touched = []
        from .window import SessionWindow
        if any(isinstance(k, SessionWindow) for k in keys):
            df, keys, touched = self._merge_sessions(st, df, keys, exprs)
        specs, key_types, local = local_partials(df, keys, exprs)
        merged, morder = gather_partials(self._session._comm, local, len(specs))
        for key in morder:
            cur = st.get(key)
            new = []
            for j, sp in enumerate(specs):
                if sp[0] == "key":
                    new.append(None)
                elif getattr(sp[2], "custom", False):
                    new.append((cur[j] if cur else []) + merged[key][j])
                else:
                    prev = [cur[j]] if cur is not None and cur[j] is not None else []
                    new.append(combine_partials(prev + merged[key][j], sp[2].fn))
            st[key] = new
            if key not in touched:
                touched.append(key)
        mode = self._writer._mode
        if mode == "complete":
            out = list(st)
        elif mode == "update":
            out = touched
        else:
            out = [k for k in st if self._expired(k, keys)]

        def parts_of(key):
            return [[] if sp[0] == "key" else (st[key][j] if getattr(sp[2], "custom", False)
                                              else [st[key][j]] if st[key][j] is not None else [])
                    for j, sp in enumerate(specs)]
        rows = [final_row(k, parts_of(k), specs) for k in out]
        if mode != "complete":  # evict groups the watermark has passed
            for k in [k for k in st if self._expired(k, keys)]:
                del st[k]
        schema = result_schema(specs, key_types)
        fix_long_columns(schema, rows)
        return rows_round_robin(self._session, schema, rows)

    def _merge_sessions(self, st, df, keys, exprs):
        """Session windows across micro-batches (Spark's merging session state store): the state's
        sessions of every key are merged with this batch's events — an event inside a session
        extends it, one between two sessions joins them — and the state is re-keyed to the merged
        sessions (their partials combined) before this batch's partials are added."""
        from .column import micros_to_datetime, ts_to_micros
        from .group import combine_partials, local_partials
        from .types import Row
        from .window import SessionWindow, materialize_sessions
        j = next(i for i, k in enumerate(keys) if isinstance(k, SessionWindow))
        prior = {}
        for key in st:
            sw = key[j]
            prior.setdefault(key[:j] + key[j + 1:], []).append((ts_to_micros(sw.start), ts_to_micros(sw.end)))
        df, keys2, remap = materialize_sessions(df, keys, prior)
        specs = local_partials(df._session._empty_frame(df.schema), keys2, exprs)[0]
        touched = []
        for key in list(st):
            ok = key[:j] + key[j + 1:]
            old = (ts_to_micros(key[j].start), ts_to_micros(key[j].end))
            new = remap.get((ok, old), old)
            if new == old:
                continue
            nk = key[:j] + (Row(start=micros_to_datetime(new[0]), end=micros_to_datetime(new[1])),) + key[j + 1:]
            cur, add = st.pop(key), None
            add = st.get(nk)
            if add is None:
                st[nk] = cur
            else:
                comb = []
                for i, sp in enumerate(specs):
                    if sp[0] == "key":
                        comb.append(None)
                    elif getattr(sp[2], "custom", False):
                        comb.append(add[i] + cur[i])
                    else:
                        parts = [p for p in (add[i], cur[i]) if p is not None]
                        comb.append(combine_partials(parts, sp[2].fn) if parts else None)
                st[nk] = comb
            if nk not in touched:
                touched.append(nk)
        return df, keys2, touched

    def _stateful_dedup(self, idx: int, df, subset):
        """Streaming dropDuplicates: a row passes if its key was never seen in an earlier batch and it
        is the key's first row in this batch (rank order, then row order). With a watermark on a key
        column, keys older than the watermark leave the state and late rows are dropped."""
        import torch
        from .dataframe import column_to_python
        from .group import _hashable
        keep_late = self._late_mask(df)
        if keep_late is not None:
            df = df._mask_rows(keep_late)
        cols = list(subset) if subset else df.columns
        vals = [column_to_python(df._column_data(c)) for c in cols]
        keys = [tuple(_hashable(v[i]) for v in vals) for i in range(df._nrows)]
        seen = self._state.setdefault(idx, {})
        comm = self._session._comm
        allk = comm.allgather_object(keys)
        mask_all, newseen = [], {}
        for r, ks in enumerate(allk):
            m = []
            for k in ks:
                ok = k not in seen and k not in newseen
                if ok:
                    newseen[k] = True
                m.append(ok)
            mask_all.append(m)
        seen.update(newseen)
        wm = self._plan.watermark
        if wm and wm[0] in cols and self._batch_wm > 0:
            from .column import ts_to_micros
            j = cols.index(wm[0])
            for k in [k for k in seen if k[j] is not None and ts_to_micros(k[j]) < self._batch_wm * 1000]:
                del seen[k]
        mask = torch.as_tensor(mask_all[comm.rank], dtype=torch.bool, device=df._device)
        return df._mask_rows(mask) if df._nrows else df

    def _advance_watermark(self, df) -> None:
        wm = self._plan.watermark
        if not wm:
            return
        col, delay = wm
        try:
            cd = df._cols[col]
        except KeyError:
            return
        if cd.is_host or len(cd) == 0:
            local = -2**62
        else:
            v = cd.values[cd.valid_mask()] if cd.valid is not None else cd.values
            local = int(v.max().item()) if v.numel() else -2**62
        gmax = int(self._session._comm.max_scalar(float(local)))
        if gmax > -2**61:
            self._watermark_ms = max(self._watermark_ms, gmax // 1000 - parse_interval_ms(delay))

    def _run_batch(self, plan) -> dict:
        with trace("stream.batch"):
            return self._run_batch_impl(plan)

    def _run_batch_impl(self, plan) -> dict:
        bid, files, ts_ms, wm_ms, replay = plan
        if replay:
            self._state = self._load_state()
        maybe_fail("stream.after_offsets", bid)  # crash point: batch planned (offsets logged), nothing written
        t0 = time.time()
        self._watermark_ms = max(self._watermark_ms, wm_ms)
        self._batch_wm = wm_ms
        with trace("stream.read"):
            df = self._read_batch(files, ts_ms)
            nrows = (self._wm_source if self._wm_source is not None else df).count()
        w = self._writer
        complete = w._mode == "complete"
        pending = None
        if self._table is not None:
            from ..io import table as tbl
            root = self._session.catalog._table_path(self._table)
            if tbl.committed_txn(root, self.id) < bid:
                mode = "overwrite" if complete else "append"
                txn = {"appId": self.id, "version": bid}
                # The sink write runs before foreachBatch (parallel part files). CML_SINK_ASYNC=1 overlaps it
                # with foreachBatch instead: the same batch time on the reference workflow, but the writer
                # threads then slowed the user's function 1-5x run to run (profiles/r4/workflow/)
                if os.environ.get("CML_SINK_ASYNC", "0") == "1":
                    pending = tbl.write_frame_async(df, root, mode, operation="STREAMING UPDATE", txn=txn)
                else:
                    with trace("stream.sink_write"):
                        tbl.write_frame(df, root, mode, "STREAMING UPDATE", txn)
        elif self._path is not None or (w._format not in (None, "console", "memory", "delta", "noop")):
            if self._path is None:
                raise ValueError("file sink needs a path")
            fmt = w._format or "parquet"
            if fmt == "delta":
                from ..io import table as tbl
                if tbl.committed_txn(self._path, self.id) < bid:
                    tbl.write_frame(df, self._path, "append", "STREAMING UPDATE", {"appId": self.id, "version": bid})
            else:  # one directory per batch, overwritten on replay: idempotent
                df.write.mode("overwrite").format(fmt).save(os.path.join(self._path, f"batch={bid}"))
        elif w._format == "console" and self._foreach_batch_absent():
            if self._session._comm.is_root:
                print(f"-------------------------------------------\nBatch: {bid}\n"
                      f"-------------------------------------------")
            df.show()
        elif w._format == "memory":
            name = self.name or "memory_sink"
            prev = None if complete else self._session.catalog._views.get(name)
            self._session.catalog._register_view(name, df if prev is None else prev.union(df), True)
        try:
            if w._foreach_batch is not None:
                with trace("stream.foreachBatch"):
                    w._foreach_batch(df, bid)
        finally:
            if pending is not None:
                with trace("stream.sink_commit"):
                    pending.finish()
        self._advance_watermark(self._wm_source if self._wm_source is not None else df)
        comm = self._session._comm
        comm.barrier()
        self._save_state(bid)
        maybe_fail("stream.before_commit", bid)  # crash point: sink done, commit not yet logged
        if comm.is_root:
            self._write_json("commits", bid, {"nextBatchWatermarkMs": self._watermark_ms})
        prog = {"id": self.id, "runId": self.runId, "name": self.name, "batchId": bid, "numInputRows": nrows,
                "numInputFiles": len(files), "timestamp": ts_ms, "replayed": replay,
                "durationMs": {"triggerExecution": int((time.time() - t0) * 1000)},
                "eventTime": {"watermark": self._watermark_ms}, "sink": self._table or self._path}
        with self._lock:
            self.recentProgress.append(prog)
            self.recentProgress = self.recentProgress[-100:]
        return prog

    def _foreach_batch_absent(self) -> bool:
        return self._writer._foreach_batch is None

    def _drain(self) -> int:
        """Run micro-batches until no new data. Returns batches run."""
        n = 0
        while not self._stop.is_set():
            plan = self._plan_next()
            if plan is None:
                break
            self._run_batch(plan)
            n += 1
        return n

    def _launch(self) -> None:
        trig = self._writer._trigger
        comm = self._session._comm
        if trig.get("once"):
            plan = self._plan_next()
            if plan is not None:
                self._run_batch(plan)
            self._stop.set()
        elif trig.get("availableNow"):
            self._drain()
            self._stop.set()
        elif comm.is_distributed:
            # SPMD: batches execute in the caller's thread (processAllAvailable / awaitTermination)
            self._drain()
        else:
            interval = trig.get("processingTime", 0) / 1000.0
            dev = self._session._device

            def loop():
                try:
                    if dev.type == "cuda":
                        import torch
                        torch.cuda.set_device(dev)
                    while not self._stop.is_set():
                        t0 = time.time()
                        self._drain()
                        wait = max(interval - (time.time() - t0), 0.05)
                        self._stop.wait(wait)
                except BaseException as e:  # surfaced by awaitTermination
                    self._error = e
                    log.exception("streaming query failed")
            self._thread = threading.Thread(target=loop, name=f"stream-{self.id[:8]}", daemon=True)
            self._thread.start()

    # ------------------------------------------------------------------ public API
    @property
    def isActive(self) -> bool:
        if self._thread is not None:
            return self._thread.is_alive() and not self._stop.is_set()
        return not self._stop.is_set()

    @property
    def lastProgress(self) -> Optional[dict]:
        with self._lock:
            return self.recentProgress[-1] if self.recentProgress else None

    @property
    def status(self) -> dict:
        return {"message": "Waiting for data to arrive" if self.isActive else "Stopped",
                "isDataAvailable": False, "isTriggerActive": self.isActive}

    def exception(self):
        return self._error

    def processAllAvailable(self) -> None:
        if self._thread is not None:
            # let the background loop see every file currently present
            while True:
                if self._error:
                    raise self._error
                with self._lock:
                    pass
                if self._session._comm.is_root and not self._pending():
                    time.sleep(0.1)
                    if not self._pending():
                        return
                time.sleep(0.05)
        else:
            self._drain()

    def _pending(self) -> bool:
        offs, commits = self._ids("offsets"), self._ids("commits")
        if offs and (not commits or offs[-1] > commits[-1]):
            return True
        return bool(self._list_new(set(self._seen_files())))

    def awaitTermination(self, timeout: Optional[float] = None) -> Optional[bool]:
        if self._thread is None:
            if not self._stop.is_set():
                deadline = None if timeout is None else time.time() + timeout
                while not self._stop.is_set() and (deadline is None or time.time() < deadline):
                    self._drain()
                    if self._stop.wait(0.1):
                        break
            return self._stop.is_set() if timeout is not None else None
        self._thread.join(timeout)
        if self._error:
            raise self._error
        return not self._thread.is_alive() if timeout is not None else None

    def stop(self) -> None:
        self._stop.set()
        if self._thread is not None:
            self._thread.join(timeout=30)
        self._session.streams._unregister(self)

    def explain(self, extended=False):
        print(f"StreamingQuery {self.name or self.id}: {self._plan.fmt} source {self._plan.path} -> "
              f"{self._table or self._path or self._writer._format}")


class StreamingQueryManager:
    def __init__(self, session):
        self._session = session
        self._queries: Dict[str, StreamingQuery] = {}

    def _register(self, q: StreamingQuery) -> None:
        self._queries[q.id] = q

    def _unregister(self, q: StreamingQuery) -> None:
        self._queries.pop(q.id, None)

    @property
    def active(self) -> List[StreamingQuery]:
        return [q for q in self._queries.values() if q.isActive]

    def get(self, qid: str) -> Optional[StreamingQuery]:
        return self._queries.get(qid)

    def awaitAnyTermination(self, timeout: Optional[float] = None):
        qs = list(self._queries.values())
        if not qs:
            return True
        return qs[0].awaitTermination(timeout)

    def resetTerminated(self) -> None:
        return None
