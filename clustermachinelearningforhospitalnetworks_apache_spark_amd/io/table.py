"""Append-only transactional table (the reference's Delta "unbounded table",
ref.py:110-115 / SURVEY.md R11), without Delta Lake.

Layout under the table directory::

    part-<version>-r<rank>-<uuid>.parquet     data files written by each rank
    _txn_log/<version:020d>.json               one JSON commit per version

A commit lists ``add``/``remove`` file actions, the schema, the operation and (for
streaming appends) the ``txnId``/``batchId`` of the query that wrote it.  The
snapshot is the replay of all commits; a streaming sink that re-runs batch N
after a crash finds ``(queryId, N)`` already committed and skips it —
idempotent, exactly-once appends.  Commits are created with O_EXCL so
concurrent writers cannot overwrite a version.
"""
from __future__ import annotations

import json
import os
import time
import uuid
from typing import Dict, List, Optional, Tuple

from ..sql import types as T

LOG_DIR = "_txn_log"


def _log_path(root: str, version: int) -> str:
    return os.path.join(root, LOG_DIR, f"{version:020d}.json")


def versions(root: str) -> List[int]:
    d = os.path.join(root, LOG_DIR)
    if not os.path.isdir(d):
        return []
    out = []
    for f in os.listdir(d):
        if f.endswith(".json") and f[:-5].isdigit():
            out.append(int(f[:-5]))
    return sorted(out)


def exists(root: str) -> bool:
    return bool(versions(root))


def snapshot(root: str, as_of: Optional[int] = None) -> Tuple[List[str], Optional[T.StructType], List[dict]]:
    """(live data files, schema, commits) of the table."""
    files: Dict[str, None] = {}
    schema = None
    commits = []
    for v in versions(root):
        if as_of is not None and v > as_of:
            break
        with open(_log_path(root, v)) as fh:
            c = json.load(fh)
        commits.append(c)
        for r in c.get("remove", []):
            files.pop(r, None)
        for a in c.get("add", []):
            files[a] = None
        if c.get("schema"):
            schema = schema_from_json(c["schema"])
    return [os.path.join(root, f) for f in files], schema, commits


def schema_from_json(js) -> T.StructType:
    if isinstance(js, str):
        js = json.loads(js)
    fields = []
    for f in js["fields"]:
        t = f["type"]
        if isinstance(t, dict):
            dt = T.VectorUDT() if t.get("type") == "udt" else (
                T.ArrayType(T.parse_type(t["elementType"])) if t.get("type") == "array" else T.StringType())
        else:
            dt = T.parse_type({"integer": "int", "long": "bigint"}.get(t, t))
        fields.append(T.StructField(f["name"], dt, f.get("nullable", True)))
    return T.StructType(fields)


def committed_txn(root: str, txn_app: str) -> int:
    """Highest batch id committed by streaming query `txn_app` (-1 if none)."""
    best = -1
    for c in snapshot(root)[2]:
        t = c.get("txn")
        if t and t.get("appId") == txn_app:
            best = max(best, int(t.get("version", -1)))
    return best


def commit(root: str, add: List[str], remove: List[str], schema: T.StructType, operation: str,
           txn: Optional[dict] = None) -> int:
    os.makedirs(os.path.join(root, LOG_DIR), exist_ok=True)
    for attempt in range(1000):
        vs = versions(root)
        v = (vs[-1] + 1) if vs else 0
        body = {"version": v, "timestamp": int(time.time() * 1000), "operation": operation,
                "add": [os.path.basename(a) for a in add], "remove": [os.path.basename(r) for r in remove],
                "schema": schema.jsonValue()}
        if txn:
            body["txn"] = txn
        try:
            fd = os.open(_log_path(root, v), os.O_WRONLY | os.O_CREAT | os.O_EXCL, 0o644)
        except FileExistsError:
            continue
        with os.fdopen(fd, "w") as fh:
            json.dump(body, fh)
        return v
    raise RuntimeError("could not commit to table log")


def new_data_file(root: str, rank: int, part: Optional[int] = None) -> str:
    os.makedirs(root, exist_ok=True)
    tail = "" if part is None else f"-c{part:03d}"
    return os.path.join(root, f"part-{int(time.time() * 1000)}-r{rank}-{uuid.uuid4().hex[:12]}{tail}.parquet")


def _part_rows() -> int:
    return max(1, int(os.environ.get("CML_TABLE_PART_ROWS", 1 << 20)))


def _write_parts(table, root: str, rank: int) -> List[str]:
    """Write one rank's Arrow table as consecutive row slices of ~CML_TABLE_PART_ROWS rows (default
    1 Mi), one Parquet file each, written by parallel threads (Arrow's writer releases the GIL) — a
    Spark task writes one part file per partition the same way. The paths come back in row order, the
    order the commit lists them and a snapshot reads them back."""
    import pyarrow.parquet as pq
    from .csv import cap_arrow_threads, host_threads
    cap_arrow_threads()
    n = table.num_rows
    # the split depends on the row count only (row ids, hence seeded row sampling, follow the files)
    parts = max(1, min(-(-n // _part_rows()), 8))
    if parts == 1:
        path = new_data_file(root, rank)
        pq.write_table(table, path)
        return [path]
    step = -(-n // parts)
    paths = [new_data_file(root, rank, i) for i in range(parts)]
    from concurrent.futures import ThreadPoolExecutor
    with ThreadPoolExecutor(min(parts, host_threads()), thread_name_prefix="cml-part-write") as ex:
        list(ex.map(lambda i: pq.write_table(table.slice(i * step, step), paths[i]), range(parts)))
    return paths


def write_frame(df, root: str, mode: str, operation: str = "WRITE", txn: Optional[dict] = None) -> Optional[int]:
    """All ranks write their shard; rank 0 commits. Returns the version (on every rank)."""
    import pyarrow.parquet as pq
    from .arrow import frame_to_arrow
    comm = df._comm
    if mode in ("error", "errorifexists") and exists(root):
        raise FileExistsError(f"table at {root} already exists (mode=error)")
    if mode == "ignore" and exists(root):
        return None
    mine = _write_parts(frame_to_arrow(df), root, comm.rank) if df._nrows > 0 else []
    added = [p for ps in comm.allgather_object(mine) for p in ps]
    version = None
    if comm.is_root:
        removed = snapshot(root)[0] if mode == "overwrite" else []
        version = commit(root, added, removed, df.schema, operation, txn)
    return comm.broadcast_object(version)


class PendingWrite:
    """A table append whose Parquet file is being written by a background thread (Arrow's writer
    releases the GIL), so the caller can run other work — the streaming query runs the user's
    foreachBatch function — before ``finish()`` joins it and commits (collectives happen in
    ``finish``, at the same point on every rank)."""

    def __init__(self, df, root: str, mode: str, operation: str, txn: Optional[dict]):
        import threading

        from .arrow import frame_to_arrow
        self.df, self.root, self.mode, self.operation, self.txn = df, root, mode, operation, txn
        self.paths: List[str] = []
        self.error: Optional[BaseException] = None
        self.thread = None
        if df._nrows > 0:
            table = frame_to_arrow(df)  # device -> host on the calling thread

            def run():
                try:
                    self.paths = _write_parts(table, root, df._comm.rank)
                except BaseException as e:  # noqa: BLE001 — re-raised in finish()
                    self.error = e
            self.thread = threading.Thread(target=run, name="cml-table-write", daemon=True)
            self.thread.start()

    def finish(self) -> Optional[int]:
        if self.thread is not None:
            self.thread.join()
        comm = self.df._comm
        failed = comm.allgather_object(self.error is not None)
        if any(failed):
            raise self.error if self.error is not None else RuntimeError("table write failed on another rank")
        added = [p for ps in comm.allgather_object(self.paths) for p in ps]
        version = None
        if comm.is_root:
            removed = snapshot(self.root)[0] if self.mode == "overwrite" else []
            version = commit(self.root, added, removed, self.df.schema, self.operation, self.txn)
        return comm.broadcast_object(version)


def write_frame_async(df, root: str, mode: str, operation: str = "WRITE",
                      txn: Optional[dict] = None) -> PendingWrite:
    """Append / overwrite like ``write_frame`` with the file write overlapped (``.finish()``)."""
    if mode not in ("append", "overwrite"):
        raise ValueError("write_frame_async supports append / overwrite")
    return PendingWrite(df, root, mode, operation, txn)


def read_table(session, root: str, version: Optional[int] = None):
    from .arrow import read_parquet_files
    files, schema, _ = snapshot(root, version)
    if schema is None:
        raise FileNotFoundError(f"no table at {root}")
    ids = list(range(len(files)))
    return read_parquet_files(session, files, schema, file_ids=ids)


def history(root: str) -> List[dict]:
    return [{"version": c["version"], "timestamp": c["timestamp"], "operation": c["operation"],
             "numFiles": len(c.get("add", []))} for c in snapshot(root)[2]]
