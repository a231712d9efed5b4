"""Session / launcher (N0 in SURVEY.md §1.2) — replaces SparkSession + the standalone
cluster of the reference (ref.py:55-58, ref.py:258).

``SparkSession.builder.appName(..).master(url).getOrCreate()`` where ``url`` is

* ``"mi355x"``, ``"mi355x[N]"``, ``"gpu[N]"``: one process per MI355X. Under
  ``torchrun`` (RANK/WORLD_SIZE in the environment) every rank binds GPU
  LOCAL_RANK and joins an RCCL communicator over xGMI; without it a single
  process uses GPU 0.
* ``"local"``, ``"local[n]"``, ``"local[*]"``: CPU execution in this process with
  n intra-op threads (the plumbing / test mode); under torchrun the ranks talk
  over gloo.
* ``"spark://host:port"`` (what the reference passes, ref.py:47) or
  ``"auto"``: GPU mode when a GPU is visible, otherwise local.
"""
from __future__ import annotations

import logging
import os
import re
import threading
import time
from typing import Any, Dict, List, Optional, Sequence

import numpy as np
import torch

from ..parallel.comm import Communicator
from . import types as T
from .builder import frame_from_pycolumns, shard_range
from .catalog import Catalog

log = logging.getLogger("cml")


class RuntimeConfig:
    def __init__(self, init: Optional[Dict[str, str]] = None):
        self._c: Dict[str, str] = dict(init or {})

    def set(self, key: str, value) -> None:
        self._c[key] = str(value) if not isinstance(value, str) else value

    def get(self, key: str, default=None):
        return self._c.get(key, default)

    def unset(self, key: str) -> None:
        self._c.pop(key, None)

    def getAll(self) -> Dict[str, str]:
        return dict(self._c)

    def isModifiable(self, key: str) -> bool:
        return True


def parse_master(master: str):
    m = (master or "auto").strip().lower()
    if m.startswith("spark://") or m.startswith("yarn") or m.startswith("k8s") or m == "auto":
        return ("gpu" if torch.cuda.is_available() else "local"), None
    mm = re.fullmatch(r"(local|mi355x|gpu|cpu)(?:\[(\*|\d+)(?:,\s*\d+)?\])?", m)
    if not mm:
        raise ValueError(f"unsupported master URL {master!r}")
    kind, n = mm.group(1), mm.group(2)
    kind = {"mi355x": "gpu", "cpu": "local"}.get(kind, kind)
    return kind, (None if n in (None, "*") else int(n))


class SparkSession:
    _active: Optional["SparkSession"] = None
    _lock = threading.Lock()

    class Builder:
        def __init__(self):
            self._opts: Dict[str, str] = {}

        def appName(self, name: str) -> "SparkSession.Builder":
            self._opts["spark.app.name"] = name
            return self

        def master(self, master: str) -> "SparkSession.Builder":
            self._opts["spark.master"] = master
            return self

        def config(self, key=None, value=None, conf=None, map=None) -> "SparkSession.Builder":
            if map:
                self._opts.update({k: str(v) for k, v in map.items()})
            if key is not None:
                self._opts[key] = str(value)
            return self

        def enableHiveSupport(self) -> "SparkSession.Builder":
            return self

        def getOrCreate(self) -> "SparkSession":
            with SparkSession._lock:
                if SparkSession._active is not None and not SparkSession._active._stopped:
                    for k, v in self._opts.items():
                        SparkSession._active.conf.set(k, v)
                    return SparkSession._active
                s = SparkSession(self._opts)
                SparkSession._active = s
                return s

        create = getOrCreate

    builder = Builder()

    def __init__(self, opts: Optional[Dict[str, str]] = None):
        SparkSession.builder = SparkSession.Builder()
        opts = dict(opts or {})
        self.conf = RuntimeConfig(opts)
        master = opts.get("spark.master", os.environ.get("CML_MASTER", "auto"))
        kind, n = parse_master(master)
        self._kind = kind
        if kind == "gpu" and n is not None:
            # mi355x[N] names the cluster the way the reference's .master(...) does (ref.py:55-58): N
            # ranks, one per GPU. A session must not silently run with another world size.
            world = int(os.environ.get("WORLD_SIZE", "1"))
            if world != n:
                raise ValueError(
                    f"master {master!r} asks for {n} GPU ranks but this process is rank "
                    f"{os.environ.get('RANK', '0')} of WORLD_SIZE={world}. Start one process per GPU with "
                    f"`python -m clustermachinelearningforhospitalnetworks_apache_spark_amd.launch "
                    f"--nproc-per-node {n} your_app.py` (or torchrun --nproc-per-node {n}), or use "
                    f"master('mi355x') to take the world size from the launcher.")
        if kind == "local" and n:
            torch.set_num_threads(max(1, n))
        # collective watchdog: a rank that stops participating fails the job after the timeout
        # instead of hanging it; RCCL errors surface asynchronously as exceptions
        os.environ.setdefault("TORCH_NCCL_ASYNC_ERROR_HANDLING", "1")
        self._comm = Communicator.from_env(want_gpu=(kind == "gpu"),
                                           timeout_s=float(opts.get("cml.comm.timeoutSeconds", 600)))
        if kind == "gpu" and not self._comm.device.type == "cuda":
            log.warning("master=%s requested GPUs but none is visible; running on CPU", opts.get("spark.master"))
        self._device = self._comm.device
        self._warmup_s = 0.0
        if self._device.type == "cuda" and str(opts.get("cml.session.warmup", os.environ.get("CML_SESSION_WARMUP", "true"))).lower() not in ("0", "false"):
            from ..utils.warmup import warm_device
            try:
                self._warmup_s = warm_device(self._device, int(float(opts.get("cml.session.poolBytes", 1 << 30))))
            except Exception as e:  # a warm-up is an optimisation: never fail a session on it
                log.warning("device warm-up skipped: %s", e)
        self._stopped = False
        self.catalog = Catalog(self)
        from .functions import UDFRegistration
        self.udf = UDFRegistration()
        if self._warmup_s > 0.0:  # the device warm-up ran: the frame path's kernels too
            from ..utils.warmup import warm_frames
            try:
                self._warmup_s += warm_frames(self)
            except Exception as e:
                log.warning("frame warm-up skipped: %s", e)
        self._streams = None
        self._start_time = time.time()
        self.sparkContext = _Context(self)
        if self._comm.is_root:
            log.info("session %s on %s (%d rank(s))", self.conf.get("spark.app.name"), self._device,
                     self._comm.world_size)

    # ------------------------------------------------------------------ properties
    @property
    def version(self) -> str:
        from .. import __version__
        return __version__

    @property
    def device(self) -> torch.device:
        return self._device

    @property
    def rank(self) -> int:
        return self._comm.rank

    @property
    def world_size(self) -> int:
        return self._comm.world_size

    @classmethod
    def getActiveSession(cls) -> Optional["SparkSession"]:
        return cls._active

    active = getActiveSession

    def newSession(self) -> "SparkSession":
        return self

    # ------------------------------------------------------------------ data sources
    @property
    def read(self):
        from ..io.reader import DataFrameReader
        return DataFrameReader(self)

    @property
    def readStream(self):
        from .streaming import DataStreamReader
        return DataStreamReader(self)

    @property
    def streams(self):
        from .streaming import StreamingQueryManager
        if self._streams is None:
            self._streams = StreamingQueryManager(self)
        return self._streams

    def createDataFrameFromTensors(self, columns: Dict[str, torch.Tensor]):
        """cml extension: a frame over THIS rank's shard of device-resident tensors, without a host
        round trip ([n, d] tensors become vector columns, [n] tensors numeric columns). Rows are
        numbered globally in rank order (rank r's rows follow ranks < r), which keeps every
        counter-based random decision independent of the GPU count."""
        from .column import ColumnData
        from .dataframe import DataFrame
        if not columns:
            raise ValueError("createDataFrameFromTensors needs at least one column")
        n = int(next(iter(columns.values())).shape[0])
        fields, cols = [], {}
        kinds = {torch.float64: T.DoubleType(), torch.float32: T.FloatType(), torch.int32: T.IntegerType(),
                 torch.int64: T.LongType(), torch.bool: T.BooleanType(), torch.int16: T.ShortType()}
        from ..utils.hoststream import hbm_budget_bytes, pinned_rows
        budget = hbm_budget_bytes(self._device, self.conf.get("cml.hbm.budgetBytes", None))
        for name, t in columns.items():
            if int(t.shape[0]) != n:
                raise ValueError("all columns need the same number of rows")
            if (t.dim() == 2 and not t.is_cuda and self._device.type == "cuda"
                    and t.numel() * t.element_size() > budget):
                # out of core: a vector column larger than cml.hbm.budgetBytes stays in host
                # memory; KMeans streams it through the GPU chunk by chunk (utils/hoststream.py). bf16 / fp8
                # rows are pinned here; other dtypes get their pinned bf16 copy on first use (one copy,
                # cached on the column: models/kmeans.py host_layout) — pinning the f32 source too would
                # hold twice the page-locked memory
                if t.dtype in (torch.bfloat16, torch.float8_e4m3fn):
                    t = pinned_rows(t)
            else:
                t = t.to(self._device)
            if t.dim() == 2:
                dt = T.VectorUDT()
            elif t.dtype in kinds:
                dt = kinds[t.dtype]
            else:
                raise TypeError(f"column {name!r}: unsupported scalar dtype {t.dtype}")
            fields.append(T.StructField(name, dt, True))
            cols[name] = ColumnData(t, None, dt)
        counts = self._comm.allgather_object(n)
        off = sum(counts[: self._comm.rank])
        rows = torch.arange(off, off + n, dtype=torch.int64, device=self._device)
        return DataFrame(self, T.StructType(fields), cols, n, rows, self._device)

    def createDataFrame(self, data, schema=None, samplingRatio=None, verifySchema=True):
        """Rows / tuples / dicts / pandas / numpy -> sharded frame.

        SPMD contract: every rank passes the same data; rank r keeps its contiguous
        block of rows, with global row ids = input positions.
        """
        import pandas as pd
        if isinstance(schema, str):
            schema = T.parse_ddl_schema(schema)
        names: Optional[List[str]] = None
        if isinstance(schema, (list, tuple)):
            names, schema = list(schema), None
        if isinstance(data, pd.DataFrame):
            names = names or [str(c) for c in data.columns]
            cols = {n: data[c].tolist() if data[c].dtype == object else data[c].to_numpy()
                    for n, c in zip(names, data.columns)}
            if schema is None:
                schema = T.StructType([T.StructField(n, _infer_pandas(data[c])) for n, c in zip(names, data.columns)])
            nrows = len(data)
        elif isinstance(data, np.ndarray):
            if data.ndim == 1:
                data = data[:, None]
            names = names or [f"_{i + 1}" for i in range(data.shape[1])]
            cols = {n: data[:, i] for i, n in enumerate(names)}
            if schema is None:
                schema = T.StructType([T.StructField(n, T.infer_type(cols[n])) for n in names])
            nrows = data.shape[0]
        else:
            rows = list(data)
            nrows = len(rows)
            if schema is not None:
                names = schema.names
            if rows and isinstance(rows[0], dict):
                names = names or list(rows[0].keys())
                cols = {n: [r.get(n) for r in rows] for n in names}
            elif rows and isinstance(rows[0], T.Row) and rows[0].__fields__:
                names = names or list(rows[0].__fields__)
                cols = {n: [r[i] for r in rows] for i, n in enumerate(names)}
            else:
                width = len(rows[0]) if rows else len(names or [])
                names = names or [f"_{i + 1}" for i in range(width)]
                cols = {n: [r[i] for r in rows] for i, n in enumerate(names)}
            if schema is None:
                schema = T.StructType([T.StructField(n, T.infer_type(np.asarray(cols[n], dtype=object)))
                                       for n in names])
        if schema is not None and names is not None and schema.names != names:
            schema = T.StructType([T.StructField(n, f.dataType, f.nullable) for n, f in zip(names, schema.fields)])
        a, b = shard_range(nrows, self._comm.rank, self._comm.world_size)
        local = {f.name: cols[f.name][a:b] for f in schema.fields}
        return frame_from_pycolumns(self, schema, local, list(range(a, b)))

    def range(self, start: int, end: Optional[int] = None, step: int = 1, numPartitions=None):
        if end is None:
            start, end = 0, start
        n = max(0, (end - start + step - 1) // step) if step > 0 else 0
        a, b = shard_range(n, self._comm.rank, self._comm.world_size)
        vals = torch.arange(start + a * step, start + b * step, step, dtype=torch.int64, device=self._device)
        from .column import ColumnData
        from .dataframe import DataFrame
        schema = T.StructType([T.StructField("id", T.LongType(), False)])
        return DataFrame(self, schema, {"id": ColumnData(vals, None, T.LongType())}, b - a,
                         torch.arange(a, b, dtype=torch.int64, device=self._device), self._device)

    def _empty_frame(self, schema: T.StructType):
        return frame_from_pycolumns(self, schema, {f.name: [] for f in schema.fields}, [])

    def table(self, name: str):
        return self.catalog._resolve(name)

    def sql(self, sqlQuery: str, args=None, **kwargs):
        from .sqlparse import execute
        if args:
            sqlQuery = sqlQuery.format(**args) if isinstance(args, dict) else sqlQuery
        return execute(self, sqlQuery)

    def stop(self) -> None:
        """Stop streams, drain the device, tear down RCCL (ref.py:258)."""
        if self._stopped:
            return
        if self._streams is not None:
            for q in list(self._streams.active):
                q.stop()
        if self._device.type == "cuda":
            torch.cuda.synchronize(self._device)
        self._comm.shutdown()
        self._stopped = True
        if SparkSession._active is self:
            SparkSession._active = None

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.stop()


class _Context:
    """Minimal SparkContext facade."""

    def __init__(self, session: SparkSession):
        self._s = session

    @property
    def appName(self) -> str:
        return self._s.conf.get("spark.app.name", "")

    @property
    def master(self) -> str:
        return self._s.conf.get("spark.master", "auto")

    @property
    def defaultParallelism(self) -> int:
        return self._s.world_size

    def setLogLevel(self, level: str) -> None:
        logging.getLogger("cml").setLevel(level.upper())

    def stop(self) -> None:
        self._s.stop()


def _infer_pandas(series) -> T.DataType:
    k = series.dtype.kind
    if k == "M":
        return T.TimestampType()
    if k == "b":
        return T.BooleanType()
    if k in "iu":
        return T.LongType() if series.dtype.itemsize >= 8 else T.IntegerType()
    if k == "f":
        return T.DoubleType() if series.dtype.itemsize >= 8 else T.FloatType()
    return T.infer_type(np.asarray(series.tolist(), dtype=object))


Session = SparkSession
