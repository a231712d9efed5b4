"""N2 communication layer: one process per GPU, RCCL over xGMI (``backend="nccl"`` is
RCCL on ROCm), gloo on CPU for ``local``/multi-process tests.

Replaces every implicit Spark aggregation path of the reference:
treeAggregate of the LinearRegression normal equations (ref.py:147), tree
histograms (ref.py:152-189), evaluator sums (ref.py:163-195), collect-to-driver
(ref.py:204) and the streaming driver's file-list decisions (ref.py:75-115).

Design notes (MI355X-first):
  * messages here are small (≤ 2 MiB) so collectives are
    latency-bound; the lever is overlap, not bandwidth.  ``allreduce_async``
    enqueues an RCCL all-reduce that runs on the process group's internal
    stream, ordered after the work already queued on the caller's stream, and
    returns a handle; ``wait`` makes the *current* stream depend on it.  The
    compute stream never blocks on the host.
  * every collective is also implemented for ``world_size == 1`` as a no-op so
    single-GPU runs pay nothing.
"""
from __future__ import annotations

import datetime
import os
from typing import Any, List, Optional

import torch
import torch.distributed as dist


class Handle:
    """Completion handle for an asynchronous collective."""

    def __init__(self, work=None, tensor=None):
        self._work = work
        self.tensor = tensor

    def wait(self):
        if self._work is not None:
            self._work.wait()
            self._work = None
        return self.tensor


class Communicator:
    """SPMD communicator bound to one rank and one device."""

    def __init__(self, rank: int = 0, world_size: int = 1, device: Optional[torch.device] = None,
                 backend: Optional[str] = None, group=None, owns_group: bool = False):
        self.rank = rank
        self.world_size = world_size
        self.device = device or torch.device("cpu")
        self.backend = backend
        self.group = group
        self._owns = owns_group
        self._cpu_group = None

    # ------------------------------------------------------------------ construction
    @classmethod
    def from_env(cls, want_gpu: bool, timeout_s: float = 600.0) -> "Communicator":
        """Build from torchrun-style env (RANK/WORLD_SIZE/LOCAL_RANK/MASTER_*)."""
        world = int(os.environ.get("WORLD_SIZE", "1"))
        rank = int(os.environ.get("RANK", "0"))
        local_rank = int(os.environ.get("LOCAL_RANK", str(rank)))
        use_gpu = want_gpu and torch.cuda.is_available()
        if use_gpu:
            ndev = torch.cuda.device_count()
            dev_index = local_rank % max(ndev, 1)
            torch.cuda.set_device(dev_index)
            device = torch.device("cuda", dev_index)
        else:
            device = torch.device("cpu")
        # CML_COMM_SELF=1: a one-rank RCCL (or gloo) process group whose collectives really run, so the
        # multi-rank code paths (split step graphs around the all-reduce, chunk-overlapped all-reduces,
        # object broadcasts) execute — and show up in a rocprofv3 trace — on a single GPU
        self_group = world == 1 and os.environ.get("CML_COMM_SELF") == "1"
        if world == 1 and not self_group:
            return cls(0, 1, device, None)
        # CML_COMM_BACKEND=gloo keeps GPU-resident shards but runs the collectives over gloo: several
        # ranks can then share one device (tests on a 1-GPU box; RCCL needs a device per rank)
        backend = os.environ.get("CML_COMM_BACKEND") or ("nccl" if use_gpu else "gloo")
        owns = False
        if not dist.is_initialized():
            os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
            os.environ.setdefault("MASTER_PORT", "29517")
            kwargs = dict(backend=backend, rank=rank, world_size=world,
                          timeout=datetime.timedelta(seconds=timeout_s))
            if use_gpu and backend == "nccl":
                kwargs["device_id"] = device
            dist.init_process_group(**kwargs)
            owns = True
        c = cls(rank, world, device, dist.get_backend(), dist.group.WORLD, owns)
        c._self_group = self_group
        if c.backend != "gloo":
            # the gloo side group of the host-side control messages, created HERE, where every rank passes in the
            # same order: dist.new_group is itself a collective, so creating it lazily at the first object
            # collective deadlocked whenever that first use was rank-conditional
            c._cpu_group = dist.new_group(backend="gloo")
        return c

    _self_group = False

    @property
    def is_distributed(self) -> bool:
        return self.world_size > 1 or self._self_group

    @property
    def is_root(self) -> bool:
        return self.rank == 0

    def cpu_group(self):
        """A gloo group for host-side control messages (objects, file lists)."""
        if not self.is_distributed:
            return None
        if self.backend == "gloo":
            return self.group
        if self._cpu_group is None:
            # (a communicator built around an existing RCCL group rather than by from_env: every rank must reach
            # this first object collective together)
            self._cpu_group = dist.new_group(backend="gloo")
        return self._cpu_group

    # ------------------------------------------------------------------ tensor collectives
    def _coerce(self, t: torch.Tensor) -> torch.Tensor:
        if self.backend == "nccl" and not t.is_cuda:
            raise ValueError("RCCL collectives need device tensors")
        return t

    def allreduce_(self, t: torch.Tensor, op: str = "sum") -> torch.Tensor:
        if self.is_distributed:
            dist.all_reduce(self._coerce(t), op=_op(op), group=self.group)
        return t

    def allreduce_async(self, t: torch.Tensor, op: str = "sum") -> Handle:
        """Enqueue an all-reduce ordered after the current stream's pending work."""
        if not self.is_distributed:
            return Handle(None, t)
        work = dist.all_reduce(self._coerce(t), op=_op(op), group=self.group, async_op=True)
        return Handle(work, t)

    def broadcast_(self, t: torch.Tensor, src: int = 0) -> torch.Tensor:
        if self.is_distributed:
            dist.broadcast(self._coerce(t), src=src, group=self.group)
        return t

    def allgather(self, t: torch.Tensor) -> List[torch.Tensor]:
        """All-gather tensors whose first dimension may differ per rank."""
        if not self.is_distributed:
            return [t]
        n = torch.tensor([t.shape[0]], dtype=torch.int64, device=t.device)
        ns = [torch.zeros_like(n) for _ in range(self.world_size)]
        dist.all_gather(ns, n, group=self.group)
        sizes = [int(x.item()) for x in ns]
        m = max(sizes)
        pad = torch.zeros((m,) + tuple(t.shape[1:]), dtype=t.dtype, device=t.device)
        pad[: t.shape[0]] = t
        outs = [torch.empty_like(pad) for _ in range(self.world_size)]
        dist.all_gather(outs, pad, group=self.group)
        return [o[:s] for o, s in zip(outs, sizes)]

    def allgather_fixed(self, t: torch.Tensor) -> torch.Tensor:
        """[world, *t.shape]: every rank's same-shape tensor, in rank order, with no size exchange and no
        host read (one all_gather_into_tensor on the device stream)."""
        if not self.is_distributed:
            return t.reshape((1,) + tuple(t.shape))
        src = t.contiguous()
        # a flat [world · numel] output: the layout every backend accepts (gloo rejects a stacked one)
        out = torch.empty(self.world_size * src.numel(), dtype=src.dtype, device=src.device)
        dist.all_gather_into_tensor(self._coerce(out), src.reshape(-1), group=self.group)
        return out.view((self.world_size,) + tuple(src.shape))

    def allgather_sized(self, t: torch.Tensor, sizes: List[int]) -> torch.Tensor:
        """Concatenation in rank order of every rank's ``t`` whose row counts ``sizes`` every rank already
        knows (one padded all_gather, no size exchange)."""
        if not self.is_distributed:
            return t
        m = max(max(sizes), 1)
        pad = torch.zeros((m,) + tuple(t.shape[1:]), dtype=t.dtype, device=t.device)
        pad[: t.shape[0]] = t
        g = self.allgather_fixed(pad)
        return torch.cat([g[r, : sizes[r]] for r in range(self.world_size)], 0)

    def allgather_cat(self, t: torch.Tensor) -> torch.Tensor:
        parts = self.allgather(t)
        return parts[0] if len(parts) == 1 else torch.cat(parts, 0)

    def alltoallv(self, t: torch.Tensor, send_counts: List[int]) -> torch.Tensor:
        """Variable all-to-all along dim 0: rows ``t[sum(send_counts[:r]) : ... + send_counts[r]]`` go
        to rank r; the result is what every rank sent here, in source-rank order (one
        ``all_to_all_single`` for the counts, one for the payload — the shuffle of sort / repartition)."""
        if not self.is_distributed:
            return t
        sc = torch.tensor([int(c) for c in send_counts], dtype=torch.int64, device=t.device)
        rc = torch.empty_like(sc)
        dist.all_to_all_single(self._coerce(rc), sc, group=self.group)
        recv = [int(x) for x in rc.tolist()]
        src = t.contiguous()
        is_bool = src.dtype == torch.bool
        if is_bool:
            src = src.view(torch.uint8)
        out = torch.empty((sum(recv),) + tuple(src.shape[1:]), dtype=src.dtype, device=src.device)
        dist.all_to_all_single(self._coerce(out), src, recv, [int(c) for c in send_counts], group=self.group)
        return out.view(torch.bool) if is_bool else out

    def sum_scalar(self, v: float, dtype=torch.float64) -> float:
        if not self.is_distributed:
            return v
        t = torch.tensor([v], dtype=dtype, device=self.device)
        self.allreduce_(t)
        return t.item()

    def max_scalar(self, v: float) -> float:
        if not self.is_distributed:
            return v
        t = torch.tensor([v], dtype=torch.float64, device=self.device)
        self.allreduce_(t, "max")
        return t.item()

    # ------------------------------------------------------------------ object collectives (host)
    def allgather_object(self, obj: Any) -> List[Any]:
        if not self.is_distributed:
            return [obj]
        out = [None] * self.world_size
        dist.all_gather_object(out, obj, group=self.cpu_group())
        return out

    def broadcast_object(self, obj: Any, src: int = 0) -> Any:
        if not self.is_distributed:
            return obj
        box = [obj]
        dist.broadcast_object_list(box, src=src, group=self.cpu_group())
        return box[0]

    def barrier(self) -> None:
        if self.is_distributed:
            if self.backend == "nccl":
                dist.barrier(group=self.group, device_ids=[self.device.index])
            else:
                dist.barrier(group=self.group)

    def shutdown(self) -> None:
        if self._owns and dist.is_initialized():
            try:
                # every rank reaches the teardown before any destroys its group: a rank that tore its
                # gloo transport down while a peer still had traffic in flight aborted under load
                # (std::terminate from a joinable transport thread)
                dist.barrier()
            except Exception:  # pragma: no cover - teardown best effort
                pass
            try:
                dist.destroy_process_group()
            except Exception:  # pragma: no cover - teardown best effort
                pass
            self._owns = False


def _op(name: str):
    return {"sum": dist.ReduceOp.SUM, "max": dist.ReduceOp.MAX, "min": dist.ReduceOp.MIN}[name]


_LOCAL = Communicator()


def local_comm() -> Communicator:
    return _LOCAL
