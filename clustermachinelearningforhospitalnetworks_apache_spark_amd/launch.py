"""N0 launcher: one process per GPU on one node (the role ``spark-submit`` + executors play for the
reference, ref.py:55-58; SURVEY.md §1.2 N0, §5.3 failure detection).

    python -m clustermachinelearningforhospitalnetworks_apache_spark_amd.launch --nproc-per-node 8 app.py [args]

* sets the torchrun-style environment per rank (RANK, LOCAL_RANK, WORLD_SIZE, LOCAL_WORLD_SIZE,
  MASTER_ADDR=127.0.0.1, MASTER_PORT) so ``SparkSession.builder.master("mi355x[8]")`` in every rank
  binds rank r to GPU r and joins one RCCL communicator;
* keeps ``HSA_ENABLE_IPC_MODE_LEGACY=0`` (dmabuf IPC, required by RCCL on this platform);
* supervises the ranks: the first rank that exits non-zero (or is killed) brings the job down —
  the survivors get SIGTERM, then SIGKILL after ``--grace`` seconds — so a dead rank never leaves
  its peers blocked in a collective until the watchdog timeout; the job exits with that rank's
  code. ``--max-restarts`` relaunches the whole job after a failure (fits resume from their
  iteration checkpoints, streams from their offset logs).

The launcher itself never touches the GPU (it only starts children), so it is safe to use from a
shell, a scheduler or a notebook.
"""
from __future__ import annotations

import argparse
import os
import signal
import socket
import subprocess
import sys
import time
from typing import List, Optional


def _free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _rank_env(base: dict, rank: int, world: int, port: int) -> dict:
    env = dict(base)
    env.update({"RANK": str(rank), "LOCAL_RANK": str(rank), "WORLD_SIZE": str(world),
                "LOCAL_WORLD_SIZE": str(world), "GROUP_RANK": "0", "MASTER_ADDR": "127.0.0.1",
                "MASTER_PORT": str(port)})
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    return env


def _terminate(procs: List[subprocess.Popen], grace: float) -> None:
    for p in procs:
        if p.poll() is None:
            try:
                os.killpg(p.pid, signal.SIGTERM)
            except (ProcessLookupError, PermissionError):
                pass
    deadline = time.time() + grace
    for p in procs:
        while p.poll() is None and time.time() < deadline:
            time.sleep(0.05)
        if p.poll() is None:
            try:
                os.killpg(p.pid, signal.SIGKILL)
            except (ProcessLookupError, PermissionError):
                pass
            p.wait()


def visible_gpu_count(sysfs: str = "/sys/class/kfd/kfd/topology/nodes") -> int:
    """GPUs this job may use, counted WITHOUT touching the HIP runtime (the launcher forks and execs the
    ranks, and a process that initialised the GPU must not do that): the KFD topology nodes with SIMDs
    (CPU nodes report simd_count 0), narrowed by HIP/ROCR/CUDA_VISIBLE_DEVICES when set."""
    n = 0
    try:
        for node in sorted(os.listdir(sysfs)):
            try:
                with open(os.path.join(sysfs, node, "properties")) as fh:
                    props = dict(line.split()[:2] for line in fh if len(line.split()) >= 2)
            except OSError:
                continue
            if int(props.get("simd_count", "0")) > 0:
                n += 1
    except OSError:
        n = 0
    for var in ("ROCR_VISIBLE_DEVICES", "HIP_VISIBLE_DEVICES", "CUDA_VISIBLE_DEVICES"):
        v = os.environ.get(var)
        if v is not None:
            ids = [t for t in v.split(",") if t.strip() != ""]
            n = min(n, len(ids)) if n else len(ids)
    return n


def run_job(cmd: List[str], nproc: int, grace: float = 10.0, port: Optional[int] = None,
            env: Optional[dict] = None) -> int:
    """Start ``nproc`` ranks of ``cmd`` and supervise them; returns the job's exit code."""
    port = port or _free_port()
    base = dict(os.environ if env is None else env)
    procs = [subprocess.Popen(cmd, env=_rank_env(base, r, nproc, port), start_new_session=True)
             for r in range(nproc)]
    failed = None
    try:
        while True:
            alive = 0
            for r, p in enumerate(procs):
                rc = p.poll()
                if rc is None:
                    alive += 1
                elif rc != 0 and failed is None:
                    failed = (r, rc)
            if failed is not None:
                print(f"[launch] rank {failed[0]} exited with code {failed[1]}; stopping the other ranks",
                      file=sys.stderr, flush=True)
                _terminate(procs, grace)
                return failed[1] if failed[1] > 0 else 128 - failed[1]
            if alive == 0:
                return 0
            time.sleep(0.1)
    except KeyboardInterrupt:
        _terminate(procs, grace)
        return 130


def main(argv: Optional[List[str]] = None) -> int:
    ap = argparse.ArgumentParser(description=__doc__.split("\n\n")[0],
                                 formatter_class=argparse.RawDescriptionHelpFormatter)
    ap.add_argument("--nproc-per-node", "--nproc", type=int, default=None,
                    help="ranks to start (default: number of visible GPUs, 1 without GPUs)")
    ap.add_argument("--max-restarts", type=int, default=0, help="relaunch the whole job after a failure")
    ap.add_argument("--grace", type=float, default=10.0, help="seconds between SIGTERM and SIGKILL")
    ap.add_argument("--master-port", type=int, default=None)
    ap.add_argument("-m", dest="module", default=None, help="run a module instead of a script")
    ap.add_argument("script", nargs="?", help="the application script")
    ap.add_argument("args", nargs=argparse.REMAINDER)
    a = ap.parse_args(argv)
    if a.module is None and a.script is None:
        ap.error("give a script or -m module")
    nproc = a.nproc_per_node
    if nproc is None:
        nproc = max(1, visible_gpu_count())
    cmd = [sys.executable] + (["-m", a.module] if a.module else [a.script]) + \
        ([a.script] if a.module and a.script else []) + list(a.args)
    rc = 1
    for attempt in range(a.max_restarts + 1):
        rc = run_job(cmd, nproc, a.grace, a.master_port)
        if rc == 0:
            break
        if attempt < a.max_restarts:
            print(f"[launch] job failed (code {rc}); restart {attempt + 1}/{a.max_restarts}", file=sys.stderr,
                  flush=True)
    return rc


if __name__ == "__main__":
    sys.exit(main())
