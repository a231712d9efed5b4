"""Two gloo ranks sharing cuda:0 run the seeded first Lloyd step with its full accumulate split in two row chunks
(CML_KMEANS_OVERLAP_ROWS=1): chunk 0's all-reduce is enqueued before chunk 1's accumulate. Under rocprofv3
(kernel + memory-copy + marker traces) the per-process databases show the order on the device.

    python scripts/overlap_timeline.py run                       (both ranks from one process)
    rocprofv3 --kernel-trace --memory-copy-trace -d DIR0 -o r0 -- \
        python3 scripts/overlap_timeline.py rank 0 2 PORT &       (one profiled process per rank; same for rank 1)
    python scripts/overlap_timeline.py show DIR0/*.db

A fifth argument ``full`` traces a pruned step on overlapping blobs instead: the split full-pass step, whose
chunk 0 all-reduce (the device-to-host copy of gloo) must start before chunk 1's K9r pass ends.

``show`` prints, for every process database, the kernels and copies between the two probe-kernel dispatches that
bracket the traced seeded step, in time order (the gloo all-reduce of a CUDA tensor appears as its
device-to-host copy).
"""
import os
import re
import socket
import sqlite3
import sys

N, D, K = 4_000_000, 256, 64


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _rank(rank, world, port, what="seeded"):
    os.environ.update({"RANK": str(rank), "WORLD_SIZE": str(world), "MASTER_ADDR": "127.0.0.1",
                       "MASTER_PORT": str(port), "CML_KMEANS_PRUNE": "1", "CML_KMEANS_OVERLAP_ROWS": "1",
                       "CML_KMEANS_SPLIT_FULL": "1"})
    import torch
    import torch.distributed as dist
    from clustermachinelearningforhospitalnetworks_apache_spark_amd.models.kmeans import LloydEngine
    from clustermachinelearningforhospitalnetworks_apache_spark_amd.parallel.comm import Communicator
    from clustermachinelearningforhospitalnetworks_apache_spark_amd.ops import kmeans_ops as KO
    from clustermachinelearningforhospitalnetworks_apache_spark_amd.utils.trace import trace
    torch.cuda.set_device(0)
    pa = torch.zeros((16, 128), dtype=torch.uint8, device="cuda")
    ps = torch.full((64,), 127, dtype=torch.int32, device="cuda")
    dist.init_process_group("gloo", rank=rank, world_size=world)
    comm = Communicator(rank, world, torch.device("cuda", 0), "gloo", dist.group.WORLD)
    g = torch.Generator(device="cuda")
    g.manual_seed(11)
    # "full": overlapping blobs — the bounds prune little, so the pruned steps run the split full pass (chunk 0's
    # all-reduce in flight during chunk 1's K9r pass, models/kmeans.py _pdev_pre_split)
    cen = torch.randn(K, D, generator=g, device="cuda") * (0.5 if what == "full" else 3)
    g.manual_seed(100 + rank)
    lab = torch.randint(0, K, (N // world,), generator=g, device="cuda")
    x = (cen[lab] + torch.randn(N // world, D, generator=g, device="cuda")).to(torch.bfloat16)
    for it in range(2):  # the second fit is the traced one (kernels loaded, allocator warm)
        eng = LloydEngine(x, D, K, comm, prune=True, use_graph=False)
        init = eng.init_kmeans_parallel(seed=5, as_device=True)
        eng.set_centers(init)
        torch.cuda.synchronize()
        if what == "full":  # past the seeded step, into the steps whose gate picks full passes
            eng.fit(4, 0.0)
            torch.cuda.synchronize()
        if it:  # the traced step, bracketed by two dispatches of a one-wave probe kernel (window markers)
            KO.mx_probe(pa, pa, ps, ps)
        with trace(f"kmeans.{what}" if it else f"warmup.{what}"):
            eng.step()
            if it:
                KO.mx_probe(pa, pa, ps, ps)
            torch.cuda.synchronize()
        if what == "full" and it:
            print(f"rank {rank}: split steps {getattr(eng._pst, 'split_steps', 0)}", flush=True)
        eng.fit(3, 0.0)
        torch.cuda.synchronize()
    dist.barrier()
    dist.destroy_process_group()


def run():
    import torch.multiprocessing as mp
    port = _free_port()
    ctx = mp.get_context("spawn")
    procs = [ctx.Process(target=_rank, args=(r, 2, port)) for r in range(2)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(300)
    sys.exit(0 if all(p.exitcode == 0 for p in procs) else 1)


def show(paths):
    for path in paths:
        c = sqlite3.connect(path)
        kcols = [r[1] for r in c.execute("pragma table_info(kernels)")]
        sid = next((x for x in ("stream_id", "queue_id") if x in kcols), None)
        ks = list(c.execute(f"select name, start, end, {sid or 0} from kernels order by start"))
        marks = [(s, e) for n, s, e, _ in ks if "mx_probe_kernel" in n]
        if len(marks) < 2:
            print(f"{path}: no probe-kernel window ({len(marks)} markers)")
            continue
        lo, hi = marks[0][1], marks[1][0]
        def short(n):
            n = re.sub(r"\(anonymous namespace\)::", "", n)
            n = re.sub(r"^void ", "", n)
            return n.split("(")[0][:70]
        ev = [(s, e, f"K q{q}", short(n)) for n, s, e, q in ks if lo <= s < hi]
        try:
            cols = [r[1] for r in c.execute("pragma table_info(memory_copies)")]
            for row in c.execute("select * from memory_copies where start >= ? and start < ?", (lo, hi)):
                r = dict(zip(cols, row))
                what = "/".join(str(r[k]) for k in ("name", "size") if k in r)
                q = r.get("stream_id", r.get("queue_id", ""))
                ev.append((r["start"], r["end"], f"C q{q}", what))
        except sqlite3.Error as exc:
            print(f"(memory copies: {exc})")
        ev.sort()
        print(f"=== {path}: traced step window {(hi - lo) / 1e6:.3f} ms, {len(ev)} events")
        for s, e, kind, name in ev:
            print(f"{(s - lo) / 1e6:9.3f} ms  {kind:6s} {(e - s) / 1e3:8.1f} us  {name}")


if __name__ == "__main__":
    if len(sys.argv) > 1 and sys.argv[1] == "show":
        show(sys.argv[2:])
    elif len(sys.argv) > 1 and sys.argv[1] == "rank":
        _rank(int(sys.argv[2]), int(sys.argv[3]), int(sys.argv[4]), sys.argv[5] if len(sys.argv) > 5 else "seeded")
    else:
        run()
