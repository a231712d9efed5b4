"""Two gloo ranks sharing cuda:0 run the seeded first Lloyd step with its full accumulate split in two row chunks
(CML_KMEANS_OVERLAP_ROWS=1): chunk 0's all-reduce is enqueued before chunk 1's accumulate. Under rocprofv3
(kernel + memory-copy + marker traces) the per-process databases show the order on the device.

    rocprofv3 --kernel-trace --memory-copy-trace --marker-trace -d DIR -o %pid% -- python scripts/overlap_timeline.py run
    python scripts/overlap_timeline.py show DIR/*.db

``show`` prints, for every process database, the kernels and copies inside the ``kmeans.seeded`` range in time
order (the gloo all-reduce of a CUDA tensor appears as its device-to-host copy).
"""
import os
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


def _rank(rank, world, port):
    os.environ.update({"RANK": str(rank), "WORLD_SIZE": str(world), "MASTER_ADDR": "127.0.0.1",
                       "MASTER_PORT": str(port), "CML_KMEANS_PRUNE": "1", "CML_KMEANS_OVERLAP_ROWS": "1"})
    import torch
    import torch.distributed as dist
    from clustermachinelearningforhospitalnetworks_apache_spark_amd.models.kmeans import LloydEngine
    from clustermachinelearningforhospitalnetworks_apache_spark_amd.parallel.comm import Communicator
    from clustermachinelearningforhospitalnetworks_apache_spark_amd.utils.trace import trace
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    comm = Communicator(rank, world, torch.device("cuda", 0), "gloo", dist.group.WORLD)
    g = torch.Generator(device="cuda")
    g.manual_seed(11)
    cen = torch.randn(K, D, generator=g, device="cuda") * 3
    g.manual_seed(100 + rank)
    lab = torch.randint(0, K, (N // world,), generator=g, device="cuda")
    x = (cen[lab] + torch.randn(N // world, D, generator=g, device="cuda")).to(torch.bfloat16)
    for it in range(2):  # the second fit is the traced one (kernels loaded, allocator warm)
        eng = LloydEngine(x, D, K, comm, prune=True, use_graph=False)
        init = eng.init_kmeans_parallel(seed=5, as_device=True)
        eng.set_centers(init)
        torch.cuda.synchronize()
        with trace("kmeans.seeded" if it else "warmup.seeded"):
            eng.step()
            torch.cuda.synchronize()
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
        try:
            rng = list(c.execute("select start, end from regions where name = 'kmeans.seeded'"))
        except sqlite3.Error:
            rng = []
        if not rng:
            continue
        lo, hi = rng[0]
        ev = [(s, e, "K", n.split("(")[0][:60]) for n, s, e in
              c.execute("select name, start, end from kernels where start >= ? and start < ?", (lo, hi))]
        try:
            for s, e, kind in c.execute("select start, end, name from memory_copies where start >= ? and start < ?",
                                        (lo, hi)):
                ev.append((s, e, "C", str(kind)))
        except sqlite3.Error as exc:
            print(f"(no memory copies table: {exc})")
        ev.sort()
        print(f"=== {path}: kmeans.seeded {(hi - lo) / 1e6:.3f} ms, {len(ev)} events")
        for s, e, kind, name in ev:
            print(f"{(s - lo) / 1e6:9.3f} ms  {kind}  {(e - s) / 1e3:8.1f} us  {name}")


if __name__ == "__main__":
    if len(sys.argv) > 1 and sys.argv[1] == "show":
        show(sys.argv[2:])
    else:
        run()
