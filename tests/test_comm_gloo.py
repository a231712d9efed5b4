"""Communicator collectives over gloo with three CPU ranks: the fixed-size all-gather the device
k-means|| init uses (one collective, no size exchange, flat layout every backend accepts) and the
sized all-gather of per-rank row blocks whose counts every rank knows."""
import os
import socket

import torch
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _main(rank, world, port, out):
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from clustermachinelearningforhospitalnetworks_apache_spark_amd.parallel.comm import Communicator
    c = Communicator(rank, world, torch.device("cpu"), "gloo", dist.group.WORLD)
    g = c.allgather_fixed(torch.tensor([[rank, 10.0 + rank]], dtype=torch.float64))
    ok = g.shape == (world, 1, 2) and all(float(g[r, 0, 1]) == 10.0 + r for r in range(world))
    sizes = [0, 2, 5][:world]
    s = c.allgather_sized(torch.full((sizes[rank], 3), float(rank)), sizes)
    ok = ok and s.shape == (sum(sizes), 3) and torch.equal(
        s[:, 0], torch.cat([torch.full((sizes[r],), float(r)) for r in range(world)]))
    with open(f"{out}.{rank}", "w") as fh:
        fh.write("ok" if ok else f"bad {g} {s}")
    dist.destroy_process_group()


def test_allgather_fixed_and_sized(tmp_path):
    out = str(tmp_path / "ag")
    mp.start_processes(_main, args=(3, _free_port(), out), nprocs=3, join=True, start_method="spawn")
    for r in range(3):
        assert open(f"{out}.{r}").read() == "ok"
