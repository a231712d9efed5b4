"""Data-parallel mini-batch SGD (models/sgd.py, K13 + K13b + K14 on GPU, torch on CPU) over gloo.

With W ranks holding the SAME shard, every all-reduced message is exactly W times the single-rank
one and the update divides by the all-reduced weight sum, so the W-rank run must reproduce the
1-rank coefficients; with disjoint shards the fit must still recover the generating model."""
import json
import os
import socket

import numpy as np
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _data(n=6000, d=6, seed=0):
    import torch
    g = torch.Generator().manual_seed(seed)
    x = torch.randn(n, d, generator=g, dtype=torch.float64)
    w = torch.linspace(-1.0, 1.5, d, dtype=torch.float64)
    p = torch.sigmoid(x @ w + 0.3)
    y = (torch.rand(n, generator=g, dtype=torch.float64) < p).double()
    return x, y, w


def _fit(comm, x, y, steps=60):
    from clustermachinelearningforhospitalnetworks_apache_spark_amd.models.sgd import LogisticSGD
    opt = LogisticSGD(x, x.shape[1], y, None, comm, 500, 0.5, 0.9)
    loss = 0.0
    for e in range(steps // opt.nb):
        loss = opt.epoch(e, 0.5)
    return opt.coef.tolist(), loss


def _rank_main(rank, world, port, out, disjoint):
    os.environ.update({"RANK": str(rank), "WORLD_SIZE": str(world), "LOCAL_RANK": str(rank),
                       "MASTER_ADDR": "127.0.0.1", "MASTER_PORT": str(port)})
    import torch
    torch.set_num_threads(1)
    from clustermachinelearningforhospitalnetworks_apache_spark_amd.parallel.comm import Communicator
    comm = Communicator.from_env(want_gpu=False)
    x, y, _ = _data()
    if disjoint:
        x, y = x[rank::world].contiguous(), y[rank::world].contiguous()
    coef, loss = _fit(comm, x, y)
    if rank == 0:
        with open(out, "w") as fh:
            json.dump({"coef": coef, "loss": loss}, fh)
    comm.shutdown()


def _run(world, tmp_path, disjoint):
    out = str(tmp_path / f"sgd_{world}_{int(disjoint)}.json")
    mp.start_processes(_rank_main, args=(world, _free_port(), out, disjoint), nprocs=world, join=True,
                       start_method="spawn")
    with open(out) as fh:
        return json.load(fh)


def test_sgd_replicated_shards_match_single_rank(tmp_path):
    from clustermachinelearningforhospitalnetworks_apache_spark_amd.parallel.comm import local_comm
    x, y, _ = _data()
    c1, l1 = _fit(local_comm(), x, y)
    r2 = _run(2, tmp_path, disjoint=False)
    np.testing.assert_allclose(r2["coef"], c1, rtol=1e-12, atol=1e-14)
    assert abs(r2["loss"] - l1) < 1e-12


def test_sgd_disjoint_shards_recover_model(tmp_path):
    _, _, w = _data()
    r = _run(2, tmp_path, disjoint=True)
    coef = np.array(r["coef"])
    cos = coef[:-1] @ w.numpy() / (np.linalg.norm(coef[:-1]) * np.linalg.norm(w.numpy()))
    assert cos > 0.98 and abs(coef[-1] - 0.3) < 0.2
