"""Multi-rank GPU engines on ONE MI355X: two ranks share cuda:0 and talk over gloo (RCCL refuses two
ranks on one device). This runs the distributed GPU code path the 8-GPU bench uses — row chunks with
asynchronous per-chunk all-reduces, incremental sums per chunk, the device-side GLM gradient
reduction — and checks it against one rank holding all rows. Data on a 1/8 grid keeps every f64 sum
exact, so the centres must agree bit for bit.
"""
import json
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu

N, D, K = 60_000, 128, 32


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _data():
    rs = np.random.RandomState(7)
    cen = rs.randn(K, D) * 3
    x = cen[rs.randint(0, K, N)] + rs.randn(N, D)
    return np.round(x * 8) / 8


def _fit(x_local, comm, chunks):
    import torch
    from clustermachinelearningforhospitalnetworks_apache_spark_amd.models.kmeans import LloydEngine
    full = _data()
    eng = LloydEngine(torch.as_tensor(x_local, device="cuda").to(torch.bfloat16), D, K, comm, row_chunks=chunks,
                      prune=False)
    eng.set_centers(full[:K])
    modes = []
    for _ in range(6):
        eng.step()
        torch.cuda.synchronize()
        modes.append(eng.delta.was_full() if eng.delta is not None else True)
    return eng.centers.cpu().numpy(), eng.training_cost(), modes


def _rank_main(rank, world, port, out_path):
    os.environ.update({"RANK": str(rank), "WORLD_SIZE": str(world), "MASTER_ADDR": "127.0.0.1",
                       "MASTER_PORT": str(port)})
    import torch
    import torch.distributed as dist
    from clustermachinelearningforhospitalnetworks_apache_spark_amd.parallel.comm import Communicator
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    comm = Communicator(rank, world, torch.device("cuda", 0), "gloo", dist.group.WORLD)
    x = _data()
    lo, hi = rank * N // world, (rank + 1) * N // world
    centers, cost, modes = _fit(x[lo:hi], comm, chunks=2)
    if rank == 0:
        with open(out_path, "w") as fh:
            json.dump({"centers": centers.tolist(), "cost": cost, "modes": modes}, fh)
    dist.barrier()
    dist.destroy_process_group()


def test_two_ranks_on_one_gpu_match_single_rank(tmp_path):
    from clustermachinelearningforhospitalnetworks_apache_spark_amd.parallel.comm import local_comm
    out = str(tmp_path / "w2.json")
    ctx = mp.get_context("spawn")
    port = _free_port()
    procs = [ctx.Process(target=_rank_main, args=(r, 2, port, out)) for r in range(2)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(180)
    assert all(p.exitcode == 0 for p in procs), [p.exitcode for p in procs]
    res = json.load(open(out))
    ref_centers, ref_cost, _ = _fit(_data(), local_comm(), chunks=1)
    np.testing.assert_array_equal(np.asarray(res["centers"]), ref_centers)
    assert abs(res["cost"] - ref_cost) <= 1e-9 * abs(ref_cost)
    assert res["modes"][0] and not all(res["modes"]), "incremental path not exercised on the ranks"


# ---- the default GPU path on two ranks: device k-means|| (pruned candidate passes), the seeded first
# step and graph-captured pruned steps split around the all-reduce (graph | all-reduce | graph)

N2, D2, K2 = 200_000, 128, 64


def _data2():
    rs = np.random.RandomState(11)
    cen = rs.randn(K2, D2) * 4
    x = cen[rs.randint(0, K2, N2)] + rs.randn(N2, D2)
    return np.round(x * 8) / 8


def _fit2(x_local, comm, use_graph=True):
    import torch
    from clustermachinelearningforhospitalnetworks_apache_spark_amd.models.kmeans import LloydEngine
    eng = LloydEngine(torch.as_tensor(x_local, device="cuda").to(torch.bfloat16), D2, K2, comm, prune=True,
                      precision="bf16", use_graph=use_graph)
    eng.track_prune = True
    init = eng.init_kmeans_parallel(seed=5)
    eng.set_centers(init)
    seeded = bool(eng._seeded)
    eng.fit(10, 0.0)
    torch.cuda.synchronize()
    return {"init": np.asarray(init).tolist(), "centers": eng.centers.cpu().numpy().tolist(),
            "cost": eng.training_cost(), "pdev": bool(eng._pdev), "seeded": seeded,
            "graph": isinstance(eng._graph, tuple) if comm.is_distributed else eng._graph is not None,
            "hist": eng.prune_history()}


def _rank_main2(rank, world, port, out_path, use_graph=True):
    os.environ.update({"RANK": str(rank), "WORLD_SIZE": str(world), "MASTER_ADDR": "127.0.0.1",
                       "MASTER_PORT": str(port), "CML_KMEANS_PRUNE": "1"})
    import torch
    import torch.distributed as dist
    from clustermachinelearningforhospitalnetworks_apache_spark_amd.parallel.comm import Communicator
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    comm = Communicator(rank, world, torch.device("cuda", 0), "gloo", dist.group.WORLD)
    x = _data2()
    lo, hi = rank * N2 // world, (rank + 1) * N2 // world
    res = _fit2(x[lo:hi], comm, use_graph)
    if rank == 0:
        with open(out_path, "w") as fh:
            json.dump(res, fh)
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("use_graph,overlap", [(False, False), (True, False), (False, True)])
def test_two_ranks_default_path_match_single_rank(tmp_path, monkeypatch, use_graph, overlap):
    """Two ranks on the default GPU path (pruned init, seeded step, eager pruned steps around the
    all-reduce — or split graphs) give the single-rank fit bit for bit: init centres, final centres and
    cost (1/8-grid data: every f64 sum is exact). ``overlap``: the seeded step's full accumulate in two
    chunks whose all-reduces overlap the next chunk (forced on at this size) — the same bits."""
    from clustermachinelearningforhospitalnetworks_apache_spark_amd.parallel.comm import local_comm
    monkeypatch.setenv("CML_KMEANS_PRUNE", "1")
    if overlap:
        monkeypatch.setenv("CML_KMEANS_OVERLAP_ROWS", "1")
    out = str(tmp_path / "w2d.json")
    ctx = mp.get_context("spawn")
    port = _free_port()
    procs = [ctx.Process(target=_rank_main2, args=(r, 2, port, out, use_graph)) for r in range(2)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(240)
    assert all(p.exitcode == 0 for p in procs), [p.exitcode for p in procs]
    res = json.load(open(out))
    ref = _fit2(_data2(), local_comm(), use_graph)
    assert res["pdev"] and ref["pdev"] and res["seeded"] and res["graph"] == use_graph, res
    np.testing.assert_array_equal(np.asarray(res["init"]), np.asarray(ref["init"]))
    np.testing.assert_array_equal(np.asarray(res["centers"]), np.asarray(ref["centers"]))
    assert abs(res["cost"] - ref["cost"]) <= 1e-9 * abs(ref["cost"])


# ---- four ranks, uneven shards: one rank with no rows, one with fewer rows than one K9r round (64),
# and one whose candidate cap is tiny (its pruned steps and its seeded first step fall back to the full
# pass while the others run candidate passes: the collectives must line up all the same)

_SPLITS4 = [0, 0, 37, 120_000, N2]  # rank r holds rows [_SPLITS4[r], _SPLITS4[r + 1])


def _rank_main4(rank, world, port, out_path):
    os.environ.update({"RANK": str(rank), "WORLD_SIZE": str(world), "MASTER_ADDR": "127.0.0.1",
                       "MASTER_PORT": str(port), "CML_KMEANS_PRUNE": "1"})
    import torch
    import torch.distributed as dist
    from clustermachinelearningforhospitalnetworks_apache_spark_amd.models.kmeans import LloydEngine
    from clustermachinelearningforhospitalnetworks_apache_spark_amd.parallel.comm import Communicator
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    comm = Communicator(rank, world, torch.device("cuda", 0), "gloo", dist.group.WORLD)
    if rank == 2:
        LloydEngine._PRUNE_CAP = 1e-4  # this rank's steps take the full-pass branch
    x = _data2()
    res = _fit2(x[_SPLITS4[rank]:_SPLITS4[rank + 1]], comm, use_graph=False)
    res["rows"] = _SPLITS4[rank + 1] - _SPLITS4[rank]
    with open(f"{out_path}.{rank}", "w") as fh:
        json.dump(res, fh)
    dist.barrier()
    dist.destroy_process_group()


def test_four_uneven_ranks_with_an_empty_one_match_single_rank(tmp_path, monkeypatch):
    """the default device path (pruned k-means|| init, seeded step, pruned steps) on
    four gloo ranks sharing the GPU — an empty rank, a 37-row rank, a rank forced onto the _PRUNE_CAP
    fallback — gives the single-rank fit bit for bit."""
    from clustermachinelearningforhospitalnetworks_apache_spark_amd.parallel.comm import local_comm
    monkeypatch.setenv("CML_KMEANS_PRUNE", "1")
    out = str(tmp_path / "w4")
    ctx = mp.get_context("spawn")
    port = _free_port()
    procs = [ctx.Process(target=_rank_main4, args=(r, 4, port, out)) for r in range(4)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(300)
    assert all(p.exitcode == 0 for p in procs), [p.exitcode for p in procs]
    res = [json.load(open(f"{out}.{r}")) for r in range(4)]
    ref = _fit2(_data2(), local_comm(), use_graph=False)
    for r in range(4):
        assert res[r]["rows"] == _SPLITS4[r + 1] - _SPLITS4[r]
        np.testing.assert_array_equal(np.asarray(res[r]["init"]), np.asarray(ref["init"]))
        np.testing.assert_array_equal(np.asarray(res[r]["centers"]), np.asarray(ref["centers"]))
        assert abs(res[r]["cost"] - ref["cost"]) <= 1e-9 * abs(ref["cost"])
    # the capped rank took the full-pass branch, the big rank pruned
    assert any(full for full, _ in res[2]["hist"]), res[2]["hist"]
    assert any(not full for full, _ in res[3]["hist"][1:]), res[3]["hist"]


# ---- precision "screen" (f32 rows, the certified exact path) over three gloo ranks, one of them empty:
# each rank's double-double sums fold in rank order, so the fit is the one-rank fit bit for bit — for data
# that is not on any grid (plain f32 rows)

_SPLITS_S = [0, 41_000, 41_000, 90_000]
NS, DS, KS = 90_000, 128, 24


def _data_s():
    rs = np.random.RandomState(19)
    cen = rs.randn(KS, DS) * 3 + 50.0
    return (cen[rs.randint(0, KS, NS)] + rs.randn(NS, DS)).astype(np.float32)


def _fit_s(x_local, comm):
    import torch
    from clustermachinelearningforhospitalnetworks_apache_spark_amd.models.kmeans import LloydEngine
    eng = LloydEngine(torch.as_tensor(x_local, device="cuda"), DS, KS, comm, precision="screen")
    init = eng.init_kmeans_parallel(seed=8)
    eng.set_centers(init)
    it = eng.fit(10, 0.0)
    return {"init": np.asarray(init).tolist(), "centers": eng.centers.cpu().numpy().tolist(), "it": it,
            "cost": eng.training_cost(), "sizes": eng.cluster_sizes()}


def _rank_main_s(rank, world, port, out_path):
    os.environ.update({"RANK": str(rank), "WORLD_SIZE": str(world), "MASTER_ADDR": "127.0.0.1",
                       "MASTER_PORT": str(port)})
    import torch
    import torch.distributed as dist
    from clustermachinelearningforhospitalnetworks_apache_spark_amd.parallel.comm import Communicator
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    comm = Communicator(rank, world, torch.device("cuda", 0), "gloo", dist.group.WORLD)
    x = _data_s()
    res = _fit_s(x[_SPLITS_S[rank]:_SPLITS_S[rank + 1]], comm)
    with open(f"{out_path}.{rank}", "w") as fh:
        json.dump(res, fh)
    dist.barrier()
    dist.destroy_process_group()


def test_screen_three_ranks_with_an_empty_one_match_single_rank(tmp_path):
    from clustermachinelearningforhospitalnetworks_apache_spark_amd.parallel.comm import local_comm
    out = str(tmp_path / "s3")
    ctx = mp.get_context("spawn")
    port = _free_port()
    procs = [ctx.Process(target=_rank_main_s, args=(r, 3, port, out)) for r in range(3)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(300)
    assert all(p.exitcode == 0 for p in procs), [p.exitcode for p in procs]
    res = [json.load(open(f"{out}.{r}")) for r in range(3)]
    ref = _fit_s(_data_s(), local_comm())
    for r in range(3):
        np.testing.assert_array_equal(np.asarray(res[r]["init"]), np.asarray(ref["init"]))
        np.testing.assert_array_equal(np.asarray(res[r]["centers"]), np.asarray(ref["centers"]))
        assert res[r]["it"] == ref["it"] and res[r]["sizes"] == ref["sizes"]
        assert abs(res[r]["cost"] - ref["cost"]) <= 1e-12 * abs(ref["cost"])


def test_bench_two_rank_launch_on_one_gpu():
    """The driver's N > 1 bench launch (torch.distributed.run, one rank per device) with both ranks on cuda:0 and
    gloo collectives (RCCL needs a device per rank): the GPU shards, the multi-rank fit and the one-line JSON
    contract (n_gpus = 2, dp2, whole-job value)."""
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ, CML_COMM_BACKEND="gloo", PYTHONPATH=root)
    out = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
                          "--master-addr", "127.0.0.1", "--master-port", str(29700 + os.getpid() % 200),
                          os.path.join(root, "bench.py"), "--gpus", "2", "--steps", "3", "--warmup", "1",
                          "--rows", "2000000", "--no-overlap"],
                         capture_output=True, text=True, env=env, timeout=110, cwd=root)
    assert out.returncode == 0, out.stderr[-3000:]
    lines = [ln for ln in out.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, out.stdout[-2000:]
    res = json.loads(lines[0])
    assert res["n_gpus"] == 2 and res["config"]["parallelism"] == "dp2" and res["dtype"] == "bf16"
    assert res["steps"] == 3 and res["value"] > 0 and res["extra"]["iterations"] == 3


# ---- the split full-pass step: on data the bounds cannot prune, each full-pass step runs in
# two row chunks and chunk 0's all-reduce is in flight during chunk 1's K9r pass; A + B must be the one-message
# step bit for bit, on two ranks and against one rank

N3, D3, K3 = 240_000, 128, 64


def _data3():
    rs = np.random.RandomState(23)
    cen = rs.randn(K3, D3) * 0.5  # overlapping blobs: the bounds prune little, the gate picks full passes
    x = cen[rs.randint(0, K3, N3)] + rs.randn(N3, D3)
    return np.round(x * 8) / 8


def _fit3(x_local, comm):
    import torch
    from clustermachinelearningforhospitalnetworks_apache_spark_amd.models.kmeans import LloydEngine
    eng = LloydEngine(torch.as_tensor(x_local, device="cuda").to(torch.bfloat16), D3, K3, comm, prune=True,
                      precision="bf16")
    eng.set_centers(eng.init_kmeans_parallel(seed=2))
    eng.fit(12, 0.0)
    torch.cuda.synchronize()
    return {"centers": eng.centers.cpu().numpy().tolist(), "cost": eng.training_cost(),
            "split": int(getattr(eng._pst, "split_steps", 0)), "pdev": bool(eng._pdev)}


def _rank_main3(rank, world, port, out_path):
    os.environ.update({"RANK": str(rank), "WORLD_SIZE": str(world), "MASTER_ADDR": "127.0.0.1",
                       "MASTER_PORT": str(port), "CML_KMEANS_OVERLAP_ROWS": "1", "CML_KMEANS_SPLIT_FULL": "1"})
    import torch
    import torch.distributed as dist
    from clustermachinelearningforhospitalnetworks_apache_spark_amd.parallel.comm import Communicator
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    comm = Communicator(rank, world, torch.device("cuda", 0), "gloo", dist.group.WORLD)
    x = _data3()
    lo, hi = rank * N3 // world, (rank + 1) * N3 // world
    res = _fit3(x[lo:hi], comm)
    with open(f"{out_path}.{rank}", "w") as fh:
        json.dump(res, fh)
    dist.barrier()
    dist.destroy_process_group()


def test_split_full_pass_steps_two_ranks_match_single_rank(tmp_path, monkeypatch):
    from clustermachinelearningforhospitalnetworks_apache_spark_amd.parallel.comm import local_comm
    out = str(tmp_path / "w3")
    ctx = mp.get_context("spawn")
    port = _free_port()
    procs = [ctx.Process(target=_rank_main3, args=(r, 2, port, out)) for r in range(2)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(240)
    assert all(p.exitcode == 0 for p in procs), [p.exitcode for p in procs]
    res = [json.load(open(f"{out}.{r}")) for r in range(2)]
    monkeypatch.setenv("CML_KMEANS_SPLIT_FULL", "0")
    ref = _fit3(_data3(), local_comm())
    assert ref["pdev"] and ref["split"] == 0
    for r in range(2):
        assert res[r]["split"] > 0, res[r]["split"]  # the overlapped steps ran
        np.testing.assert_array_equal(np.asarray(res[r]["centers"]), np.asarray(ref["centers"]))
        assert res[r]["cost"] == ref["cost"]
    # and on one rank: the split step (forced) is the one-message step bit for bit
    monkeypatch.setenv("CML_KMEANS_SPLIT_FULL", "1")
    monkeypatch.setenv("CML_KMEANS_OVERLAP_ROWS", "1")
    one = _fit3(_data3(), local_comm())
    assert one["split"] > 0
    np.testing.assert_array_equal(np.asarray(one["centers"]), np.asarray(ref["centers"]))
    assert one["cost"] == ref["cost"]
