"""Exact bound-pruned Lloyd steps (``LloydEngine(prune=True)``, K9p ``kmeans_prune.hip``) against the
full step: the same labels, sums and centres at every iteration, with most rows pruned once the
centres settle. CPU tests run the torch form of every pass; GPU tests the HIP bounds kernel, the
gathered K9 re-assignment and the hipBLASLt lower bounds."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

from clustermachinelearningforhospitalnetworks_apache_spark_amd.models.kmeans import LloydEngine
from clustermachinelearningforhospitalnetworks_apache_spark_amd.ops import kmeans_ops as K


def _blobs(n, d, k, seed, scale=3.0, device="cpu", dtype=torch.float64):
    g = torch.Generator(device=device)
    g.manual_seed(seed)
    cen = torch.randn(k, d, generator=g, device=device) * scale
    lab = torch.randint(0, k, (n,), generator=g, device=device)
    return (cen[lab] + torch.randn(n, d, generator=g, device=device)).to(dtype)


def _pair(x, d, k, init, steps, **kw):
    a = LloydEngine(x, d, k, **kw)
    b = LloydEngine(x, d, k, prune=True, **kw)
    a.set_centers(init)
    b.set_centers(init)
    stats = []
    for _ in range(steps):
        a.step()
        b.step()
        stats.append(b.prune_stats())
        n = a.n
        assert torch.equal(a.labels[:n].long(), b.labels[:n].long())
        torch.testing.assert_close(b.centers, a.centers, rtol=1e-12, atol=1e-12)
        # full step: Σ of the assign's f32 row distances; pruned: Σ_j (Q_j - 2 c_j·S_j + n_j |c_j|²) in f64
        rtol = 1e-5 if x.is_cuda else 1e-9
        assert abs(float(b.last_cost) - float(a.last_cost)) <= rtol * max(1.0, abs(float(a.last_cost)))
        assert torch.equal(a._shift2 <= 1e-8, b._shift2 <= 1e-8)
    return a, b, stats


@pytest.mark.parametrize("n,d,k,scale", [(20_003, 8, 12, 3.0), (6_001, 32, 40, 1.0), (5_000, 5, 3, 6.0)])
def test_pruned_equals_full_cpu(n, d, k, scale):
    x = _blobs(n, d, k, seed=n, scale=scale)
    init = x[torch.randperm(n, generator=torch.Generator().manual_seed(1))[:k]].numpy()
    _, _, stats = _pair(x, d, k, init, 12)
    assert stats[0]["full"], "the first step has no bounds yet"
    assert any(not s["full"] and s["reassigned_rows"] < n // 4 for s in stats[1:])


def test_pruned_duplicate_centres_and_single_centre_cpu():
    x = _blobs(4_000, 6, 5, seed=3)
    init = np.repeat(x[:3].numpy(), [2, 2, 1], axis=0)  # coincident centres: never prunable by thr
    _pair(x, 6, 5, init, 6)
    _pair(x, 6, 1, x[:1].numpy(), 3)


def test_pruned_spherical_cpu():
    x = _blobs(3_000, 10, 6, seed=5) + 0.5
    init = x[:6].numpy()
    _pair(x, 10, 6, init, 8, spherical=True)


def test_pruned_fit_converges_like_full_cpu():
    x = _blobs(8_000, 4, 6, seed=9, scale=5.0)
    init = x[:6].numpy()
    a = LloydEngine(x, 4, 6)
    b = LloydEngine(x, 4, 6, prune=True)
    a.set_centers(init)
    b.set_centers(init)
    assert a.fit(50, 1e-6) == b.fit(50, 1e-6)
    torch.testing.assert_close(b.centers, a.centers, rtol=1e-12, atol=1e-12)
    assert abs(a.training_cost() - b.training_cost()) <= 1e-9 * a.training_cost()


def test_bounds_pass_cpu_semantics():
    lab = torch.tensor([0, 1, 1, 0, 2])
    ub = torch.tensor([1.0, 1.0, 3.0, 0.5, 1.0], dtype=torch.float64)
    lb = torch.tensor([5.0, 1.5, 9.0, 0.0, 1.0], dtype=torch.float64)
    drift = torch.tensor([0.5, 0.0, 0.25], dtype=torch.float64)
    dmax = torch.tensor([0.5, 0.25, 0.0], dtype=torch.float64)
    thr = torch.tensor([1.0, 0.5, 0.0], dtype=torch.float64)
    cand = torch.zeros(5, dtype=torch.int64)
    cnt = torch.zeros(1, dtype=torch.int64)
    K.prune_bounds(lab, ub, lb, drift, dmax, thr, 0.0, 3, cand, cnt)
    assert ub.tolist() == [1.5, 1.0, 3.0, 1.0, 1.25]
    assert lb.tolist() == [4.75, 1.0, 8.5, 0.0, 0.5]
    # row 0: 1.5 <= 4.75; row 1: 1.0 <= lb 1.0; row 2: 3 <= 8.5; row 3: 1.0 <= thr 1.0; row 4 fails both
    assert cnt.item() == 1 and cand[0].item() == 4


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _rank_main(rank, world, port, out):
    os.environ.update({"RANK": str(rank), "WORLD_SIZE": str(world), "LOCAL_RANK": str(rank),
                       "MASTER_ADDR": "127.0.0.1", "MASTER_PORT": str(port), "CML_FORCE_CPU": "1"})
    torch.set_num_threads(1)
    from clustermachinelearningforhospitalnetworks_apache_spark_amd.parallel.comm import Communicator
    comm = Communicator.from_env(want_gpu=False)
    x = _blobs(9_000, 6, 8, seed=4)
    init = x[:8].numpy()
    shard = x[rank::world].contiguous()
    eng = LloydEngine(shard, 6, 8, comm, prune=True)
    eng.set_centers(init)
    for _ in range(10):
        eng.step()
    if rank == 0:
        np.save(out, eng.centers.numpy())
    comm.shutdown()


def test_pruned_distributed_gloo_matches_single_rank(tmp_path):
    out = str(tmp_path / "c.npy")
    mp.start_processes(_rank_main, args=(2, _free_port(), out), nprocs=2, join=True, start_method="spawn")
    x = _blobs(9_000, 6, 8, seed=4)
    ref = LloydEngine(x, 6, 8)
    ref.set_centers(x[:8].numpy())
    for _ in range(10):
        ref.step()
    np.testing.assert_allclose(np.load(out), ref.centers.numpy(), rtol=1e-12, atol=1e-12)


# ------------------------------------------------------------------------------------------- GPU
@pytest.mark.gpu
@pytest.mark.parametrize("n,d,k,scale", [(300_001, 256, 256, 1.0), (200_000, 128, 64, 1.0), (50_000, 64, 300, 3.0),
                                         (60_000, 64, 200, 0.5)])
def test_pruned_equals_full_gpu(n, d, k, scale):
    x = _blobs(n, d, k, seed=7, scale=scale, device="cuda", dtype=torch.bfloat16)
    init = x[torch.randperm(n, device="cuda")[:k]].double().cpu().numpy()
    _, b, stats = _pair(x, d, k, init, 10, use_graph=False)
    assert b._pst.ub.dtype == torch.float32
    if scale >= 1.0:  # separated blobs: the bounds prune; overlapping ones (0.5) re-assign in full
        assert any(not s["full"] for s in stats[1:]), stats


@pytest.mark.gpu
def test_pruned_fp8_rows_gpu():
    n, d, k = 200_000, 256, 64
    x = _blobs(n, d, k, seed=11, scale=1.0, device="cuda", dtype=torch.float32).clamp(-400, 400)
    x8 = x.to(torch.float8_e4m3fn)
    init = x8[:k].float().double().cpu().numpy()
    _pair(x8, d, k, init, 8, use_graph=False)


@pytest.mark.gpu
def test_bounds_kernel_matches_torch_pass():
    n, k = 1_000_003, 200
    g = torch.Generator(device="cuda")
    g.manual_seed(0)
    lab = torch.randint(0, k, (n,), device="cuda", generator=g, dtype=torch.int32)
    ub = torch.rand(n, device="cuda", generator=g) * 4
    lb = torch.rand(n, device="cuda", generator=g) * 8
    drift = torch.rand(k, device="cuda", generator=g) * 0.1
    top = torch.topk(drift, 2)
    dmax = torch.stack([top.values[0], top.values[1], top.indices[0].float()])
    thr = torch.rand(k, device="cuda", generator=g) * 3
    cand = torch.zeros(n, dtype=torch.int32, device="cuda")
    cnt = torch.zeros(1, dtype=torch.int32, device="cuda")
    ub_c, lb_c = ub.double().cpu(), lb.double().cpu()
    cand_c = torch.zeros(n, dtype=torch.int64)
    cnt_c = torch.zeros(1, dtype=torch.int64)
    K.prune_bounds(lab, ub, lb, drift, dmax, thr, 0.01, k, cand, cnt)
    K.prune_bounds(lab.cpu(), ub_c, lb_c, drift.double().cpu(), dmax.double().cpu(), thr.double().cpu(), 0.01, k,
                   cand_c, cnt_c)
    torch.testing.assert_close(ub.cpu().double(), ub_c, rtol=1e-6, atol=0)
    torch.testing.assert_close(lb.cpu().double(), lb_c, rtol=1e-6, atol=1e-6)
    m = int(cnt.item())
    got = set(cand[:m].cpu().tolist())
    want = set(cand_c[: int(cnt_c.item())].tolist())
    # the kernel rounds its bounds outwards: it may keep a few more candidates, never fewer
    assert want <= got and len(got - want) <= max(10, m // 10000)
    assert len(got) == m


def test_kmeans_estimator_prune_conf_cpu():
    import pandas as pd
    from clustermachinelearningforhospitalnetworks_apache_spark_amd.ml.clustering import KMeans
    from clustermachinelearningforhospitalnetworks_apache_spark_amd.ml.feature import VectorAssembler
    from clustermachinelearningforhospitalnetworks_apache_spark_amd.sql import SparkSession
    spark = SparkSession.builder.master("local[1]").getOrCreate()
    x = _blobs(5_000, 4, 5, seed=21, scale=4.0).numpy()
    df = spark.createDataFrame(pd.DataFrame(x, columns=list("abcd")))
    df = VectorAssembler(inputCols=list("abcd"), outputCol="features").transform(df)
    try:
        spark.conf.set("cml.ml.kmeans.prune", "false")
        full = KMeans(k=5, seed=3, maxIter=30).fit(df)
        spark.conf.set("cml.ml.kmeans.prune", "true")
        pruned = KMeans(k=5, seed=3, maxIter=30).fit(df)
    finally:
        spark.conf.unset("cml.ml.kmeans.prune")
    np.testing.assert_allclose(np.array(pruned.clusterCenters()), np.array(full.clusterCenters()), rtol=1e-12,
                               atol=1e-12)
    assert pruned.summary.numIter == full.summary.numIter
    assert pruned.summary.clusterSizes == full.summary.clusterSizes
    assert abs(pruned.summary.trainingCost - full.summary.trainingCost) <= 1e-9 * full.summary.trainingCost


@pytest.mark.gpu
@pytest.mark.parametrize("m,k", [(100_003, 256), (777, 64), (5, 12)])
def test_lower_bound_kernel_matches_torch(m, k):
    g = torch.Generator(device="cuda")
    g.manual_seed(m)
    dist = torch.randn(m, k, device="cuda", generator=g) * 100
    lab = torch.randint(0, k, (m,), device="cuda", generator=g, dtype=torch.int32)
    xn = torch.rand(m, device="cuda", generator=g) * 500 + 200
    out = torch.empty(m, device="cuda")
    K.prune_lower(dist, lab, xn, 300.0, 3e-5, out)
    ref = dist.double().scatter(1, lab.long()[:, None], float("inf")).min(1).values + xn.double()
    ref = (ref - 3e-5 * (xn.double() + 300.0)).clamp(min=0).sqrt()
    torch.testing.assert_close(out.double(), ref, rtol=2e-6, atol=1e-5)
    assert bool((out.double() <= ref * (1 + 1e-7) + 1e-6).all())
