"""Exact bound-pruned Lloyd steps (``LloydEngine(prune=True)``, K9p ``kmeans_prune.hip``) against the
full step: the same labels, sums and centres at every iteration, with most rows pruned once the
centres settle. CPU tests run the torch form of every pass; GPU tests the device pruned step (K9p
bounds + gate, K9r top-2 full pass and candidate pass, incremental sums, centre statistics) where
the K9r assign applies, and the torch-bounds form (gathered K9 re-assignment, GEMM lower bounds)
for the other shapes."""
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
    a = LloydEngine(x, d, k, prune=False, **kw)
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
        # GPU: f64 costs of the same labels and bf16 centres (the device pruned step and the full step both
        # from the exact sums and f64 norms; the torch-bounds form by the exact cost pass);
        # CPU: full = Σ of the f64 row distances, pruned = Σ_j (Q_j - 2 c_j·S_j + n_j |c_j|²) in f64
        rtol = 1e-12 if x.is_cuda else 1e-9
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
    a = LloydEngine(x, 4, 6, prune=False)
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
@pytest.mark.parametrize("n,d,k,scale", [(300_001, 256, 256, 1.0), (200_000, 128, 64, 1.0), (120_000, 512, 128, 1.0),
                                         (50_000, 64, 300, 3.0),
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


# ---------------------------------------------------------------- device pruned-step kernels
def _rr_setup(n, d, k, seed):
    from clustermachinelearningforhospitalnetworks_apache_spark_amd.models.kmeans import to_device_matrix
    from clustermachinelearningforhospitalnetworks_apache_spark_amd.utils.device import padded_dim, round_up
    x = to_device_matrix(_blobs(n, d, k, seed=seed, device="cuda", dtype=torch.bfloat16), d)
    dp = x.shape[1]
    kp = round_up(k, 32)
    pick = torch.randint(0, n, (k,), device="cuda", generator=torch.Generator(device="cuda").manual_seed(seed))
    cent = x[pick, :d]
    cent = cent.double().contiguous()
    cb = torch.zeros((kp, dp), dtype=torch.bfloat16, device="cuda")
    cn = torch.zeros(kp, dtype=torch.float32, device="cuda")
    K.update_centers(None, k, d, cent.clone(), cb, dp, kp, cn, None)
    xn = K.row_sqnorm(x, n, dp)
    return x, dp, kp, cb, cn, xn


def _exact_top2(x, d, cb, k):
    xf = x[:, :d].double()
    c = cb[:k, :d].double()
    dist = (xf * xf).sum(1, keepdim=True) - 2 * xf @ c.T + (c * c).sum(1)[None]
    top = torch.topk(dist, min(2, k), dim=1, largest=False)
    return dist, top.values, top.indices


@pytest.mark.gpu
@pytest.mark.parametrize("n,d,k", [(70_001, 256, 256), (33_333, 128, 64), (20_000, 512, 100), (1, 256, 2),
                                   (4_097, 256, 1)])
def test_rr_top2_full_pass_bounds(n, d, k):
    """K9r mode 1: labels equal the plain K9r pass; ub >= the exact distance to the label's centre and
    lb <= the exact distance to every other centre (f64 over the same bf16 operands), tight within tau."""
    x, dp, kp, cb, cn, xn = _rr_setup(n, d, k, seed=n)
    plan = K.plan_assign(n, dp, k)
    assert plan.rr_ct > 0
    lab0 = torch.zeros(n, dtype=torch.int32, device="cuda")
    K.assign_bf16(x, n, dp, cb, cn, plan, lab0, None, torch.zeros(plan.grid, dtype=torch.float64, device="cuda"),
                  xnorm=xn)
    lab = torch.zeros(n, dtype=torch.int32, device="cuda")
    ub = torch.zeros(n, device="cuda")
    lb = torch.zeros(n, device="cuda")
    from clustermachinelearningforhospitalnetworks_apache_spark_amd.models.kmeans import LloydEngine
    tau = LloydEngine.prune_tau(dp)
    mc = torch.tensor([float(cn[:k].max())], device="cuda")
    K.assign_rr_ext(1, x, n, dp, cb, cn, plan, xn, lab, None, ub, lb, mc, tau)
    torch.cuda.synchronize()
    assert torch.equal(lab, lab0)
    dist, vals, _ = _exact_top2(x, d, cb, k)
    own = dist.gather(1, lab.long()[:, None]).squeeze(1).clamp(min=0).sqrt()
    assert bool((ub.double() >= own * (1 - 1e-12)).all())
    if k > 1:
        other = dist.scatter(1, lab.long()[:, None], float("inf")).min(1).values.clamp(min=0).sqrt()
        assert bool((lb.double() <= other * (1 + 1e-12)).all())
        slack = (tau * (xn.double() + float(mc)) + 1e-6 * other ** 2).sqrt() * 2 + 1e-3
        assert bool(((other - lb.double()) <= slack).all())
    else:
        assert bool(torch.isinf(lb).all())


@pytest.mark.gpu
@pytest.mark.parametrize("n,d,k,m", [(90_000, 256, 256, 5_000), (90_000, 256, 256, 0), (50_000, 128, 64, 49_999),
                                     (30_000, 512, 128, 777), (64, 256, 33, 64)])
def test_rr_candidate_pass_matches_full(n, d, k, m):
    """K9r mode 2 on a scattered candidate list (count read on the device): the candidates get the
    labels and bounds mode 1 gives them; every other row is untouched; the change log lists exactly
    the candidates whose label changed, with their old label."""
    x, dp, kp, cb, cn, xn = _rr_setup(n, d, k, seed=n + m)
    plan = K.plan_assign(n, dp, k)
    from clustermachinelearningforhospitalnetworks_apache_spark_amd.models.kmeans import LloydEngine
    tau = LloydEngine.prune_tau(dp)
    mc = torch.tensor([float(cn[:k].max())], device="cuda")
    ref_lab = torch.zeros(n, dtype=torch.int32, device="cuda")
    ref_ub, ref_lb = torch.zeros(n, device="cuda"), torch.zeros(n, device="cuda")
    K.assign_rr_ext(1, x, n, dp, cb, cn, plan, xn, ref_lab, None, ref_ub, ref_lb, mc, tau)
    g = torch.Generator(device="cuda").manual_seed(m)
    old = torch.randint(0, k, (n,), device="cuda", generator=g, dtype=torch.int32)
    cand = torch.randperm(n, device="cuda", generator=g)[:m].to(torch.int32)
    tr = plan.round_rows
    cap = max(m, 1)
    pad = -(-cap // tr) * tr + tr
    idx = torch.zeros(pad, dtype=torch.int32, device="cuda")
    idx[:m] = cand
    clab = torch.zeros(pad, dtype=torch.int32, device="cuda")
    clab[:m] = old[cand.long()]
    cxn = torch.zeros(pad, device="cuda")
    cxn[:m] = xn[cand.long()]
    cnt = torch.tensor([m], dtype=torch.int32, device="cuda")
    lab = old.clone()
    ub = torch.full((n,), -1.0, device="cuda")
    lb = torch.full((n,), -1.0, device="cuda")
    per_wg = -(-(-(-cap // tr)) // plan.grid) * tr
    dl = K.DeltaState(n, k, d, dp, 1, k * d + k + 1, x.device, plan.grid, cap=max(cap, 1024), pcap=max(per_wg, 64))
    K.assign_rr_ext(2, x, cap, dp, cb, cn, plan, cxn, lab, None, ub, lb, mc, tau, delta=dl, idx=idx, n_dev=cnt,
                    lab_in=clab)
    torch.cuda.synchronize()
    sel = torch.zeros(n, dtype=torch.bool, device="cuda")
    sel[cand.long()] = True
    assert torch.equal(lab[sel], ref_lab[sel]) and torch.equal(lab[~sel], old[~sel])
    assert torch.equal(ub[sel], ref_ub[sel]) and torch.equal(lb[sel], ref_lb[sel])
    assert bool((ub[~sel] == -1).all()) and bool((lb[~sel] == -1).all())
    assert int(dl.overflow.item()) == 0
    rows, olds = [], []
    for b in range(plan.grid):
        c = int(dl.wg_count[b].item())
        rows.append(dl.rows[b * dl.pcap: b * dl.pcap + c])
        olds.append(dl.old[b * dl.pcap: b * dl.pcap + c])
    rows = torch.cat(rows).long()
    olds = torch.cat(olds)
    changed = sel & (ref_lab != old)
    assert sorted(rows.tolist()) == sorted(torch.nonzero(changed).flatten().tolist())
    assert torch.equal(olds, old[rows])


@pytest.mark.gpu
@pytest.mark.parametrize("k,d", [(256, 256), (37, 100), (1, 16), (2, 512)])
def test_centre_stats_kernel_matches_torch(k, d):
    g = torch.Generator(device="cuda").manual_seed(k * d)
    dp = -(-d // 16) * 16
    cb = (torch.randn(k + 3, dp, device="cuda", generator=g) * 3).to(torch.bfloat16)
    cb[:, d:] = 0
    old = (cb.float() + torch.randn(k + 3, dp, device="cuda", generator=g) * 0.1).to(torch.bfloat16)
    old[:, d:] = 0
    if k > 2:
        cb[2] = cb[1]  # coincident centres: half distance 0 -> thr = -inf
    f = dict(cn=torch.zeros(k, dtype=torch.float64, device="cuda"),
             half=torch.zeros(k, dtype=torch.float64, device="cuda"),
             drift=torch.zeros(k, device="cuda"), thr=torch.zeros(k, device="cuda"), dmax=torch.zeros(3, device="cuda"),
             mc=torch.zeros(1, device="cuda"), c2=torch.zeros(1, device="cuda"),
             count=torch.full((1,), 7, dtype=torch.int32, device="cuda"),
             force=torch.ones(1, dtype=torch.int32, device="cuda"))
    mx = torch.tensor([1234.5], device="cuda")
    tau = 3e-5
    K.centre_stats(cb, old, k, d, mx, tau, f["cn"], f["half"], f["drift"], f["thr"], f["dmax"], f["mc"], f["c2"],
                   f["count"], f["force"])
    torch.cuda.synchronize()
    c = cb[:k, :d].double()
    o = old[:k, :d].double()
    cn = (c * c).sum(1)
    torch.testing.assert_close(f["cn"], cn, rtol=1e-12, atol=1e-9)
    dr = (c - o).pow(2).sum(1).sqrt()
    assert bool((f["drift"].double() >= dr * (1 - 1e-7)).all())
    torch.testing.assert_close(f["drift"].double(), dr, rtol=2e-6, atol=1e-7)
    top = torch.topk(dr, min(2, k)).values
    assert abs(float(f["dmax"][0]) - float(top[0])) <= 2e-6 * float(top[0]) + 1e-7
    if k > 1:
        assert abs(float(f["dmax"][1]) - float(top[-1])) <= 2e-6 * float(top[-1]) + 1e-7
        d2 = (cn[:, None] + cn[None, :] - 2 * c @ c.T).clamp(min=0)
        d2 = ((c[:, None, :] - c[None, :, :]) ** 2).sum(-1)
        d2.fill_diagonal_(float("inf"))
        half = 0.5 * d2.min(1).values.sqrt()
        sl = tau * (1234.5 + float(cn.max()))
        ref = torch.where(half > 0, (half - sl / (2 * half)) * (1 - 1e-6), torch.full_like(half, -float("inf")))
        torch.testing.assert_close(f["thr"].double(), ref, rtol=1e-6, atol=1e-6)
    else:
        assert bool(torch.isinf(f["thr"]).all())
    assert abs(float(f["mc"]) - float(cn.max())) <= 1e-6 * float(cn.max())
    assert abs(float(f["c2"]) - 2 * tau * (1234.5 + float(cn.max()))) <= 1e-6 * float(f["c2"])
    assert int(f["count"]) == 0 and int(f["force"]) == 0


@pytest.mark.gpu
@pytest.mark.parametrize("fp8,prune", [(False, True), (False, False), (True, True)])
def test_training_cost_exact_on_offset_data_gpu(fp8, prune):
    """trainingCost on data far from the origin (blobs + 300: |x|² ~ 2.3e7 per row against a cost of ~256
    per row) equals the f64 oracle Σ|x_i - c_lab(i)|² over the same labels and bf16 centres at 1e-9 (the
    expanded Σ(Q - 2c·S + n|c|²) form with f32 norms was off by percents here)."""
    n, d, k = 200_000, 256, 64
    x = _blobs(n, d, k, seed=17, scale=1.0, device="cuda", dtype=torch.float32) + 300.0
    x = x.clamp(-440, 440).to(torch.float8_e4m3fn) if fp8 else x.to(torch.bfloat16)
    eng = LloydEngine(x, d, k, prune=prune, use_graph=False)
    eng.set_centers(x[:k].float().double().cpu().numpy())
    for _ in range(4):
        eng.step()
    cb = (eng._pst.cb_old if eng._pdev else eng._cb_cost)[:k, :d].double()
    lab = eng.labels[:n].long()
    xf = x[:, :d].float().double()
    ref = float(((xf - cb[lab]) ** 2).sum())
    got = eng.training_cost()
    assert abs(got - ref) <= 1e-9 * ref, (got, ref)
    # the kernel alone, on the padded device matrix
    xm = eng.x
    c1 = float(K.cost_pass(xm, n, eng.dp, eng.labels, eng.cb).item())
    ref1 = float(((xf - eng.cb[:k, :d].double()[lab]) ** 2).sum())
    assert abs(c1 - ref1) <= 1e-9 * ref1


@pytest.mark.gpu
@pytest.mark.parametrize("scale", [0.5, 3.0])
def test_prune_backoff_same_fit(monkeypatch, scale):
    """After a pruned step goes over the candidate cap, the next steps skip the bounds pass and run full
    (CML_KMEANS_PRUNE_BACKOFF): the fit is bit for bit the one that retries the bounds every step."""
    n, d, k = 150_000, 128, 64
    x = _blobs(n, d, k, seed=5, scale=scale, device="cuda", dtype=torch.bfloat16)
    res = {}
    for nb in ("0", "2"):
        monkeypatch.setenv("CML_KMEANS_PRUNE_BACKOFF", nb)
        eng = LloydEngine(x, d, k)
        assert eng._pdev
        eng.track_prune = True
        eng.set_centers(eng.init_kmeans_parallel(seed=4))
        eng.fit(12, 0.0)
        res[nb] = (eng.centers.cpu().numpy(), eng.labels[:n].clone(), eng.training_cost(), eng.prune_history())
    (c0, l0, t0, h0), (c1, l1, t1, h1) = res["0"], res["2"]
    assert np.array_equal(c0, c1) and torch.equal(l0, l1) and t0 == t1
    if scale < 1.0:  # overlapping blobs: the backed-off steps are all full
        assert sum(1 for f, _ in h1 if f) >= sum(1 for f, _ in h0 if f)
