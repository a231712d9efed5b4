"""Weighted KMeans (Spark's weightCol, KMeans.scala runAlgorithm: centre = Σw·x / Σw, trainingCost =
Σ w·d², k-means|| candidates weighted by their rows' summed weight) against a numpy weighted Lloyd,
the unit-weight ≡ unweighted identity (bit for bit), integer weights ≡ duplicated rows, zero weights ≡
dropped rows, weight validation, W=2 gloo ranks, and (GPU) device fit == CPU fit bit for bit."""
import json
import os
import socket

import numpy as np
import pandas as pd
import pytest
import torch
import torch.multiprocessing as mp

from clustermachinelearningforhospitalnetworks_apache_spark_amd.models.kmeans import LloydEngine


def numpy_weighted_lloyd(x, w, c, iters):
    cost = None
    for _ in range(iters):
        d = ((x[:, None, :] - c[None]) ** 2).sum(2)
        lab = d.argmin(1)
        cost = float((d[np.arange(len(x)), lab] * w).sum())
        new = c.copy()
        for j in range(c.shape[0]):
            m = lab == j
            if w[m].sum() > 0:
                new[j] = (x[m] * w[m, None]).sum(0) / w[m].sum()
        c = new
    return c, cost


def _blobs(n=1200, d=4, seed=0):
    rs = np.random.RandomState(seed)
    cen = rs.randn(5, d) * 5
    return cen[rs.randint(0, 5, n)] + rs.randn(n, d), rs


def test_weighted_engine_matches_numpy():
    x, rs = _blobs()
    w = rs.uniform(0.0, 3.0, len(x))
    init = x[:6].copy()
    eng = LloydEngine(torch.as_tensor(x), 4, 6, weights=torch.as_tensor(w))
    eng.set_centers(init)
    for _ in range(6):
        eng.step()
    want, cost = numpy_weighted_lloyd(x, w, init, 6)
    np.testing.assert_allclose(eng.centers.numpy(), want, rtol=1e-11, atol=1e-11)
    assert eng.training_cost() == pytest.approx(cost, rel=1e-11)


def test_integer_weights_equal_duplicated_rows():
    x, rs = _blobs(600)
    reps = rs.randint(1, 4, len(x))
    init = x[:5].copy()
    a = LloydEngine(torch.as_tensor(x), 4, 5, weights=torch.as_tensor(reps.astype(float)))
    b = LloydEngine(torch.as_tensor(np.repeat(x, reps, 0)), 4, 5)
    for e in (a, b):
        e.set_centers(init)
        e.fit(10, 0.0)
    np.testing.assert_allclose(a.centers.numpy(), b.centers.numpy(), rtol=1e-12, atol=1e-12)
    assert a.training_cost() == pytest.approx(b.training_cost(), rel=1e-12)


def test_zero_weights_equal_dropped_rows():
    x, rs = _blobs(800)
    w = (rs.rand(len(x)) < 0.7).astype(float)
    init = x[w > 0][:5].copy()
    a = LloydEngine(torch.as_tensor(x), 4, 5, weights=torch.as_tensor(w))
    b = LloydEngine(torch.as_tensor(x[w > 0]), 4, 5)
    for e in (a, b):
        e.set_centers(init)
        e.fit(8, 0.0)
    np.testing.assert_allclose(a.centers.numpy(), b.centers.numpy(), rtol=1e-12, atol=1e-12)


def _frame(spark, x, w=None):
    from clustermachinelearningforhospitalnetworks_apache_spark_amd.ml.feature import VectorAssembler
    pdf = pd.DataFrame(x, columns=[f"f{i}" for i in range(x.shape[1])])
    if w is not None:
        pdf["w"] = w
    df = spark.createDataFrame(pdf)
    return VectorAssembler(inputCols=[f"f{i}" for i in range(x.shape[1])], outputCol="features").transform(df)


@pytest.fixture(scope="module")
def spark():
    from clustermachinelearningforhospitalnetworks_apache_spark_amd.sql import SparkSession
    return SparkSession.builder.master("local[1]").getOrCreate()


def test_unit_weights_equal_unweighted_fit(spark):
    from clustermachinelearningforhospitalnetworks_apache_spark_amd.ml.clustering import KMeans
    x, _ = _blobs(1500)
    f = _frame(spark, x, np.ones(len(x)))
    m1 = KMeans(k=5, seed=3, weightCol="w").fit(f)
    m0 = KMeans(k=5, seed=3).fit(f)
    assert np.array_equal(np.array(m1.clusterCenters()), np.array(m0.clusterCenters()))
    assert m1.summary.trainingCost == m0.summary.trainingCost
    assert m1.summary.clusterSizes == m0.summary.clusterSizes


def test_weights_move_centres_and_validate(spark):
    from clustermachinelearningforhospitalnetworks_apache_spark_amd.ml.clustering import KMeans
    x = np.array([[0.0], [1.0], [10.0], [11.0]])
    f = _frame(spark, x, [3.0, 1.0, 1.0, 0.0])
    m = KMeans(k=2, seed=1, weightCol="w", initMode="random").fit(f)
    cs = sorted(c[0] for c in m.clusterCenters())
    assert cs == pytest.approx([0.25, 10.0])
    assert m.summary.trainingCost == pytest.approx(3 * 0.25 ** 2 + 0.75 ** 2)
    assert sorted(m.summary.clusterSizes) == [2, 2]  # row counts, as Spark's summary
    with pytest.raises(ValueError):
        KMeans(k=2, weightCol="w").fit(_frame(spark, x, [1.0, -1.0, 1.0, 1.0]))
    with pytest.raises(ValueError):
        KMeans(k=2, weightCol="w").fit(_frame(spark, x, [1.0, np.inf, 1.0, 1.0]))


# ------------------------------------------------------------------------------------------ W=2 gloo

def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _workload(out):
    from clustermachinelearningforhospitalnetworks_apache_spark_amd.ml.clustering import KMeans
    from clustermachinelearningforhospitalnetworks_apache_spark_amd.sql import SparkSession
    spark = SparkSession.builder.master("local[1]").getOrCreate()
    x, rs = _blobs(1000, seed=5)
    w = rs.uniform(0.1, 2.0, len(x))
    m = KMeans(k=4, seed=9, weightCol="w", maxIter=15).fit(_frame(spark, x, w))
    if spark._comm.rank == 0:
        with open(out, "w") as fh:
            json.dump({"c": np.array(m.clusterCenters()).tolist(), "cost": m.summary.trainingCost}, fh)
    spark.stop()


def _rank_main(rank, world, port, out):
    os.environ.update({"RANK": str(rank), "WORLD_SIZE": str(world), "LOCAL_RANK": str(rank),
                       "MASTER_ADDR": "127.0.0.1", "MASTER_PORT": str(port), "CML_FORCE_CPU": "1"})
    torch.set_num_threads(1)
    _workload(out)


def test_weighted_two_ranks_match_one(tmp_path):
    o1, o2 = str(tmp_path / "w1.json"), str(tmp_path / "w2.json")
    for key in ("RANK", "WORLD_SIZE", "LOCAL_RANK"):
        os.environ.pop(key, None)
    _workload(o1)
    mp.start_processes(_rank_main, args=(2, _free_port(), o2), nprocs=2, join=True, start_method="spawn")
    r1, r2 = (json.load(open(p)) for p in (o1, o2))
    np.testing.assert_allclose(r2["c"], r1["c"], rtol=1e-10, atol=1e-10)
    assert r2["cost"] == pytest.approx(r1["cost"], rel=1e-10)


@pytest.mark.gpu
def test_weighted_gpu_fit_equals_cpu_fit():
    x, rs = _blobs(5000, d=6, seed=11)
    w = rs.uniform(0.0, 4.0, len(x))
    res = []
    for dev in ("cpu", "cuda"):
        xt = torch.as_tensor(x, device=dev)
        eng = LloydEngine(xt, 6, 7, weights=torch.as_tensor(w, device=dev))
        init = eng.init_kmeans_parallel(seed=4)
        eng.set_centers(init)
        eng.fit(12, 0.0)
        res.append((init, eng.centers.cpu().numpy(), eng.training_cost()))
    assert np.array_equal(res[0][0], res[1][0])
    assert np.array_equal(res[0][1], res[1][1])
    assert res[0][2] == res[1][2]


def _bad_weight_rank(rank, world, port, out):
    os.environ.update({"RANK": str(rank), "WORLD_SIZE": str(world), "LOCAL_RANK": str(rank),
                       "MASTER_ADDR": "127.0.0.1", "MASTER_PORT": str(port), "CML_FORCE_CPU": "1"})
    torch.set_num_threads(1)
    from clustermachinelearningforhospitalnetworks_apache_spark_amd.ml.clustering import KMeans
    from clustermachinelearningforhospitalnetworks_apache_spark_amd.sql import SparkSession
    spark = SparkSession.builder.master("local[1]").getOrCreate()
    x, rs = _blobs(400, seed=6)
    w = rs.uniform(0.1, 2.0, len(x))
    w[-1] = -1.0  # one bad weight: it lands on exactly one rank's shard
    try:
        KMeans(k=3, seed=1, weightCol="w", maxIter=3).fit(_frame(spark, x, w))
        msg = "no error"
    except ValueError as e:
        msg = str(e)
    with open(f"{out}.{rank}", "w") as fh:
        fh.write(msg)
    spark.stop()


def test_bad_weight_on_one_rank_raises_on_every_rank(tmp_path):
    """the weight check is agreed across ranks, so every rank raises the same ValueError at
    once instead of the clean ranks blocking in the init collectives until the watchdog fires."""
    out = str(tmp_path / "bad")
    mp.start_processes(_bad_weight_rank, args=(2, _free_port(), out), nprocs=2, join=True, start_method="spawn")
    for r in range(2):
        assert "finite and non-negative" in open(f"{out}.{r}").read()
