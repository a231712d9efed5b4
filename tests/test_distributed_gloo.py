"""Distributed correctness without GPUs: the same SPMD code on W gloo ranks must match
W=1 (row ids, counter-based randomness and fixed-order reductions make it GPU-count
invariant). Mirrors the RCCL path: only the backend differs."""
import json
import os
import socket

import numpy as np
import pandas as pd
import pytest
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _workload(out_path, rank, master="local[1]"):
    import torch
    from clustermachinelearningforhospitalnetworks_apache_spark_amd.ml.classification import LogisticRegression
    from clustermachinelearningforhospitalnetworks_apache_spark_amd.ml.clustering import KMeans
    from clustermachinelearningforhospitalnetworks_apache_spark_amd.ml.evaluation import RegressionEvaluator
    from clustermachinelearningforhospitalnetworks_apache_spark_amd.ml.feature import StandardScaler, VectorAssembler
    from clustermachinelearningforhospitalnetworks_apache_spark_amd.ml.regression import (DecisionTreeRegressor,
                                                                                            LinearRegression,
                                                                                            RandomForestRegressor)
    from clustermachinelearningforhospitalnetworks_apache_spark_amd.sql import SparkSession
    from clustermachinelearningforhospitalnetworks_apache_spark_amd.sql import functions as F
    spark = SparkSession.builder.master(master).getOrCreate()
    rs = np.random.RandomState(0)
    n = 3001
    X = rs.randn(n, 4) * [1, 2, 3, 4] + [0, 1, 2, 3]
    y = X @ [0.5, -1, 0.25, 2] + 1 + rs.randn(n) * 0.3
    pdf = pd.DataFrame(X, columns=list("abcd"))
    pdf["y"] = y
    pdf["g"] = [f"k{i % 5}" for i in range(n)]
    df = spark.createDataFrame(pdf)
    f = VectorAssembler(inputCols=list("abcd"), outputCol="features").transform(df)
    tr, te = f.randomSplit([0.7, 0.3], seed=42)
    res = {"world": spark.world_size, "count": f.count(), "train": tr.count(), "gpu": master != "local[1]",
           "train_ids": sorted(int(r.a * 1e9) for r in tr.select("a").collect())[:50]}
    lr = LinearRegression(featuresCol="features", labelCol="y").fit(tr)
    res["lr"] = lr.coefficients.toArray().tolist() + [lr.intercept]
    res["rmse"] = RegressionEvaluator(labelCol="y").evaluate(lr.transform(te))
    sc = StandardScaler(inputCol="features", outputCol="s", withMean=True).fit(f)
    res["std"] = sc.std.toArray().tolist()
    dt = DecisionTreeRegressor(featuresCol="features", labelCol="y").fit(tr)
    res["dt_imp"] = dt.featureImportances.toArray().tolist()
    res["dt_nodes"] = dt.numNodes
    rf = RandomForestRegressor(featuresCol="features", labelCol="y", numTrees=4).fit(tr)
    res["rf_imp"] = rf.featureImportances.toArray().tolist()
    from clustermachinelearningforhospitalnetworks_apache_spark_amd.ml.classification import GBTClassifier
    from clustermachinelearningforhospitalnetworks_apache_spark_amd.ml.regression import GBTRegressor
    gb = GBTRegressor(featuresCol="features", labelCol="y", maxIter=5).fit(tr)
    res["gbt"] = gb.featureImportances.toArray().tolist() + [RegressionEvaluator(labelCol="y").evaluate(
        gb.transform(te))]
    gbl = f.withColumn("label", F.when(F.col("y") > 1.0, 1).otherwise(0)).withColumn("v", F.col("d") > 5.0)
    gc = GBTClassifier(maxIter=30, stepSize=0.5, validationIndicatorCol="v").fit(gbl)
    res["gbtc"] = [gc.getNumTrees] + gc.evaluateEachIteration(gbl)
    from clustermachinelearningforhospitalnetworks_apache_spark_amd.ml.feature import PCA, QuantileDiscretizer
    from clustermachinelearningforhospitalnetworks_apache_spark_amd.ml.stat import Correlation
    res["corr"] = [Correlation.corr(f, "features", m).head()[0].toArray().tolist() for m in ("pearson", "spearman")]
    res["pca"] = PCA(k=2, inputCol="features", outputCol="p").fit(f).explainedVariance.toArray().tolist()
    from clustermachinelearningforhospitalnetworks_apache_spark_amd.ml.regression import GeneralizedLinearRegression
    pois = f.withColumn("cnt", F.when(F.col("y") > 1.0, 3).otherwise(1))
    glr = GeneralizedLinearRegression(family="poisson", labelCol="cnt").fit(pois)
    res["glr"] = glr.coefficients.toArray().tolist() + [glr.intercept, glr.summary.deviance]
    from clustermachinelearningforhospitalnetworks_apache_spark_amd.ml.classification import NaiveBayes
    nbm = NaiveBayes(modelType="gaussian").fit(f.withColumn("label", F.when(F.col("y") > 1.0, 1).otherwise(0)))
    res["nb"] = np.r_[nbm.theta.toArray().ravel(), nbm.sigma.toArray().ravel(), nbm.pi.toArray()].tolist()
    res["qd"] = QuantileDiscretizer(numBuckets=4, inputCol="b", outputCol="q").fit(f).getSplits()[1:-1]
    km = KMeans(k=3, seed=5, maxIter=10).fit(f)
    res["km"] = np.stack(km.clusterCenters()).tolist()
    res["km_cost"] = km.summary.trainingCost
    lab = f.withColumn("label", F.when(F.col("y") > 1.0, 1).otherwise(0))
    lg = LogisticRegression(maxIter=50).fit(lab)
    res["logreg"] = lg.coefficients.toArray().tolist() + [lg.intercept]
    g = spark.createDataFrame(pdf).groupBy("g").agg(F.sum("y").alias("s")).orderBy("g").collect()
    res["groupby"] = [(r.g, r.s) for r in g]
    res["sql"] = spark.createDataFrame(pdf).filter("a > 0 AND b < 2").count()
    from clustermachinelearningforhospitalnetworks_apache_spark_amd.sql import aggregate_fast as _AF
    rich = lambda: [list(r) for r in spark.createDataFrame(pdf.assign(h=(pdf.index * 13) % 97)).groupBy(  # noqa: E731
        "g", "h").agg(F.sum("y"), F.avg("a"), F.stddev("b"), F.min("c"), F.max("d"), F.count("*"),
                      F.first("a"), F.last("b")).collect()]
    res["agg_dev"] = rich()
    _AF.ENABLED = False
    res["agg_py"] = rich()
    _AF.ENABLED = True
    from clustermachinelearningforhospitalnetworks_apache_spark_amd.ml.feature import (Imputer, OneHotEncoder,
                                                                                         StringIndexer)
    from clustermachinelearningforhospitalnetworks_apache_spark_amd.ml.tuning import CrossValidator, ParamGridBuilder
    dte = DecisionTreeRegressor(featuresCol="features", labelCol="y")
    cv = CrossValidator(estimator=dte, estimatorParamMaps=ParamGridBuilder().addGrid(dte.maxDepth, [2, 4]).build(),
                        evaluator=RegressionEvaluator(labelCol="y"), numFolds=3, seed=9).fit(f)
    res["cv"] = cv.avgMetrics
    gi = StringIndexer(inputCol="g", outputCol="gi").fit(df).transform(df)
    res["ohe"] = OneHotEncoder(inputCol="gi", outputCol="gv").fit(gi).categorySizes
    holes = spark.createDataFrame(pdf.assign(a=pdf["a"].where(pdf.index % 7 != 0)))
    res["imp"] = [Imputer(strategy=s, inputCol="a", outputCol="ai").fit(holes).surrogates[0]
                  for s in ("mean", "median", "mode")]
    from clustermachinelearningforhospitalnetworks_apache_spark_amd.sql import Window
    w = Window.partitionBy("g").orderBy("a")
    wd = spark.createDataFrame(pdf).select("g", "a", F.row_number().over(w).alias("rn"),
                                           F.sum("y").over(w.rowsBetween(-3, 0)).alias("s"),
                                           F.lag("b", 1).over(w).alias("lb")).orderBy("g", "a").collect()
    res["win"] = [[r.g, r.rn, r.s, r.lb] for r in wd][:300]
    # relational shuffles: sort (all-to-all exchange), dedup, joins, repartition; strings
    # dictionary-encoded (per-rank dictionaries merged by the shuffles)
    from clustermachinelearningforhospitalnetworks_apache_spark_amd.sql import builder as _B
    _B.DICT_MIN_ROWS = 64
    rel = spark.createDataFrame(pdf.assign(k=(pdf.index * 7) % 13, q=pdf["g"].where(pdf.index % 11 != 0)))
    srt = rel.orderBy(F.col("q").desc_nulls_first(), "k", F.col("a").desc())
    res["sort_rows"] = [[r.q, r.k, r.a] for r in srt.select("q", "k", "a").collect()]
    res["dedup"] = [[r.q, r.k] for r in rel.select("q", "k").distinct().collect()]
    dim = spark.createDataFrame(pd.DataFrame({"k": list(range(0, 15, 2)) + [4],
                                              "kname": [f"n{i}" for i in range(9)]}))
    res["join"] = {h: [[r.a, r.k, r.kname] for r in rel.join(dim, "k", h).select("a", "k", "kname").collect()]
                   for h in ("inner", "left", "right", "full")}
    res["semi"] = [rel.join(dim, "k", h).count() for h in ("leftsemi", "leftanti")]
    rel.createOrReplaceTempView("rel")
    dim.createOrReplaceTempView("dim")
    res["sql_join"] = [[r.a, r.kname] for r in spark.sql(
        "SELECT rel.a, dim.kname FROM rel JOIN dim ON rel.k = dim.k WHERE rel.a > 0").collect()]
    rp = rel.filter("a > 1").repartition(4)
    res["repart"] = [[r.a, r.k] for r in rp.select("a", "k").collect()]
    kq = rel.select("k", "q")
    other = spark.createDataFrame(pdf.assign(k=(pdf.index * 5) % 13, q=pdf["g"]).iloc[::3][["k", "q"]])
    res["setops"] = [[tuple(r) for r in getattr(kq, m)(other).collect()]
                     for m in ("intersect", "intersectAll", "subtract", "exceptAll")]
    assert type(rel._cols["q"]).__name__ == "DictColumnData"
    aip = rel.groupBy("q", "k").applyInPandas(
        lambda g: pd.DataFrame({"q": [g.q.iloc[0]], "k": [int(g.k.iloc[0])], "n": [len(g)], "s": [float(g.a.sum())]}),
        "q string, k long, n long, s double").collect()
    res["aip"] = sorted([[r.q, r.k, r.n, round(r.s, 9)] for r in aip], key=str)
    _B.DICT_MIN_ROWS = 32768
    from clustermachinelearningforhospitalnetworks_apache_spark_amd.ml.clustering import BisectingKMeans
    res["bkm"] = np.stack(BisectingKMeans(k=4, seed=2).fit(f).clusterCenters()).tolist()
    # round-2 additions: device aggregates merged across ranks, selectors, SVM, GMM, AFT, isotonic
    st = spark.createDataFrame(pdf).select(F.skewness("a"), F.kurtosis("b"), F.corr("a", "y"), F.covar_samp("c", "d"),
                                           F.median("d"), F.percentile("a", [0.25, 0.75])).collect()[0]
    res["stat_aggs"] = [st[0], st[1], st[2], st[3], st[4]] + list(st[5])
    from clustermachinelearningforhospitalnetworks_apache_spark_amd.ml.stat import Summarizer
    sm = f.select(Summarizer.metrics("mean", "variance", "max").summary(F.col("features"))).collect()[0][0]
    res["summ"] = np.r_[sm.mean.toArray(), sm.variance.toArray(), sm.max.toArray()].tolist()
    from clustermachinelearningforhospitalnetworks_apache_spark_amd.ml.classification import LinearSVC
    from clustermachinelearningforhospitalnetworks_apache_spark_amd.ml.clustering import GaussianMixture
    from clustermachinelearningforhospitalnetworks_apache_spark_amd.ml.feature import RobustScaler
    from clustermachinelearningforhospitalnetworks_apache_spark_amd.ml.regression import (AFTSurvivalRegression,
                                                                                            IsotonicRegression)
    sv = LinearSVC(maxIter=30, regParam=0.01).fit(lab)
    res["svc"] = sv.coefficients.toArray().tolist() + [sv.intercept]
    res["gmm"] = GaussianMixture(k=2, seed=4, maxIter=10).fit(f).weights
    res["robust"] = RobustScaler(inputCol="features", outputCol="r").fit(f).range.toArray().tolist()
    surv = f.withColumn("t", F.exp(F.col("a") * 0.3)).withColumn("cens", F.when(F.col("b") > 0.0, 1.0).otherwise(0.0))
    aft = AFTSurvivalRegression(labelCol="t", censorCol="cens", maxIter=30).fit(surv)
    res["aft"] = aft.coefficients.toArray().tolist() + [aft.intercept, aft.scale]
    res["iso"] = IsotonicRegression(labelCol="y", featureIndex=3).fit(f).predictions.toArray().tolist()[:50]
    # LDA (online VB: counter-based mini-batches and γ init) and power iteration clustering
    from clustermachinelearningforhospitalnetworks_apache_spark_amd.ml.clustering import (LDA,
                                                                                          PowerIterationClustering)
    from clustermachinelearningforhospitalnetworks_apache_spark_amd.ml.feature import VectorAssembler as VA
    cnt = pd.DataFrame(np.floor(np.abs(pdf[["a", "b", "c", "d"]].to_numpy()) * 3), columns=list("pqrs"))
    cdf = VA(inputCols=list("pqrs"), outputCol="features").transform(spark.createDataFrame(cnt))
    lda = LDA(k=2, maxIter=5, seed=3, subsamplingRate=0.3).fit(cdf)
    res["lda"] = lda.topicsMatrix().toArray().ravel().tolist()
    edges = [(i, j, 1.0 if i < 6 else 3.0) for b in (0, 6) for i in range(b, b + 6) for j in range(i + 1, b + 6)]
    edges.append((5, 6, 0.01))
    res["pic"] = sorted([r.id, r.cluster] for r in PowerIterationClustering(k=2, weightCol="weight").assignClusters(
        spark.createDataFrame(edges, "src long, dst long, weight double")).collect())
    # stateful streaming: a complete-mode aggregation over CSV uploads planned by rank 0
    sdir = os.path.join(os.path.dirname(out_path), f"stream_w{spark.world_size}")
    if rank == 0:
        os.makedirs(sdir, exist_ok=True)
        for i in range(3):
            part = pdf.iloc[i * 200:(i + 1) * 200]
            pd.DataFrame({"hospital_id": part["g"], "event_time": "2025-04-01 10:00:00", "v": part["y"]}).to_csv(
                os.path.join(sdir, f"up_{i}.csv"), index=False)
    spark._comm.barrier()
    got = []
    q = (spark.readStream.option("header", True).schema("hospital_id STRING, event_time TIMESTAMP, v DOUBLE")
         .csv(sdir).groupBy("hospital_id").agg(F.count("*").alias("n"), F.sum("v").alias("s"))
         .writeStream.outputMode("complete")
         .foreachBatch(lambda d, b: got.append(sorted([r.hospital_id, r.n, r.s] for r in d.collect())))
         .option("checkpointLocation", sdir + "_ck").trigger(availableNow=True).start())
    q.awaitTermination()
    res["stream_agg"] = got[-1]
    if rank == 0:
        with open(out_path, "w") as fh:
            json.dump(res, fh)
    spark.stop()


def _rank_main(rank, world, port, out_path, gpu=False):
    os.environ.update({"RANK": str(rank), "WORLD_SIZE": str(world), "LOCAL_RANK": str(rank),
                       "MASTER_ADDR": "127.0.0.1", "MASTER_PORT": str(port)})
    if gpu:  # every rank on the one visible GPU, collectives over gloo (RCCL needs a GPU per rank)
        os.environ["CML_COMM_BACKEND"] = "gloo"
    else:
        os.environ["CML_FORCE_CPU"] = "1"
    import torch
    torch.set_num_threads(1)
    _workload(out_path, rank, "mi355x" if gpu else "local[1]")


def _run(world, tmp_path, gpu=False):
    out = str(tmp_path / f"res_w{world}{'_gpu' if gpu else ''}.json")
    if world == 1:
        for k in ("RANK", "WORLD_SIZE", "LOCAL_RANK"):
            os.environ.pop(k, None)
        _workload(out, 0, "mi355x" if gpu else "local[1]")
    else:
        # the free port can be taken by a concurrent test between probing and binding (pytest -n):
        # one fresh-port retry; a real mismatch fails deterministically on both attempts
        for attempt in range(2):
            try:
                mp.start_processes(_rank_main, args=(world, _free_port(), out, gpu), nprocs=world, join=True,
                                   start_method="spawn")
                break
            except mp.ProcessRaisedException as e:
                if attempt == 1 or "address already in use" not in str(e).lower() and "EADDRINUSE" not in str(e):
                    raise
    with open(out) as fh:
        return json.load(fh)


def _check_invariant(r1, rw, world):
    assert rw["world"] == world and r1["world"] == 1
    assert rw["count"] == r1["count"] and rw["train"] == r1["train"]
    assert rw["train_ids"] == r1["train_ids"]
    np.testing.assert_allclose(rw["lr"], r1["lr"], rtol=1e-9, atol=1e-11)
    assert abs(rw["rmse"] - r1["rmse"]) < 1e-9
    np.testing.assert_allclose(rw["std"], r1["std"], rtol=1e-10)
    np.testing.assert_allclose(rw["dt_imp"], r1["dt_imp"], rtol=1e-9, atol=1e-12)
    assert rw["dt_nodes"] == r1["dt_nodes"]
    np.testing.assert_allclose(rw["rf_imp"], r1["rf_imp"], rtol=1e-9, atol=1e-12)
    np.testing.assert_allclose(rw["gbt"], r1["gbt"], rtol=1e-9, atol=1e-12)
    assert rw["gbtc"][0] == r1["gbtc"][0]
    np.testing.assert_allclose(rw["gbtc"], r1["gbtc"], rtol=1e-9)
    np.testing.assert_allclose(rw["corr"], r1["corr"], rtol=1e-9, atol=1e-12)
    np.testing.assert_allclose(rw["pca"], r1["pca"], rtol=1e-9)
    assert rw["qd"] == r1["qd"]
    np.testing.assert_allclose(rw["nb"], r1["nb"], rtol=1e-9, atol=1e-12)
    np.testing.assert_allclose(rw["glr"], r1["glr"], rtol=1e-9, atol=1e-12)
    np.testing.assert_allclose(rw["km"], r1["km"], rtol=1e-9, atol=1e-9)
    assert abs(rw["km_cost"] - r1["km_cost"]) < 1e-6 * r1["km_cost"]
    np.testing.assert_allclose(rw["logreg"], r1["logreg"], rtol=1e-6, atol=1e-8)
    assert [g for g, _ in rw["groupby"]] == [g for g, _ in r1["groupby"]]
    np.testing.assert_allclose([s for _, s in rw["groupby"]], [s for _, s in r1["groupby"]], rtol=1e-12)
    assert rw["sql"] == r1["sql"]
    np.testing.assert_allclose(rw["cv"], r1["cv"], rtol=1e-9)
    assert rw["ohe"] == r1["ohe"] == [5]
    np.testing.assert_allclose(rw["imp"], r1["imp"], rtol=1e-12)
    assert [x[:2] for x in rw["win"]] == [x[:2] for x in r1["win"]]
    np.testing.assert_allclose([x[2] for x in rw["win"]], [x[2] for x in r1["win"]], rtol=1e-12)
    assert [x[3] for x in rw["win"]] == [x[3] for x in r1["win"]]
    for r in (r1, rw):  # device merge == Python merge (exact on CPU; GPU index_add sums are atomics)
        assert [x[:2] + x[7:8] for x in r["agg_dev"]] == [x[:2] + x[7:8] for x in r["agg_py"]]
        np.testing.assert_allclose([x[2:7] + x[8:] for x in r["agg_dev"]], [x[2:7] + x[8:] for x in r["agg_py"]],
                                   rtol=0 if not r.get("gpu") else 1e-12)
    for key in ("sort_rows", "dedup", "join", "semi", "sql_join", "repart", "setops", "aip"):
        assert rw[key] == r1[key], key
    np.testing.assert_allclose(rw["bkm"], r1["bkm"], rtol=1e-9, atol=1e-9)
    np.testing.assert_allclose(rw["stat_aggs"], r1["stat_aggs"], rtol=1e-9)
    np.testing.assert_allclose(rw["summ"], r1["summ"], rtol=1e-10)
    np.testing.assert_allclose(rw["robust"], r1["robust"], rtol=1e-12)
    np.testing.assert_allclose(rw["iso"], r1["iso"], rtol=1e-10)
    np.testing.assert_allclose(rw["svc"], r1["svc"], rtol=1e-5, atol=1e-7)
    np.testing.assert_allclose(rw["aft"], r1["aft"], rtol=1e-5, atol=1e-7)
    np.testing.assert_allclose(rw["gmm"], r1["gmm"], rtol=1e-6)
    np.testing.assert_allclose(rw["lda"], r1["lda"], rtol=1e-6)
    assert rw["pic"] == r1["pic"]
    assert [x[:2] for x in rw["stream_agg"]] == [x[:2] for x in r1["stream_agg"]]
    np.testing.assert_allclose([x[2] for x in rw["stream_agg"]], [x[2] for x in r1["stream_agg"]], rtol=1e-12)
    assert sum(x[1] for x in r1["stream_agg"]) == 600


@pytest.mark.parametrize("world", [2, 3, 4, 8])
def test_spmd_results_invariant_to_world_size(tmp_path, world):
    _check_invariant(_run(1, tmp_path), _run(world, tmp_path), world)


@pytest.mark.gpu
def test_spmd_gpu_ranks_invariant_to_world_size(tmp_path):
    """The same workload with GPU-resident shards and the HIP kernels: 2 ranks sharing the one
    visible MI355X (gloo collectives) against 1 rank."""
    _check_invariant(_run(1, tmp_path, gpu=True), _run(2, tmp_path, gpu=True), 2)
