"""A rank that holds no rows (Spark partitions can be empty: ref.py:57 cluster, ref.py:128 window
filter) must not change any result: k-means|| + Lloyd (full and pruned steps), trees, linear models,
evaluators, the scaler and a streaming micro-batch with fewer files than ranks, on W=3 gloo ranks
where rank 2's shard is filtered to nothing, against W=1."""
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


def _workload(out_path, rank, tmpdir):
    import torch
    from clustermachinelearningforhospitalnetworks_apache_spark_amd.ml.classification import (
        DecisionTreeClassifier, LogisticRegression, RandomForestClassifier)
    from clustermachinelearningforhospitalnetworks_apache_spark_amd.ml.clustering import KMeans
    from clustermachinelearningforhospitalnetworks_apache_spark_amd.ml.evaluation import (
        MulticlassClassificationEvaluator, RegressionEvaluator)
    from clustermachinelearningforhospitalnetworks_apache_spark_amd.ml.feature import StandardScaler, VectorAssembler
    from clustermachinelearningforhospitalnetworks_apache_spark_amd.ml.regression import (
        DecisionTreeRegressor, LinearRegression, RandomForestRegressor)
    from clustermachinelearningforhospitalnetworks_apache_spark_amd.sql import SparkSession
    from clustermachinelearningforhospitalnetworks_apache_spark_amd.sql import functions as F
    spark = SparkSession.builder.master("local[1]").getOrCreate()
    rs = np.random.RandomState(3)
    n = 1500
    cen = rs.randn(5, 4) * 6
    X = cen[rs.randint(0, 5, n)] + rs.randn(n, 4)
    X = X[np.argsort(X[:, 0])]  # sorted by a: the last contiguous shard is the largest a
    pdf = pd.DataFrame(X, columns=list("abcd"))
    pdf["y"] = X @ [0.5, -1, 0.25, 2] + 1 + rs.randn(n) * 0.3
    pdf["label"] = (pdf["y"] > pdf["y"].median()).astype(float)
    thr = float(np.quantile(X[:, 0], 0.6))
    df = spark.createDataFrame(pdf).filter(F.col("a") < thr)
    local_rows = spark._comm.allgather_object(int(df._nrows))
    f = VectorAssembler(inputCols=list("abcd"), outputCol="features").transform(df)
    res = {"world": spark.world_size, "count": f.count(), "local_rows": local_rows}
    for prune in ("false", "true"):
        spark.conf.set("cml.ml.kmeans.prune", prune)
        km = KMeans(k=5, seed=7, maxIter=15).fit(f)
        res[f"km_{prune}"] = np.array(km.clusterCenters()).tolist()
        res[f"km_cost_{prune}"] = km.summary.trainingCost
        res[f"km_sizes_{prune}"] = km.summary.clusterSizes
    spark.conf.unset("cml.ml.kmeans.prune")
    lr = LinearRegression(labelCol="y").fit(f)
    res["lr"] = lr.coefficients.toArray().tolist() + [lr.intercept]
    res["rmse"] = RegressionEvaluator(labelCol="y").evaluate(lr.transform(f))
    res["std"] = StandardScaler(inputCol="features", outputCol="s").fit(f).std.toArray().tolist()
    dt = DecisionTreeRegressor(labelCol="y").fit(f)
    res["dt"] = dt.featureImportances.toArray().tolist() + [dt.numNodes]
    rf = RandomForestRegressor(labelCol="y", numTrees=3).fit(f)
    res["rf"] = rf.featureImportances.toArray().tolist()
    dtc = DecisionTreeClassifier(labelCol="label").fit(f)
    res["acc"] = MulticlassClassificationEvaluator(labelCol="label", metricName="accuracy").evaluate(
        dtc.transform(f))
    rfc = RandomForestClassifier(labelCol="label", numTrees=3).fit(f)
    res["rfc"] = rfc.featureImportances.toArray().tolist()
    lg = LogisticRegression(labelCol="label", maxIter=20).fit(f)
    res["logreg"] = lg.coefficients.toArray().tolist() + [lg.intercept]
    # streaming: one micro-batch of 2 files on 3 ranks (a rank without files)
    src = os.path.join(tmpdir, "in")
    if rank == 0:
        os.makedirs(src, exist_ok=True)
        for i in range(2):
            pdf.iloc[i * 10:(i + 1) * 10][["a", "b", "y"]].to_csv(os.path.join(src, f"p{i}.csv"), index=False)
    spark._comm.barrier()
    from clustermachinelearningforhospitalnetworks_apache_spark_amd.sql import types as T
    schema = T.StructType([T.StructField("a", T.DoubleType()), T.StructField("b", T.DoubleType()),
                           T.StructField("y", T.DoubleType())])
    seen = []
    q = (spark.readStream.option("header", True).schema(schema).csv(src).writeStream
         .foreachBatch(lambda bdf, bid: seen.append((bid, bdf.count(), bdf.agg(F.sum("y")).collect()[0][0])))
         .option("checkpointLocation", os.path.join(tmpdir, "ck")).trigger(availableNow=True).start())
    q.awaitTermination()
    res["stream"] = seen
    if rank == 0:
        with open(out_path, "w") as fh:
            json.dump(res, fh)
    spark.stop()


def _rank_main(rank, world, port, out_path, tmpdir):
    os.environ.update({"RANK": str(rank), "WORLD_SIZE": str(world), "LOCAL_RANK": str(rank),
                       "MASTER_ADDR": "127.0.0.1", "MASTER_PORT": str(port), "CML_FORCE_CPU": "1"})
    import torch
    torch.set_num_threads(1)
    _workload(out_path, rank, tmpdir)


def _run(world, tmp_path):
    out = str(tmp_path / f"res_w{world}.json")
    tmpdir = str(tmp_path / f"w{world}")
    os.makedirs(tmpdir, exist_ok=True)
    if world == 1:
        for key in ("RANK", "WORLD_SIZE", "LOCAL_RANK"):
            os.environ.pop(key, None)
        _workload(out, 0, tmpdir)
    else:
        mp.start_processes(_rank_main, args=(world, _free_port(), out, tmpdir), nprocs=world, join=True,
                           start_method="spawn")
    with open(out) as fh:
        return json.load(fh)


def test_empty_rank_results_match_single_rank(tmp_path):
    r1, r3 = _run(1, tmp_path), _run(3, tmp_path)
    assert r3["world"] == 3 and r3["count"] == r1["count"]
    assert r3["local_rows"][2] == 0 and sum(r3["local_rows"]) == r1["count"]
    for key in ("km_false", "km_true", "lr", "std", "dt", "rf", "rfc", "logreg"):
        np.testing.assert_allclose(r3[key], r1[key], rtol=1e-7, atol=1e-9, err_msg=key)
    for key in ("km_cost_false", "km_cost_true", "rmse", "acc"):
        assert abs(r3[key] - r1[key]) <= 1e-9 * max(1.0, abs(r1[key])), key
    assert r3["km_sizes_false"] == r1["km_sizes_false"] == r1["km_sizes_true"]
    assert [s[:2] for s in r3["stream"]] == [s[:2] for s in r1["stream"]]
    np.testing.assert_allclose([s[2] for s in r3["stream"]], [s[2] for s in r1["stream"]], rtol=1e-12)
