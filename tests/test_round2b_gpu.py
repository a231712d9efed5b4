"""GPU runs of the later round-2 additions against the local[1] CPU session: device hash lanes,
device group-by, LDA, PowerIterationClustering, Word2Vec, DCT and FeatureHasher."""
import datetime as dt

import numpy as np
import pandas as pd
import pytest

from clustermachinelearningforhospitalnetworks_apache_spark_amd.sql import SparkSession
from clustermachinelearningforhospitalnetworks_apache_spark_amd.sql import functions as F

pytestmark = pytest.mark.gpu


def _run(master):
    from clustermachinelearningforhospitalnetworks_apache_spark_amd.ml.clustering import LDA, PowerIterationClustering
    from clustermachinelearningforhospitalnetworks_apache_spark_amd.ml.feature import (
        DCT, FeatureHasher, VectorAssembler, Word2Vec)
    spark = SparkSession.builder.appName("r2b").master(master).getOrCreate()
    try:
        rs = np.random.RandomState(5)
        n = 5000
        pdf = pd.DataFrame({"i": rs.randint(-2 ** 31, 2 ** 31, n).astype(np.int64), "l": rs.randint(-2 ** 62, 2 ** 62, n),
                            "d": rs.normal(size=n), "h": rs.randint(0, 40, n), "w": np.array(["icu", "er", "gen"])[
                                rs.randint(0, 3, n)]})
        df = spark.createDataFrame(pdf)
        if master == "mi355x":
            assert df._device.type == "cuda"
        out = {}
        out["hash"] = [tuple(r) for r in df.select(F.hash("i", "l", "d", "w"), F.xxhash64("i", "l", "d", "w")).collect()]
        out["grp"] = sorted(tuple(r) for r in df.groupBy("w", "h").agg(F.count("*"), F.sum("l"), F.avg("d"),
                                                                      F.max("i")).collect())
        cnt = pd.DataFrame(np.floor(np.abs(rs.normal(size=(600, 6))) * 3), columns=list("abcdef"))
        cdf = VectorAssembler(inputCols=list("abcdef"), outputCol="features").transform(spark.createDataFrame(cnt))
        out["lda"] = LDA(k=3, maxIter=5, seed=2, subsamplingRate=0.5).fit(cdf).topicsMatrix().toArray()
        out["dct"] = np.stack([v.toArray() for v in DCT(inputCol="features", outputCol="y").transform(cdf)
                               .toPandas()["y"]])
        out["fh"] = np.stack([v.toArray() for v in FeatureHasher(inputCols=["d", "w"], numFeatures=64,
                                                                 outputCol="f").transform(df).toPandas()["f"]])
        edges = [(i, j, 1.0 if i < 6 else 3.0) for b in (0, 6) for i in range(b, b + 6) for j in range(i + 1, b + 6)]
        edges.append((5, 6, 0.01))
        out["pic"] = sorted(tuple(r) for r in PowerIterationClustering(k=2, weightCol="weight").assignClusters(
            spark.createDataFrame(edges, "src long, dst long, weight double")).collect())
        sents = [([["icu", "vent", "sedation"], ["birth", "midwife", "newborn"]][i % 2] * 3,) for i in range(200)]
        w2v = Word2Vec(vectorSize=8, minCount=1, seed=3, inputCol="t", maxIter=2).fit(
            spark.createDataFrame(sents, "t array<string>"))
        out["w2v"] = np.stack([r.vector.toArray() for r in w2v.getVectors().collect()])
        return out
    finally:
        spark.stop()


def test_round2b_gpu_equals_cpu():
    g, c = _run("mi355x"), _run("local[1]")
    assert g["hash"] == c["hash"]
    assert [r[:3] for r in g["grp"]] == [r[:3] for r in c["grp"]]
    np.testing.assert_allclose([r[4] for r in g["grp"]], [r[4] for r in c["grp"]], rtol=1e-12)
    assert [r[5] for r in g["grp"]] == [r[5] for r in c["grp"]]
    np.testing.assert_allclose(g["lda"], c["lda"], rtol=1e-8)
    np.testing.assert_allclose(g["dct"], c["dct"], atol=1e-12)
    np.testing.assert_array_equal(g["fh"], c["fh"])
    assert g["pic"] == c["pic"]
    np.testing.assert_allclose(g["w2v"], c["w2v"], rtol=1e-4, atol=1e-6)
