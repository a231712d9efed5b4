"""VectorAssembler(handleInvalid="error") on one dense vector column aliases it and defers the NaN check
to the consumer (Spark's transform is lazy and raises when rows are consumed): StandardScaler.fit takes
it over from its moments (no extra read), other estimators run it in _feature_matrix, row subsets
(randomSplit) inherit it, and a clean column never raises."""
import pytest
import torch

from clustermachinelearningforhospitalnetworks_apache_spark_amd.ml.clustering import KMeans
from clustermachinelearningforhospitalnetworks_apache_spark_amd.ml.feature import StandardScaler, VectorAssembler
from clustermachinelearningforhospitalnetworks_apache_spark_amd.sql import SparkSession


def _frame(nan_row=None):
    spark = SparkSession.builder.master("local[1]").getOrCreate()
    g = torch.Generator().manual_seed(0)
    x = torch.randn(2000, 6, generator=g, dtype=torch.float64)
    if nan_row is not None:
        x[nan_row, 2] = float("nan")
    spark.conf.set("cml.ml.features.dtype", "float64")
    return spark.createDataFrameFromTensors({"raw": x})


def test_clean_column_passes_and_aliases():
    df = _frame()
    out = VectorAssembler(inputCols=["raw"], outputCol="f").transform(df)
    assert out._feature_matrix("f").data_ptr() == df._feature_matrix("raw").data_ptr()
    StandardScaler(inputCol="f", outputCol="s").fit(out)
    KMeans(k=3, seed=1, maxIter=3).fit(out.withColumnRenamed("f", "features"))


@pytest.mark.parametrize("consumer", ["scaler", "kmeans", "split", "binarizer", "collect", "assembler", "topandas"])
def test_nan_raises_at_the_consumer(consumer):
    df = _frame(nan_row=1234)
    out = VectorAssembler(inputCols=["raw"], outputCol="features").transform(df)  # no raise yet
    with pytest.raises(ValueError, match="handleInvalid='error'"):
        if consumer == "scaler":
            StandardScaler(inputCol="features", outputCol="s").fit(out)
        elif consumer == "kmeans":
            KMeans(k=3, seed=1, maxIter=3).fit(out)
        elif consumer == "binarizer":  # readers of the vector values, not only fits, raise
            from clustermachinelearningforhospitalnetworks_apache_spark_amd.ml.feature import Binarizer
            Binarizer(threshold=0.0, inputCol="features", outputCol="b").transform(out).collect()
        elif consumer == "collect":
            out.select("features").collect()
        elif consumer == "assembler":
            VectorAssembler(inputCols=["features"], outputCol="g", handleInvalid="keep").transform(out).collect()
        elif consumer == "topandas":
            out.toPandas()
        else:
            a, b = out.randomSplit([0.5, 0.5], seed=3)
            part = a if bool(torch.isnan(a._cols["features"]._vals()).any()) else b
            KMeans(k=3, seed=1, maxIter=3).fit(part)


def _nan_rank_main(rank, world, port, out_dir):
    import os
    os.environ.update({"RANK": str(rank), "WORLD_SIZE": str(world), "LOCAL_RANK": str(rank),
                       "MASTER_ADDR": "127.0.0.1", "MASTER_PORT": str(port), "CML_FORCE_CPU": "1"})
    import torch as _t
    _t.set_num_threads(1)
    from clustermachinelearningforhospitalnetworks_apache_spark_amd.sql import SparkSession as S
    spark = S.builder.master("local[1]").getOrCreate()
    spark.conf.set("cml.ml.features.dtype", "float64")
    x = _t.randn(500, 4, dtype=_t.float64)
    if rank == 1:
        x[7, 1] = float("nan")  # only this rank's shard holds a NaN
    df = spark.createDataFrameFromTensors({"raw": x})
    out = VectorAssembler(inputCols=["raw"], outputCol="features").transform(df)
    res = "no error"
    try:
        out.select("features").collect()
    except ValueError as e:
        res = "raised" if "handleInvalid" in str(e) else repr(e)
    with open(os.path.join(out_dir, f"r{rank}"), "w") as fh:
        fh.write(res)
    spark.stop()


def test_nan_on_one_rank_raises_on_every_rank(tmp_path):
    """the deferred check of a consumer (collect) agrees on the verdict over the ranks, so the
    NaN-free rank raises too instead of blocking in collect's gather until the collective timeout."""
    import socket
    import torch.multiprocessing as mp
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    mp.start_processes(_nan_rank_main, args=(2, port, str(tmp_path)), nprocs=2, join=True, start_method="spawn")
    assert [(tmp_path / f"r{r}").read_text() for r in range(2)] == ["raised", "raised"]
