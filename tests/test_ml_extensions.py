"""Framework extensions beyond Spark's params stay loadable by Spark: they are written under
cml* metadata keys, not in paramMap/defaultParamMap. Also the fp8 StandardScaler output (config 5)
feeding KMeans / LogisticRegression on the CPU path."""
import json
import os

import numpy as np
import pandas as pd
import torch

from helpers import session
from clustermachinelearningforhospitalnetworks_apache_spark_amd.ml.classification import (LogisticRegression,
                                                                                            LogisticRegressionModel)
from clustermachinelearningforhospitalnetworks_apache_spark_amd.ml.clustering import KMeans
from clustermachinelearningforhospitalnetworks_apache_spark_amd.ml.feature import StandardScaler, VectorAssembler
from clustermachinelearningforhospitalnetworks_apache_spark_amd.ml.pipeline import Pipeline, PipelineModel


def _df(spark, n=2000, d=5, seed=0):
    rs = np.random.RandomState(seed)
    x = rs.randn(n, d) * [1, 3, 10, 0.5, 2][:d] + 4
    y = (x[:, 0] - 4 + 0.3 * (x[:, 1] - 4) > 0).astype(float)
    pdf = pd.DataFrame(x, columns=[f"f{i}" for i in range(d)])
    pdf["label"] = y
    return spark.createDataFrame(pdf)


def test_extension_params_outside_spark_param_maps(tmp_path):
    spark = session()
    df = VectorAssembler(inputCols=[f"f{i}" for i in range(5)], outputCol="features").transform(_df(spark))
    m = LogisticRegression(solver="sgd", maxIter=5, stepSize=0.1).fit(df)
    p = str(tmp_path / "lr")
    m.write().overwrite().save(p)
    with open(os.path.join(p, "metadata", "part-00000")) as fh:
        md = json.loads(fh.readline())
    for key in ("solver", "stepSize", "batchSize", "momentum"):
        assert key not in md["paramMap"] and key not in md["defaultParamMap"]
    assert md["cmlParamMap"]["solver"] == "sgd" and "momentum" in md["cmlDefaultParamMap"]
    back = LogisticRegressionModel.load(p)
    assert back.getOrDefault("solver") == "sgd" and back.getOrDefault("stepSize") == 0.1
    np.testing.assert_allclose(back.coefficients.toArray(), m.coefficients.toArray())


def test_fp8_standardized_pipeline_cpu(tmp_path):
    spark = session()
    df = _df(spark, n=3000)
    pipe = Pipeline(stages=[
        VectorAssembler(inputCols=[f"f{i}" for i in range(5)], outputCol="raw"),
        StandardScaler(inputCol="raw", outputCol="features", withMean=True, outputDtype="fp8"),
        KMeans(k=3, seed=7, maxIter=5, predictionCol="cluster"),
        LogisticRegression(maxIter=30),
    ])
    model = pipe.fit(df)
    out = model.transform(df)
    feats = out._feature_matrix("features")
    assert feats.dtype == torch.float8_e4m3fn
    raw = out._feature_matrix("raw").double()
    z = (raw - raw.mean(0)) / raw.std(0)
    np.testing.assert_array_equal(feats.double().numpy(), z.clamp(-448, 448).to(torch.float8_e4m3fn).double().numpy())
    acc = (out.toPandas()["prediction"] == out.toPandas()["label"]).mean()
    assert acc > 0.9
    model.write().overwrite().save(str(tmp_path / "pm"))
    back = PipelineModel.load(str(tmp_path / "pm"))
    assert back.stages[1].getOrDefault("outputDtype") == "fp8"
