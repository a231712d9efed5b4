"""pyspark.ml.tuning (ParamGridBuilder / CrossValidator / TrainValidationSplit) and the OneHotEncoder /
Imputer feature stages, against hand-computed numpy oracles. CPU (local session)."""
import math

import numpy as np
import pandas as pd
import pytest

from helpers import session
from clustermachinelearningforhospitalnetworks_apache_spark_amd.ml import util as U
from clustermachinelearningforhospitalnetworks_apache_spark_amd.ml.evaluation import RegressionEvaluator
from clustermachinelearningforhospitalnetworks_apache_spark_amd.ml.feature import (Imputer, ImputerModel,
                                                                                     OneHotEncoder,
                                                                                     OneHotEncoderModel,
                                                                                     StringIndexer, VectorAssembler)
from clustermachinelearningforhospitalnetworks_apache_spark_amd.ml.regression import (DecisionTreeRegressor,
                                                                                        LinearRegression)
from clustermachinelearningforhospitalnetworks_apache_spark_amd.ml.tuning import (CrossValidator,
                                                                                    CrossValidatorModel,
                                                                                    ParamGridBuilder,
                                                                                    TrainValidationSplit,
                                                                                    TrainValidationSplitModel)


def _reg_df(spark, n=1200, seed=3):
    rs = np.random.RandomState(seed)
    x = rs.rand(n, 3) * 10
    y = np.where(x[:, 0] > 5, 8.0, 2.0) + 0.5 * x[:, 1] + rs.randn(n) * 0.3
    pdf = pd.DataFrame(x, columns=["a", "b", "c"])
    pdf["y"] = y
    df = spark.createDataFrame(pdf)
    return VectorAssembler(inputCols=["a", "b", "c"], outputCol="features").transform(df)


def test_param_grid_builder_cartesian():
    dt = DecisionTreeRegressor()
    grid = ParamGridBuilder().addGrid(dt.maxDepth, [1, 3]).addGrid(dt.maxBins, [8, 16, 32]) \
        .baseOn({dt.minInstancesPerNode: 2}).build()
    assert len(grid) == 6
    assert {(g[dt.maxDepth], g[dt.maxBins]) for g in grid} == {(d, b) for d in (1, 3) for b in (8, 16, 32)}
    assert all(g[dt.minInstancesPerNode] == 2 for g in grid)


def test_cross_validator_picks_deeper_tree_and_matches_manual_folds(tmp_path):
    spark = session()
    df = _reg_df(spark)
    dt = DecisionTreeRegressor(labelCol="y")
    grid = ParamGridBuilder().addGrid(dt.maxDepth, [1, 4]).build()
    ev = RegressionEvaluator(labelCol="y", metricName="rmse")
    cv = CrossValidator(estimator=dt, estimatorParamMaps=grid, evaluator=ev, numFolds=3, seed=11)
    m = cv.fit(df)
    assert len(m.avgMetrics) == 2 and len(m.stdMetrics) == 2
    assert m.avgMetrics[1] < m.avgMetrics[0]  # depth 4 captures the step + slope better
    assert m.bestModel.getOrDefault("maxDepth") == 4
    # oracle: the same folds by hand
    folds = df.randomSplit([1.0] * 3, seed=11)
    manual = []
    for pm in grid:
        ms = []
        for i in range(3):
            tr = None
            for j in range(3):
                if j != i:
                    tr = folds[j] if tr is None else tr.union(folds[j])
            ms.append(ev.evaluate(dt.fit(tr, pm).transform(folds[i])))
        manual.append(np.mean(ms))
    np.testing.assert_allclose(m.avgMetrics, manual, rtol=1e-12)
    # transform = best model's transform; save/load round trip
    p1 = m.transform(df).toPandas()["prediction"].to_numpy()
    p2 = m.bestModel.transform(df).toPandas()["prediction"].to_numpy()
    np.testing.assert_array_equal(p1, p2)
    path = str(tmp_path / "cv")
    m.write().overwrite().save(path)
    back = CrossValidatorModel.load(path)
    assert isinstance(U.load(path), CrossValidatorModel)
    np.testing.assert_allclose(back.avgMetrics, m.avgMetrics)
    np.testing.assert_array_equal(back.transform(df).toPandas()["prediction"].to_numpy(), p1)


def test_cross_validator_fold_col_and_sub_models():
    spark = session()
    rs = np.random.RandomState(0)
    x = rs.rand(300) * 4
    pdf = pd.DataFrame({"x": x, "y": 2 * x + 1 + rs.randn(300) * 0.01, "fold": np.arange(300) % 3})
    df = VectorAssembler(inputCols=["x"], outputCol="features").transform(spark.createDataFrame(pdf))
    lr = LinearRegression(labelCol="y")
    grid = ParamGridBuilder().addGrid(lr.regParam, [0.0, 10.0]).build()
    cv = CrossValidator(estimator=lr, estimatorParamMaps=grid, evaluator=RegressionEvaluator(labelCol="y"),
                        numFolds=3, foldCol="fold", collectSubModels=True)
    m = cv.fit(df)
    assert m.bestModel.getOrDefault("regParam") == 0.0
    assert len(m.subModels) == 3 and len(m.subModels[0]) == 2
    # fold 0 validation = rows with fold == 0: refit by hand
    tr = df.filter(df["fold"] != 0)
    va = df.filter(df["fold"] == 0)
    ref = RegressionEvaluator(labelCol="y").evaluate(lr.fit(tr, grid[0]).transform(va))
    got = RegressionEvaluator(labelCol="y").evaluate(m.subModels[0][0].transform(va))
    assert math.isclose(ref, got, rel_tol=1e-12)


def test_train_validation_split(tmp_path):
    spark = session()
    df = _reg_df(spark, n=800, seed=5)
    dt = DecisionTreeRegressor(labelCol="y")
    grid = ParamGridBuilder().addGrid(dt.maxDepth, [1, 5]).build()
    ev = RegressionEvaluator(labelCol="y")
    m = TrainValidationSplit(estimator=dt, estimatorParamMaps=grid, evaluator=ev, trainRatio=0.7, seed=2).fit(df)
    tr, va = df.randomSplit([0.7, 0.3], seed=2)
    manual = [ev.evaluate(dt.fit(tr, pm).transform(va)) for pm in grid]
    np.testing.assert_allclose(m.validationMetrics, manual, rtol=1e-12)
    assert m.bestModel.getOrDefault("maxDepth") == 5
    path = str(tmp_path / "tvs")
    m.save(path)
    back = TrainValidationSplitModel.load(path)
    np.testing.assert_allclose(back.validationMetrics, m.validationMetrics)


def test_one_hot_encoder_after_string_indexer(tmp_path):
    spark = session()
    pdf = pd.DataFrame({"hospital_id": ["h1", "h2", "h3", "h1", "h2", "h1"]})
    df = StringIndexer(inputCol="hospital_id", outputCol="hidx").fit(spark.createDataFrame(pdf)).transform(
        spark.createDataFrame(pdf))
    idx = df.toPandas()["hidx"].to_numpy().astype(int)  # h1 -> 0 (most frequent), h2 -> 1, h3 -> 2
    enc = OneHotEncoder(inputCols=["hidx"], outputCols=["hvec"])
    m = enc.fit(df)
    assert m.categorySizes == [3]
    out = np.stack([v.toArray() for v in m.transform(df).toPandas()["hvec"]])
    ref = np.eye(3)[idx][:, :2]  # dropLast
    np.testing.assert_array_equal(out, ref)
    m2 = OneHotEncoder(inputCol="hidx", outputCol="hvec", dropLast=False).fit(df)
    out2 = np.stack([v.toArray() for v in m2.transform(df).toPandas()["hvec"]])
    np.testing.assert_array_equal(out2, np.eye(3)[idx])
    # handleInvalid: unseen index 5 -> error, or the extra slot with 'keep'
    bad = spark.createDataFrame(pd.DataFrame({"hidx": [0.0, 5.0]}))
    with pytest.raises(ValueError):
        m.transform(bad).toPandas()
    mk = OneHotEncoderModel([3])
    mk.setInputCols(["hidx"]).setOutputCols(["hvec"]).setHandleInvalid("keep")
    outk = np.stack([v.toArray() for v in mk.transform(bad).toPandas()["hvec"]])
    np.testing.assert_array_equal(outk, [[1, 0, 0], [0, 0, 0]])  # size 3 + 1 keep - 1 dropLast; invalid = last
    path = str(tmp_path / "ohe")
    m.save(path)
    back = OneHotEncoderModel.load(path)
    assert back.categorySizes == [3] and back.getOrDefault("outputCols") == ["hvec"]


@pytest.mark.parametrize("strategy", ["mean", "median", "mode"])
def test_imputer(strategy, tmp_path):
    spark = session()
    a = [1.0, 2.0, None, 4.0, 4.0, float("nan"), 10.0]
    b = [3, None, 3, 7, 1, 1, 3]
    df = spark.createDataFrame(pd.DataFrame({"a": a, "b": pd.array(b, dtype="Int32")}))
    m = Imputer(strategy=strategy, inputCols=["a", "b"], outputCols=["a_i", "b_i"]).fit(df)
    av = np.array([1.0, 2.0, 4.0, 4.0, 10.0])
    bv = np.array([3, 3, 7, 1, 1, 3], dtype=float)
    if strategy == "mean":
        ref = [av.mean(), bv.mean()]
    elif strategy == "median":
        ref = [np.sort(av)[(av.size - 1) // 2], np.sort(bv)[(bv.size - 1) // 2]]
    else:
        ref = [4.0, 3.0]
    np.testing.assert_allclose(m.surrogates, ref)
    out = m.transform(df).toPandas()
    np.testing.assert_allclose(out["a_i"].to_numpy(dtype=float),
                               [1.0, 2.0, ref[0], 4.0, 4.0, ref[0], 10.0])
    np.testing.assert_array_equal(out["b_i"].to_numpy(dtype=float),
                                  [3, int(ref[1]), 3, 7, 1, 1, 3])
    path = str(tmp_path / "imp")
    m.save(path)
    back = ImputerModel.load(path)
    np.testing.assert_allclose(back.surrogates, m.surrogates)
    assert list(back.surrogateDF.columns) == ["a", "b"]
