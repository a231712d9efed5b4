"""MaxAbsScaler, RobustScaler, ElementwiseProduct, PolynomialExpansion, Interaction, VectorSlicer,
VectorIndexer, SQLTransformer, selectors, RFormula; ml.stat ANOVA / F-value / KS tests and Summarizer.
Oracles: numpy / scipy / sklearn formulas of the same definitions; Spark persistence round trips."""
import numpy as np
import pytest

from helpers import session
from clustermachinelearningforhospitalnetworks_apache_spark_amd.ml import Pipeline, PipelineModel
from clustermachinelearningforhospitalnetworks_apache_spark_amd.ml import util as U
from clustermachinelearningforhospitalnetworks_apache_spark_amd.ml.feature import (
    ChiSqSelector, ElementwiseProduct, Interaction, MaxAbsScaler, MaxAbsScalerModel, PolynomialExpansion, RFormula,
    RFormulaModel, RobustScaler, RobustScalerModel, SQLTransformer, UnivariateFeatureSelector,
    VarianceThresholdSelector, VectorAssembler, VectorIndexer, VectorIndexerModel, VectorSlicer)
from clustermachinelearningforhospitalnetworks_apache_spark_amd.ml.stat import (
    ANOVATest, ChiSquareTest, FValueTest, KolmogorovSmirnovTest, Summarizer)


@pytest.fixture(scope="module")
def spark():
    return session()


def _vec(df, name):
    return np.stack([v.toArray() for v in df.toPandas()[name]])


def _frame(spark, X, extra=None):
    cols = [f"c{j}" for j in range(X.shape[1])]
    rows = [tuple(float(v) for v in r) + (tuple(extra[i]) if extra is not None else ()) for i, r in enumerate(X)]
    schema = ", ".join(f"{c} DOUBLE" for c in cols)
    if extra is not None:
        schema += ", " + ", ".join(f"e{j} DOUBLE" for j in range(len(extra[0])))
    df = spark.createDataFrame(rows, schema)
    return VectorAssembler(inputCols=cols, outputCol="f").transform(df)


def test_maxabs_and_robust_scaler(spark, tmp_path):
    rs = np.random.RandomState(0)
    X = rs.normal(size=(301, 4)) * [1, 5, 0, 2] + [0, 1, 0, -3]
    df = _frame(spark, X)
    m = MaxAbsScaler(inputCol="f", outputCol="s").fit(df)
    ma = np.abs(X).max(0)
    np.testing.assert_allclose(m.maxAbs.toArray(), ma)
    np.testing.assert_allclose(_vec(m.transform(df), "s"), X / np.where(ma == 0, 1, ma))
    m.write().overwrite().save(str(tmp_path / "mas"))
    np.testing.assert_allclose(MaxAbsScalerModel.load(str(tmp_path / "mas")).maxAbs.toArray(), ma)

    r = RobustScaler(inputCol="f", outputCol="r", withCentering=True).fit(df)
    srt = np.sort(X, 0)
    q = lambda p: srt[max(int(np.ceil(p * len(X))) - 1, 0)]
    np.testing.assert_allclose(r.median.toArray(), q(0.5))
    rng = q(0.75) - q(0.25)
    np.testing.assert_allclose(r.range.toArray(), rng)
    scale = np.where(rng == 0, 0, 1 / np.where(rng == 0, 1, rng))
    np.testing.assert_allclose(_vec(r.transform(df), "r"), (X - q(0.5)) * scale)
    r.write().overwrite().save(str(tmp_path / "rs"))
    back = U.load(str(tmp_path / "rs"))
    assert isinstance(back, RobustScalerModel) and back.getWithCentering()
    np.testing.assert_allclose(back.range.toArray(), rng)


def test_elementwise_polynomial_interaction(spark):
    X = np.array([[1.0, 2.0, 3.0], [-1.0, 0.5, 2.0]])
    df = _frame(spark, X)
    ep = ElementwiseProduct(scalingVec=[2.0, 0.0, -1.0], inputCol="f", outputCol="e").transform(df)
    np.testing.assert_allclose(_vec(ep, "e"), X * [2, 0, -1])
    # Spark's documented order for (x, y), degree 2: x, x^2, y, x*y, y^2
    df2 = _frame(spark, np.array([[2.0, 3.0]]))
    pe = PolynomialExpansion(degree=2, inputCol="f", outputCol="p").transform(df2)
    np.testing.assert_allclose(_vec(pe, "p")[0], [2, 4, 3, 6, 9])
    pe3 = PolynomialExpansion(degree=3, inputCol="f", outputCol="p").transform(df)
    x, y, z = X[0]
    got = _vec(pe3, "p")
    assert got.shape == (2, 19)
    # every monomial of degree <= 3 appears exactly once
    expect = sorted(x ** a * y ** b * z ** c for a in range(4) for b in range(4) for c in range(4)
                    if 0 < a + b + c <= 3)
    np.testing.assert_allclose(sorted(got[0]), expect)
    it = Interaction(inputCols=["c0", "f"], outputCol="i").transform(df)
    np.testing.assert_allclose(_vec(it, "i"), X[:, :1] * X)


def test_vector_slicer_by_index_and_name(spark):
    X = np.arange(12, dtype=float).reshape(3, 4)
    df = _frame(spark, X)
    out = VectorSlicer(inputCol="f", outputCol="s", indices=[3], names=["c1"]).transform(df)
    np.testing.assert_allclose(_vec(out, "s"), X[:, [3, 1]])
    with pytest.raises(ValueError):
        VectorSlicer(inputCol="f", outputCol="s", names=["nope"]).transform(df)


def test_vector_indexer(spark, tmp_path):
    X = np.array([[0.0, 1.5, -1.0], [2.0, 2.5, 0.0], [0.0, 3.5, -1.0], [5.0, 4.5, 2.0]])
    df = _frame(spark, X)
    m = VectorIndexer(maxCategories=3, inputCol="f", outputCol="ix").fit(df)
    # feature 0: {0, 2, 5} -> 0 first; feature 1 has 4 values -> continuous; feature 2: {-1, 0, 2}
    assert sorted(m.categoryMaps) == [0, 2]
    assert m.categoryMaps[0] == {0.0: 0, 2.0: 1, 5.0: 2}
    assert m.categoryMaps[2] == {0.0: 0, -1.0: 1, 2.0: 2}
    got = _vec(m.transform(df), "ix")
    np.testing.assert_allclose(got, [[0, 1.5, 1], [1, 2.5, 0], [0, 3.5, 1], [2, 4.5, 2]])
    m.write().overwrite().save(str(tmp_path / "vi"))
    back = VectorIndexerModel.load(str(tmp_path / "vi"))
    assert back.categoryMaps == m.categoryMaps
    bad = _frame(spark, np.array([[7.0, 1.0, 0.0]]))
    with pytest.raises(ValueError):
        back.transform(bad)
    assert back.setHandleInvalid("skip").transform(bad).count() == 0
    np.testing.assert_allclose(_vec(back.setHandleInvalid("keep").transform(bad), "ix"), [[3, 1, 0]])


def test_sql_transformer(spark):
    df = spark.createDataFrame([(1, 2.0), (2, 5.0)], "id INT, v DOUBLE")
    out = SQLTransformer(statement="SELECT id, v * 2 AS v2 FROM __THIS__ WHERE v > 3").transform(df)
    assert [tuple(r) for r in out.collect()] == [(2, 10.0)]


def test_selectors(spark, tmp_path):
    rs = np.random.RandomState(3)
    n = 400
    y = rs.randint(0, 3, n).astype(float)
    informative = y + rs.randint(0, 2, n)          # categorical, depends on y
    noise = rs.randint(0, 4, n).astype(float)       # categorical, independent
    const = np.ones(n)
    X = np.stack([noise, informative, const], 1)
    df = _frame(spark, X, extra=y[:, None])
    vt = VarianceThresholdSelector(featuresCol="f", outputCol="v").fit(df)
    assert vt.selectedFeatures == [0, 1]
    np.testing.assert_allclose(_vec(vt.transform(df), "v"), X[:, :2])
    cs = ChiSqSelector(numTopFeatures=1, featuresCol="f", outputCol="c", labelCol="e0").fit(df)
    assert cs.selectedFeatures == [1]
    cs.write().overwrite().save(str(tmp_path / "cs"))
    assert U.load(str(tmp_path / "cs")).selectedFeatures == [1]
    fpr = ChiSqSelector(selectorType="fpr", fpr=1e-6, featuresCol="f", outputCol="c", labelCol="e0").fit(df)
    assert fpr.selectedFeatures == [1]
    # continuous features vs continuous label: F-value regression test picks the correlated one
    Xc = rs.normal(size=(n, 3))
    yc = 3 * Xc[:, 2] + 0.1 * rs.normal(size=n)
    dfc = _frame(spark, Xc, extra=yc[:, None])
    u = UnivariateFeatureSelector(featuresCol="f", outputCol="u", labelCol="e0", featureType="continuous",
                                  labelType="continuous", selectionThreshold=1).fit(dfc)
    assert u.selectedFeatures == [2]


def test_anova_fvalue_chisq_vs_scipy(spark):
    from scipy import stats
    rs = np.random.RandomState(5)
    n = 300
    y = rs.randint(0, 3, n).astype(float)
    X = np.stack([rs.normal(size=n) + y, rs.normal(size=n)], 1)
    df = _frame(spark, X, extra=y[:, None])
    r = ANOVATest.test(df, "f", "e0").collect()[0]
    for j in range(2):
        F, p = stats.f_oneway(*[X[y == c, j] for c in range(3)])
        assert r.fValues[j] == pytest.approx(F, rel=1e-9)
        assert r.pValues[j] == pytest.approx(p, rel=1e-6, abs=1e-300)
    assert r.degreesOfFreedom == [n - 1, n - 1]
    yc = X[:, 0] * 2 + rs.normal(size=n)
    dfc = _frame(spark, X, extra=yc[:, None])
    fv = FValueTest.test(dfc, "f", "e0").collect()[0]
    from sklearn.feature_selection import f_regression
    F, p = f_regression(X, yc)
    np.testing.assert_allclose(fv.fValues.toArray(), F, rtol=1e-9)
    np.testing.assert_allclose(fv.pValues.toArray(), p, rtol=1e-6, atol=1e-300)
    flat = ChiSquareTest.test(_frame(spark, np.round(X), extra=y[:, None]), "f", "e0", flatten=True)
    assert flat.count() == 2 and set(flat.columns) == {"featureIndex", "pValue", "degreesOfFreedom", "statistic"}


def test_kolmogorov_smirnov(spark):
    from scipy import stats
    rs = np.random.RandomState(2)
    v = rs.normal(1.0, 2.0, 200)
    df = spark.createDataFrame([(float(a),) for a in v], "x DOUBLE")
    r = KolmogorovSmirnovTest.test(df, "x", "norm", 1.0, 2.0).collect()[0]
    ref = stats.kstest(v, "norm", args=(1.0, 2.0), method="exact")
    assert r.statistic == pytest.approx(ref.statistic, rel=1e-12)
    assert r.pValue == pytest.approx(ref.pvalue, rel=1e-6)
    r0 = KolmogorovSmirnovTest.test(df, "x", "norm").collect()[0]
    assert r0.pValue < 1e-6


def test_summarizer(spark):
    from clustermachinelearningforhospitalnetworks_apache_spark_amd.sql import functions as F
    rs = np.random.RandomState(4)
    X = rs.normal(size=(50, 3))
    X[::5, 1] = 0.0
    w = rs.uniform(0.5, 2.0, 50)
    g = np.arange(50) % 2
    df = _frame(spark, X, extra=np.stack([w, g], 1))
    res = df.select(Summarizer.metrics("mean", "variance", "count", "numNonZeros", "max", "min", "normL1",
                                       "normL2", "weightSum", "std", "sum").summary(F.col("f"))).collect()[0][0]
    np.testing.assert_allclose(res.mean.toArray(), X.mean(0))
    np.testing.assert_allclose(res.variance.toArray(), X.var(0, ddof=1))
    np.testing.assert_allclose(res.std.toArray(), X.std(0, ddof=1))
    np.testing.assert_allclose(res.sum.toArray(), X.sum(0))
    assert res["count"] == 50 and res.weightSum == pytest.approx(50.0)
    np.testing.assert_allclose(res.numNonZeros.toArray(), (X != 0).sum(0))
    np.testing.assert_allclose(res.max.toArray(), X.max(0))
    np.testing.assert_allclose(res.min.toArray(), X.min(0))
    np.testing.assert_allclose(res.normL1.toArray(), np.abs(X).sum(0))
    np.testing.assert_allclose(res.normL2.toArray(), np.sqrt((X * X).sum(0)))
    # weighted: Spark's unbiased weighted variance (denominator W - sum(w^2)/W)
    wm = df.select(Summarizer.mean(F.col("f"), F.col("e0")), Summarizer.variance("f", "e0")).collect()[0]
    mu = (w[:, None] * X).sum(0) / w.sum()
    np.testing.assert_allclose(wm[0].toArray(), mu)
    den = w.sum() - (w * w).sum() / w.sum()
    np.testing.assert_allclose(wm[1].toArray(), (w[:, None] * (X - mu) ** 2).sum(0) / den)
    # grouped
    gm = {r[0]: r[1].toArray() for r in df.groupBy("e1").agg(Summarizer.mean(F.col("f"))).collect()}
    np.testing.assert_allclose(gm[0.0], X[g == 0].mean(0))
    np.testing.assert_allclose(gm[1.0], X[g == 1].mean(0))


def test_rformula(spark, tmp_path):
    rows = [("a", 1.0, 10.0, "yes"), ("b", 2.0, 11.0, "no"), ("a", 3.0, 12.0, "yes"), ("c", 4.0, 13.0, "no"),
            ("a", 5.0, 14.0, "no")]
    df = spark.createDataFrame(rows, "ward STRING, age DOUBLE, los DOUBLE, readmit STRING")
    m = RFormula(formula="readmit ~ ward + age").fit(df)
    out = m.transform(df)
    f = _vec(out, "features")
    # ward indexed by frequency (a, then b/c alphabetical tie-break), one-hot dropping the last
    np.testing.assert_allclose(f, [[1, 0, 1], [0, 1, 2], [1, 0, 3], [0, 0, 4], [1, 0, 5]])
    lab = np.asarray(out.toPandas()["label"].tolist())
    np.testing.assert_allclose(lab, [1, 0, 1, 0, 0])  # 'no' is the most frequent label
    assert out.columns == ["ward", "age", "los", "readmit", "features", "label"]
    from clustermachinelearningforhospitalnetworks_apache_spark_amd.ml.feature_more import vector_attr_names
    assert vector_attr_names(out, "features") == ["ward_a", "ward_b", "age"]
    # no intercept: the first string term keeps every category
    f0 = _vec(RFormula(formula="los ~ ward + age - 1").fit(df).transform(df), "features")
    assert f0.shape[1] == 4
    # '.' minus a term, and an interaction
    mi = RFormula(formula="los ~ . - readmit + ward:age").fit(df)
    fi = _vec(mi.transform(df), "features")
    assert fi.shape[1] == 2 + 1 + 3
    np.testing.assert_allclose(fi[:, 3:], np.eye(3)[[0, 1, 0, 2, 0]] * np.array([1, 2, 3, 4, 5.])[:, None])
    np.testing.assert_allclose(np.asarray(mi.transform(df).toPandas()["label"].tolist()), [10, 11, 12, 13, 14])
    m.write().overwrite().save(str(tmp_path / "rf"))
    back = U.load(str(tmp_path / "rf"))
    assert isinstance(back, RFormulaModel)
    np.testing.assert_allclose(_vec(back.transform(df), "features"), f)
    # inside a pipeline, with the label column absent at scoring time
    pm = Pipeline(stages=[RFormula(formula="readmit ~ ward + age")]).fit(df)
    scored = pm.transform(df.select("ward", "age"))
    assert "label" not in scored.columns and _vec(scored, "features").shape == (5, 3)


def test_ml_functions_vector_array(spark):
    from clustermachinelearningforhospitalnetworks_apache_spark_amd.ml.functions import array_to_vector, vector_to_array
    from clustermachinelearningforhospitalnetworks_apache_spark_amd.sql import functions as F
    X = np.array([[1.0, 2.0], [3.5, -1.0]])
    df = _frame(spark, X)
    arr = df.select(vector_to_array(F.col("f")).alias("a"))
    assert [r.a for r in arr.collect()] == [[1.0, 2.0], [3.5, -1.0]]
    back = arr.select(array_to_vector("a").alias("v"))
    np.testing.assert_allclose(_vec(back, "v"), X)
    f32 = df.select(vector_to_array("f", "float32").alias("a")).schema["a"].dataType.simpleString()
    assert f32 == "array<float>"
