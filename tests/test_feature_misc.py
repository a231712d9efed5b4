"""DCT (vs scipy's orthonormal DCT-II / DCT-III), FeatureHasher (hash positions from MurmurHash3
x86_32 seed 42 on "col" / "col=value", Spark's documented example), VectorSizeHint, and
Java's Double.toString used for categorical values."""
import numpy as np
import pandas as pd
import pytest
import scipy.fft

from clustermachinelearningforhospitalnetworks_apache_spark_amd.ml.feature import (
    DCT, FeatureHasher, VectorAssembler, VectorSizeHint)
from clustermachinelearningforhospitalnetworks_apache_spark_amd.ml.feature_text import murmur3_32
from clustermachinelearningforhospitalnetworks_apache_spark_amd.ml.util import java_double_str
from clustermachinelearningforhospitalnetworks_apache_spark_amd.sql import SparkSession


@pytest.fixture(scope="module")
def spark():
    s = SparkSession.builder.appName("fmisc").master("local[1]").getOrCreate()
    yield s
    s.stop()


def _vecs(df, col):
    return np.stack([v.toArray() for v in df.toPandas()[col]])


def test_dct_matches_scipy(spark):
    rs = np.random.RandomState(0)
    X = rs.normal(size=(20, 7))
    df = VectorAssembler(inputCols=[f"c{i}" for i in range(7)], outputCol="f").transform(
        spark.createDataFrame(pd.DataFrame(X, columns=[f"c{i}" for i in range(7)])))
    y = _vecs(DCT(inputCol="f", outputCol="y").transform(df), "y")
    np.testing.assert_allclose(y, scipy.fft.dct(X, type=2, norm="ortho", axis=1), atol=1e-12)
    z = _vecs(DCT(inverse=True, inputCol="f", outputCol="z").transform(df), "z")
    np.testing.assert_allclose(z, scipy.fft.idct(X, type=2, norm="ortho", axis=1), atol=1e-12)
    # round trip
    back = _vecs(DCT(inverse=True, inputCol="y", outputCol="b").transform(
        DCT(inputCol="f", outputCol="y").transform(df)), "b")
    np.testing.assert_allclose(back, X, atol=1e-12)


def test_feature_hasher(spark):
    pdf = pd.DataFrame({"real": [2.2, 3.3, 4.4, 5.5], "bool": [True, False, True, False],
                        "stringNum": ["1", "2", "3", "4"], "string": ["foo", "bar", "baz", "foo"]})
    df = spark.createDataFrame(pdf)
    nf = 262144
    out = FeatureHasher(inputCols=["real", "bool", "stringNum", "string"], outputCol="features").transform(df)
    X = _vecs(out, "features")
    assert X.shape == (4, nf)
    h = lambda t: murmur3_32(t.encode(), 42) % nf
    for i, r in enumerate(pdf.to_dict("records")):
        expect = {}
        for k, v in ((h("real"), r["real"]), (h(f"bool={'true' if r['bool'] else 'false'}"), 1.0),
                     (h(f"stringNum={r['stringNum']}"), 1.0), (h(f"string={r['string']}"), 1.0)):
            expect[k] = expect.get(k, 0.0) + v
        nz = {int(j): X[i, j] for j in np.nonzero(X[i])[0]}
        assert nz == pytest.approx(expect)
    # the index of the numeric column in Spark's documented example (FeatureHasher scaladoc)
    assert h("real") == 174475
    # numeric column treated as categorical; nulls skipped; collisions add up with small numFeatures
    df2 = spark.createDataFrame([(1.0, 3), (2.0, 3), (None, 4)], "a double, b int")
    X2 = _vecs(FeatureHasher(inputCols=["a", "b"], categoricalCols=["b"], numFeatures=16,
                             outputCol="f").transform(df2), "f")
    for i, (a, b) in enumerate([(1.0, 3), (2.0, 3), (None, 4)]):
        e = np.zeros(16)
        if a is not None:
            e[murmur3_32(b"a", 42) % 16] += a
        e[murmur3_32(f"b={b}".encode(), 42) % 16] += 1.0
        np.testing.assert_allclose(X2[i], e)


def test_vector_size_hint(spark):
    df = VectorAssembler(inputCols=["a", "b"], outputCol="v").transform(
        spark.createDataFrame(pd.DataFrame({"a": [1.0, 2.0], "b": [3.0, 4.0]})))
    out = VectorSizeHint(inputCol="v", size=2).transform(df)
    assert out.schema["v"].metadata["ml_attr"]["num_attrs"] == 2
    with pytest.raises(ValueError):
        VectorSizeHint(inputCol="v", size=3).transform(df)
    assert VectorSizeHint(inputCol="v", size=3, handleInvalid="skip").transform(df).count() == 0
    assert VectorSizeHint(inputCol="v", size=3, handleInvalid="optimistic").transform(df).count() == 2


@pytest.mark.parametrize("v,s", [(1.0, "1.0"), (0.001, "0.001"), (1e-4, "1.0E-4"), (1e7, "1.0E7"),
                                 (12345678.9, "1.23456789E7"), (-2.5, "-2.5"), (100.0, "100.0"),
                                 (1234567.0, "1234567.0"), (float("nan"), "NaN"), (-0.0, "-0.0"),
                                 (1e21, "1.0E21"), (0.5, "0.5")])
def test_java_double_str(v, s):
    assert java_double_str(v) == s
