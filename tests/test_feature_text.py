"""Text features on Spark's documented examples; HashingTF's MurmurHash3 (standard test vectors),
IDF formula, CountVectorizer vocabulary rules, persistence."""
import numpy as np
import pytest

from helpers import session
from clustermachinelearningforhospitalnetworks_apache_spark_amd.ml import util as U
from clustermachinelearningforhospitalnetworks_apache_spark_amd.ml.feature import (
    IDF, CountVectorizer, CountVectorizerModel, HashingTF, NGram, RegexTokenizer, StopWordsRemover, Tokenizer)
from clustermachinelearningforhospitalnetworks_apache_spark_amd.ml.feature_text import murmur3_32


@pytest.fixture(scope="module")
def spark():
    return session()


def test_murmur3_vectors():
    assert murmur3_32(b"", 0) == 0
    assert murmur3_32(b"hello", 0) & 0xFFFFFFFF == 0x248BFA47
    assert murmur3_32(b"The quick brown fox jumps over the lazy dog", 0) & 0xFFFFFFFF == 0x2E4FF723


def test_tokenizers_stopwords_ngram(spark):
    df = spark.createDataFrame([(0, "Hi I heard about Spark"), (1, "I wish Java could use case classes"),
                                (2, "Logistic,regression,models,are,neat")], "id INT, sentence STRING")
    t = Tokenizer(inputCol="sentence", outputCol="words").transform(df)
    assert [len(r.words) for r in t.collect()] == [5, 7, 1]
    rt = RegexTokenizer(inputCol="sentence", outputCol="words", pattern="\\W").transform(df)
    assert [len(r.words) for r in rt.collect()] == [5, 7, 5]
    sw = spark.createDataFrame([(0, ["I", "saw", "the", "red", "balloon"]), (1, ["Mary", "had", "a", "little", "lamb"])],
                               "id INT, raw ARRAY<STRING>")
    out = StopWordsRemover(inputCol="raw", outputCol="filtered").transform(sw).collect()
    assert [r.filtered for r in out] == [["saw", "red", "balloon"], ["Mary", "little", "lamb"]]
    ng = NGram(n=2, inputCol="words", outputCol="ngrams").transform(t).collect()[0].ngrams
    assert ng == ["hi i", "i heard", "heard about", "about spark"]


def test_hashing_tf_idf(spark, tmp_path):
    docs = [["a", "b", "a"], ["b", "c"], ["d"]]
    df = spark.createDataFrame([(i, d) for i, d in enumerate(docs)], "id INT, words ARRAY<STRING>")
    htf = HashingTF(inputCol="words", outputCol="tf", numFeatures=32)
    tf = htf.transform(df)
    x = np.stack([v.toArray() for v in tf.toPandas()["tf"]])
    for i, d in enumerate(docs):
        ref = np.zeros(32)
        for w in d:
            ref[murmur3_32(w.encode(), 42) % 32] += 1
        np.testing.assert_array_equal(x[i], ref)
    assert htf.indexOf("a") == murmur3_32(b"a", 42) % 32
    idf = IDF(inputCol="tf", outputCol="tfidf").fit(tf)
    docf = (x > 0).sum(0)
    np.testing.assert_allclose(idf.idf.toArray(), np.log(4.0 / (docf + 1.0)))
    assert idf.numDocs == 3 and idf.docFreq == docf.tolist()
    out = np.stack([v.toArray() for v in idf.transform(tf).toPandas()["tfidf"]])
    np.testing.assert_allclose(out, x * np.log(4.0 / (docf + 1.0)))
    idf.write().overwrite().save(str(tmp_path / "idf"))
    np.testing.assert_allclose(U.load(str(tmp_path / "idf")).idf.toArray(), idf.idf.toArray())
    spark.conf.set("cml.ml.text.maxDenseBytes", "100")
    with pytest.raises(MemoryError):
        HashingTF(inputCol="words", outputCol="tf2").transform(df)
    spark.conf.set("cml.ml.text.maxDenseBytes", str(8 << 30))


def test_count_vectorizer(spark, tmp_path):
    df = spark.createDataFrame([(0, "a b c".split(" ")), (1, "a b b c a".split(" "))], "id INT, words ARRAY<STRING>")
    m = CountVectorizer(inputCol="words", outputCol="features", vocabSize=3, minDF=2.0).fit(df)
    assert m.vocabulary == ["a", "b", "c"]
    x = np.stack([v.toArray() for v in m.transform(df).toPandas()["features"]])
    np.testing.assert_array_equal(x, [[1, 1, 1], [2, 2, 1]])
    xb = np.stack([v.toArray() for v in m.setBinary(True).transform(df).toPandas()["features"]])
    np.testing.assert_array_equal(xb, [[1, 1, 1], [1, 1, 1]])
    assert CountVectorizer(inputCol="words", outputCol="f", vocabSize=1).fit(df).vocabulary == ["a"]
    m.write().overwrite().save(str(tmp_path / "cv"))
    assert U.load(str(tmp_path / "cv")).vocabulary == ["a", "b", "c"]
    fixed = CountVectorizerModel.from_vocabulary(["c", "a"], inputCol="words", outputCol="f")
    np.testing.assert_array_equal(np.stack([v.toArray() for v in fixed.transform(df).toPandas()["f"]]),
                                  [[1, 1], [1, 2]])
