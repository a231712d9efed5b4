"""Word2Vec: Huffman codes against word2vec.c's construction, skip-gram training that places
co-occurring words together, Spark's transform averaging (OOV words in the denominator), and
persistence. Trained vectors are parity unpinned (Spark's XORShift stream)."""
import numpy as np
import pytest

from clustermachinelearningforhospitalnetworks_apache_spark_amd.ml.feature import Word2Vec, Word2VecModel
from clustermachinelearningforhospitalnetworks_apache_spark_amd.ml.word2vec import huffman
from clustermachinelearningforhospitalnetworks_apache_spark_amd.sql import SparkSession


@pytest.fixture(scope="module")
def spark():
    s = SparkSession.builder.appName("w2v").master("local[1]").getOrCreate()
    yield s
    s.stop()


def test_huffman_prefix_code():
    counts = [45, 13, 12, 16, 9, 5]
    counts = sorted(counts, reverse=True)
    codes, points = huffman(counts)
    strs = ["".join(map(str, c)) for c in codes]
    # prefix-free, Kraft equality (full binary tree), frequent words get short codes
    for i, a in enumerate(strs):
        for j, b in enumerate(strs):
            assert i == j or not b.startswith(a)
    assert sum(2.0 ** -len(c) for c in codes) == pytest.approx(1.0)
    lens = [len(c) for c in codes]
    assert lens == sorted(lens)
    assert sum(c * l for c, l in zip(counts, lens)) == 224   # optimal (textbook example: 2.24 bits/sym)
    for p in points:
        assert p[0] == len(counts) - 2                        # every path starts at the root
        assert all(0 <= x <= len(counts) - 2 for x in p)


def _corpus(rs, n=400):
    a = ["icu", "ventilator", "sedation", "intubation"]
    b = ["maternity", "delivery", "newborn", "midwife"]
    out = []
    for i in range(n):
        grp = a if i % 2 == 0 else b
        out.append((list(rs.choice(grp, size=8)),))
    return out


def test_word2vec_similarity_and_transform(spark, tmp_path):
    rs = np.random.RandomState(0)
    df = spark.createDataFrame(_corpus(rs), "text array<string>")
    w2v = Word2Vec(vectorSize=16, minCount=1, seed=42, inputCol="text", outputCol="vec", maxIter=5, windowSize=3,
                   stepSize=0.05)
    model = w2v.fit(df)
    vecs = {r.word: r.vector.toArray() for r in model.getVectors().collect()}
    assert len(vecs) == 8 and all(v.shape == (16,) for v in vecs.values())
    syn = [w for w, _ in model.findSynonymsArray("icu", 3)]
    assert set(syn) <= {"ventilator", "sedation", "intubation"}
    syn2 = [r.word for r in model.findSynonyms("delivery", 3).collect()]
    assert set(syn2) <= {"maternity", "newborn", "midwife"}
    # transform: sum of known word vectors / sentence length (OOV words count)
    t = spark.createDataFrame([(["icu", "sedation", "zzz"],), ([],)], "text array<string>")
    out = [r.vec.toArray() for r in model.transform(t).collect()]
    np.testing.assert_allclose(out[0], (vecs["icu"] + vecs["sedation"]) / 3.0, rtol=1e-6)
    np.testing.assert_allclose(out[1], np.zeros(16))
    p = str(tmp_path / "w2v")
    model.save(p)
    m2 = Word2VecModel.load(p)
    v2 = {r.word: r.vector.toArray() for r in m2.getVectors().collect()}
    for k in vecs:
        np.testing.assert_array_equal(v2[k], vecs[k])
    # deterministic for a seed
    again = {r.word: r.vector.toArray() for r in w2v.fit(df).getVectors().collect()}
    for k in vecs:
        np.testing.assert_array_equal(again[k], vecs[k])


def test_word2vec_min_count(spark):
    df = spark.createDataFrame([(["a", "b", "a"],), (["a", "c"],)], "text array<string>")
    m = Word2Vec(vectorSize=4, minCount=2, inputCol="text", seed=1).fit(df)
    assert [r.word for r in m.getVectors().collect()] == ["a"]
    with pytest.raises(ValueError):
        Word2Vec(vectorSize=4, minCount=5, inputCol="text").fit(df)
