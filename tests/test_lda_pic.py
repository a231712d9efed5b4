"""LDA (online variational Bayes) and PowerIterationClustering.

Parity is unpinned (Spark's Breeze / XORShift random streams are not reproducible); the tests
check (1) the batched device E-step against Spark's per-document loop written out in numpy,
(2) recovery of planted topics / planted graph clusters, (3) persistence round trips."""
import numpy as np
import pandas as pd
import pytest
import torch

from clustermachinelearningforhospitalnetworks_apache_spark_amd.ml.clustering import (
    LDA, LocalLDAModel, PowerIterationClustering)
from clustermachinelearningforhospitalnetworks_apache_spark_amd.ml.feature import VectorAssembler
from clustermachinelearningforhospitalnetworks_apache_spark_amd.ml.lda import dirichlet_expectation, e_step
from clustermachinelearningforhospitalnetworks_apache_spark_amd.sql import SparkSession
from scipy.special import digamma


@pytest.fixture(scope="module")
def spark():
    s = SparkSession.builder.appName("ldapic").master("local[1]").getOrCreate()
    yield s
    s.stop()


def _spark_doc_loop(cts, e_beta, alpha, gamma0):
    """OnlineLDAOptimizer.variationalTopicInference for one document, verbatim in numpy."""
    ids = np.nonzero(cts)[0]
    c = cts[ids]
    eb = e_beta[:, ids].T                      # [ids, k]
    g = gamma0.copy()
    et = np.exp(digamma(g) - digamma(g.sum()))
    phinorm = eb @ et + 1e-100
    change = 1.0
    while change > 1e-3:
        last = g.copy()
        g = et * (eb.T @ (c / phinorm)) + alpha
        et = np.exp(digamma(g) - digamma(g.sum()))
        phinorm = eb @ et + 1e-100
        change = np.abs(g - last).sum() / g.shape[0]
    ss = np.zeros_like(e_beta)
    ss[:, ids] = np.outer(et, c / phinorm)
    return g, ss


def test_batched_e_step_matches_per_document_loop():
    rs = np.random.RandomState(0)
    k, V, B = 4, 25, 12
    lam = rs.gamma(100, 0.01, size=(k, V)) + rs.rand(k, V) * 3
    e_beta = np.exp(digamma(lam) - digamma(lam.sum(1, keepdims=True)))
    alpha = np.full(k, 0.3)
    X = rs.poisson(1.5, size=(B, V)).astype(float)
    g0 = rs.gamma(100, 0.01, size=(B, k))
    g, ss, _, _ = e_step(torch.as_tensor(X), torch.as_tensor(e_beta), torch.as_tensor(alpha), torch.as_tensor(g0))
    ref_ss = np.zeros((k, V))
    for i in range(B):
        gi, si = _spark_doc_loop(X[i], e_beta, alpha, g0[i])
        np.testing.assert_allclose(g[i].numpy(), gi, rtol=1e-10)
        ref_ss += si
    np.testing.assert_allclose(ss.numpy(), ref_ss, rtol=1e-10)
    np.testing.assert_allclose(dirichlet_expectation(torch.as_tensor(lam)).numpy(),
                               digamma(lam) - digamma(lam.sum(1, keepdims=True)), rtol=1e-12)


def _corpus(spark, n_docs=240, k=3, block=8, seed=1):
    rs = np.random.RandomState(seed)
    V = k * block
    rows, topic = [], []
    for d in range(n_docs):
        t = d % k
        p = np.full(V, 0.01)
        p[t * block:(t + 1) * block] = 1.0
        rows.append(rs.multinomial(40, p / p.sum()).astype(float))
        topic.append(t)
    cols = [f"w{i}" for i in range(V)]
    df = VectorAssembler(inputCols=cols, outputCol="features").transform(
        spark.createDataFrame(pd.DataFrame(np.array(rows), columns=cols)))
    return df, np.array(topic), V


def test_lda_recovers_planted_topics(spark, tmp_path):
    df, topic, V = _corpus(spark)
    lda = LDA(k=3, maxIter=60, seed=7, subsamplingRate=0.5, learningOffset=8.0)
    model = lda.fit(df)
    assert model.vocabSize() == V and not model.isDistributed()
    tops = model.describeTopics(8).collect()
    assert [r.topic for r in tops] == [0, 1, 2]
    blocks = sorted({min(r.termIndices) // 8 for r in tops})
    for r in tops:
        assert len({i // 8 for i in r.termIndices}) == 1           # each topic = one planted block
        assert abs(sum(r.termWeights) - 1.0) < 0.2
    assert blocks == [0, 1, 2]
    td = np.stack([v.toArray() for v in model.transform(df).toPandas()["topicDistribution"]])
    np.testing.assert_allclose(td.sum(1), 1.0, rtol=1e-12)
    lab = td.argmax(1)
    for t in range(3):                                             # documents of a planted topic agree
        vals, cnt = np.unique(lab[topic == t], return_counts=True)
        assert cnt.max() / cnt.sum() > 0.95
    ll = model.logLikelihood(df)
    lp = model.logPerplexity(df)
    assert np.isfinite(ll) and ll < 0 and lp == pytest.approx(-ll / float(240 * 40), rel=1e-12)
    # a model fitted for one iteration explains the corpus worse
    weak = LDA(k=3, maxIter=1, seed=7, subsamplingRate=0.05).fit(df)
    assert weak.logLikelihood(df) < ll
    assert model.topicsMatrix().numRows == V and model.topicsMatrix().numCols == 3
    assert len(model.estimatedDocConcentration()) == 3
    p = str(tmp_path / "lda")
    model.save(p)
    m2 = LocalLDAModel.load(p)
    np.testing.assert_array_equal(m2.topicsMatrix().toArray(), model.topicsMatrix().toArray())
    td2 = np.stack([v.toArray() for v in m2.transform(df).toPandas()["topicDistribution"]])
    np.testing.assert_allclose(td2, td, rtol=1e-12)


def test_lda_rejects_bad_optimizer(spark):
    df, _, _ = _corpus(spark, n_docs=12)
    with pytest.raises(ValueError):
        LDA(k=2, optimizer="gibbs").fit(df)
    with pytest.raises(ValueError):
        LDA(k=2, optimizer="em", docConcentration=[0.5]).fit(df)


def _spark_em_iteration(X, ndoc, nterm, alpha, eta):
    """One EMLDAOptimizer iteration written per edge (computePTopic), in numpy."""
    V, k = nterm.shape
    nk = nterm.sum(0)
    nd, nt = np.zeros_like(ndoc), np.zeros_like(nterm)
    for j, w in zip(*np.nonzero(X)):
        g = (nterm[w] + eta - 1) * (ndoc[j] + alpha - 1) / (nk + V * (eta - 1))
        g = g / g.sum() * X[j, w]
        nd[j] += g
        nt[w] += g
    return nd, nt


def test_em_dense_update_matches_edge_loop():
    rs = np.random.RandomState(1)
    n, V, k, alpha, eta = 9, 7, 3, 50.0 / 3 + 1, 1.1
    X = rs.poisson(1.0, size=(n, V)).astype(float)
    ndoc = rs.rand(n, k) * 3
    nterm = rs.rand(V, k) * 3
    A = ndoc + alpha - 1
    B = (nterm + eta - 1) / (nterm.sum(0) + V * (eta - 1))
    Q = np.where(X > 0, X / (A @ B.T), 0.0)
    nd_ref, nt_ref = _spark_em_iteration(X, ndoc, nterm, alpha, eta)
    np.testing.assert_allclose(A * (Q @ B), nd_ref, rtol=1e-12)
    np.testing.assert_allclose(B * (Q.T @ A), nt_ref, rtol=1e-12)


def test_lda_em_distributed_model(spark, tmp_path):
    from clustermachinelearningforhospitalnetworks_apache_spark_amd.ml.clustering import DistributedLDAModel
    df, topic, V = _corpus(spark)
    m = LDA(k=3, maxIter=30, seed=4, optimizer="em").fit(df)
    assert isinstance(m, DistributedLDAModel) and m.isDistributed()
    tops = m.describeTopics(8).collect()
    assert sorted({min(r.termIndices) // 8 for r in tops}) == [0, 1, 2]
    for r in tops:
        assert len({i // 8 for i in r.termIndices}) == 1
    # counts: every token is assigned once
    assert m.topicsMatrix().toArray().sum() == pytest.approx(240 * 40, rel=1e-9)
    few = LDA(k=3, maxIter=2, seed=4, optimizer="em").fit(df)
    assert m.trainingLogLikelihood + m.logPrior() >= few.trainingLogLikelihood + few.logPrior()
    loc = m.toLocal()
    assert not loc.isDistributed()
    td = np.stack([v.toArray() for v in loc.transform(df).toPandas()["topicDistribution"]])
    lab = td.argmax(1)
    for t in range(3):
        vals, cnt = np.unique(lab[topic == t], return_counts=True)
        assert cnt.max() / cnt.sum() > 0.95
    p = str(tmp_path / "em")
    m.save(p)
    m2 = DistributedLDAModel.load(p)
    np.testing.assert_array_equal(m2.topicsMatrix().toArray(), m.topicsMatrix().toArray())
    assert m2.trainingLogLikelihood == m.trainingLogLikelihood


def _two_cliques(spark, weak=0.01):
    edges = []
    for base, wt in ((0, 1.0), (10, 3.0)):
        for i in range(base, base + 6):
            for j in range(i + 1, base + 6):
                edges.append((i, j, wt))
    edges.append((5, 10, weak))
    edges.append((3, 3, 5.0))  # self loop: ignored
    return spark.createDataFrame(edges, "src long, dst long, weight double")


@pytest.mark.parametrize("mode", ["degree", "random"])
def test_pic_separates_cliques(spark, mode):
    df = _two_cliques(spark)
    out = PowerIterationClustering(k=2, maxIter=40, initMode=mode, weightCol="weight").assignClusters(df)
    rows = sorted((r.id, r.cluster) for r in out.collect())
    assert [i for i, _ in rows] == list(range(6)) + list(range(10, 16))
    a = {c for i, c in rows if i < 10}
    b = {c for i, c in rows if i >= 10}
    assert len(a) == 1 and len(b) == 1 and a != b


def test_pic_params_persist(spark, tmp_path):
    pic = PowerIterationClustering(k=3, maxIter=7, initMode="degree", srcCol="a", dstCol="b")
    p = str(tmp_path / "pic")
    pic.save(p)
    q = PowerIterationClustering.load(p)
    assert (q.getK(), q.getMaxIter(), q.getInitMode(), q.getSrcCol(), q.getDstCol()) == (3, 7, "degree", "a", "b")
    with pytest.raises(ValueError):
        PowerIterationClustering(k=2, initMode="bogus").assignClusters(_two_cliques(spark))
