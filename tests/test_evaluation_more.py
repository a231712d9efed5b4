"""MultilabelClassificationEvaluator and RankingEvaluator on Spark's documented examples
(MultilabelMetrics / RankingMetrics suites) and hand-computed values."""
import math

import pytest

from helpers import session
from clustermachinelearningforhospitalnetworks_apache_spark_amd.ml.evaluation import (
    MultilabelClassificationEvaluator, RankingEvaluator)


@pytest.fixture(scope="module")
def spark():
    return session()


def test_multilabel_spark_example(spark):
    # Spark's MultilabelMetricsSuite data
    rows = [([0.0, 1.0], [0.0, 2.0]), ([0.0, 2.0], [0.0, 1.0]), ([], [0.0]), ([2.0], [2.0]),
            ([2.0, 0.0], [2.0, 0.0]), ([0.0, 1.0, 2.0], [0.0, 1.0]), ([1.0], [1.0, 2.0])]
    df = spark.createDataFrame(rows, "prediction ARRAY<DOUBLE>, label ARRAY<DOUBLE>")
    ev = lambda m, **kw: MultilabelClassificationEvaluator(metricName=m, **kw).evaluate(df)  # noqa: E731
    num_docs, num_labels = 7.0, 3.0
    assert ev("subsetAccuracy") == pytest.approx(2.0 / num_docs)
    assert ev("accuracy") == pytest.approx((1.0 / 3 + 1.0 / 3 + 0 + 1 + 1 + 2.0 / 3 + 1.0 / 2) / num_docs)
    assert ev("hammingLoss") == pytest.approx((2 + 2 + 1 + 0 + 0 + 1 + 1) / (num_docs * num_labels))
    assert ev("precision") == pytest.approx((1.0 / 2 + 1.0 / 2 + 0 + 1 + 1 + 2.0 / 3 + 1) / num_docs)
    assert ev("recall") == pytest.approx((1.0 / 2 + 1.0 / 2 + 0 + 1 + 1 + 1 + 1.0 / 2) / num_docs)
    assert ev("f1Measure") == pytest.approx((2.0 / 4 + 2.0 / 4 + 0 + 1 + 1 + 4.0 / 5 + 2.0 / 3) / num_docs)
    tp, fp, fn = 8.0, 3.0, 4.0  # Σ|P∩L|, Σ|P-L|, Σ|L-P|
    assert ev("microPrecision") == pytest.approx(tp / (tp + fp))
    assert ev("microRecall") == pytest.approx(tp / (tp + fn))
    assert ev("microF1Measure") == pytest.approx(2 * tp / (2 * tp + fp + fn))
    # label 0: tp 4, fp 0, fn 1
    assert ev("precisionByLabel", metricLabel=0.0) == pytest.approx(1.0)
    assert ev("recallByLabel", metricLabel=0.0) == pytest.approx(4.0 / 5)
    assert not MultilabelClassificationEvaluator(metricName="hammingLoss").isLargerBetter()


def test_ranking_spark_example(spark):
    # Spark's RankingMetricsSuite data
    rows = [([1.0, 6.0, 2.0, 7.0, 8.0, 3.0, 9.0, 10.0, 4.0, 5.0], [1.0, 2.0, 3.0, 4.0, 5.0]),
            ([4.0, 1.0, 5.0, 6.0, 2.0, 7.0, 3.0, 8.0, 9.0, 10.0], [1.0, 2.0, 3.0]),
            ([1.0, 2.0, 3.0, 4.0, 5.0], [])]
    df = spark.createDataFrame(rows, "prediction ARRAY<DOUBLE>, label ARRAY<DOUBLE>")
    ev = lambda m, k=10: RankingEvaluator(metricName=m, k=k).evaluate(df)  # noqa: E731
    assert ev("precisionAtK", 1) == pytest.approx(1.0 / 3)
    assert ev("precisionAtK", 2) == pytest.approx(1.0 / 3)
    assert ev("precisionAtK", 3) == pytest.approx(1.0 / 3)
    assert ev("precisionAtK", 4) == pytest.approx(0.75 / 3)
    assert ev("precisionAtK", 5) == pytest.approx(0.8 / 3)
    assert ev("precisionAtK", 10) == pytest.approx(0.8 / 3)
    assert ev("meanAveragePrecision") == pytest.approx(0.355026, abs=1e-6)
    assert ev("ndcgAtK", 3) == pytest.approx(1.0 / 3)
    assert ev("ndcgAtK", 5) == pytest.approx(0.328788, abs=1e-6)
    assert ev("ndcgAtK", 10) == pytest.approx(0.487913, abs=1e-6)
