"""FPGrowth (itemsets vs brute-force counting, association rules, transform, persistence) and
PrefixSpan (Spark's documented example)."""
from itertools import combinations

import pytest

from helpers import session
from clustermachinelearningforhospitalnetworks_apache_spark_amd.ml import util as U
from clustermachinelearningforhospitalnetworks_apache_spark_amd.ml.fpm import FPGrowth, PrefixSpan


@pytest.fixture(scope="module")
def spark():
    return session()


def test_fpgrowth_matches_bruteforce(spark, tmp_path):
    import random
    rnd = random.Random(0)
    codes = ["I10", "E11", "N18", "J44", "I50", "F32"]
    trans = [sorted(rnd.sample(codes, rnd.randint(1, 4))) for _ in range(60)]
    df = spark.createDataFrame([(i, t) for i, t in enumerate(trans)], "id INT, items ARRAY<STRING>")
    m = FPGrowth(itemsCol="items", minSupport=0.2, minConfidence=0.5).fit(df)
    got = {tuple(sorted(r.items)): r.freq for r in m.freqItemsets.collect()}
    brute = {}
    for k in range(1, 5):
        for combo in combinations(codes, k):
            c = sum(1 for t in trans if set(combo) <= set(t))
            if c >= 12:
                brute[tuple(sorted(combo))] = c
    assert got == brute
    rules = m.associationRules.collect()
    assert rules and all(r.confidence >= 0.5 for r in rules)
    r0 = rules[0]
    both = tuple(sorted(r0.antecedent + r0.consequent))
    assert r0.confidence == pytest.approx(brute[both] / brute[tuple(sorted(r0.antecedent))])
    assert r0.support == pytest.approx(brute[both] / 60)
    assert r0.lift == pytest.approx(r0.confidence / (brute[(r0.consequent[0],)] / 60))
    pred = m.transform(df).select("items", "prediction").collect()
    for row in pred:
        assert not set(row.prediction) & set(row["items"])
    p = str(tmp_path / "fp")
    m.write().overwrite().save(p)
    back = U.load(p)
    assert {tuple(sorted(r.items)): r.freq for r in back.freqItemsets.collect()} == got


def test_prefixspan_spark_example(spark):
    # the example of Spark's PrefixSpan documentation (minSupport 0.5, maxPatternLength 5)
    rows = [([[1, 2], [3]],), ([[1], [3, 2], [1, 2]],), ([[1, 2], [5]],), ([[6]],)]
    df = spark.createDataFrame(rows, "sequence ARRAY<ARRAY<INT>>")
    out = PrefixSpan(minSupport=0.5, maxPatternLength=5).findFrequentSequentialPatterns(df)
    got = sorted((str(r.sequence), r.freq) for r in out.collect())
    want = sorted([("[[1]]", 3), ("[[1], [3]]", 2), ("[[2]]", 3), ("[[3]]", 2), ("[[1, 2]]", 3)])
    assert got == want
