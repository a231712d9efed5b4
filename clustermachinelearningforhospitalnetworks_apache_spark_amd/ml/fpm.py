"""Frequent pattern mining (pyspark.ml.fpm): FPGrowth with association rules, and PrefixSpan.

Hospital use: co-occurring diagnoses / procedures per admission (FPGrowth) and frequent ordered
care pathways (PrefixSpan). Item counting is distributed (each rank counts its transactions, one
all-gather of the count maps); the FP-tree / projected-database recursion runs on the host over the
gathered, frequency-filtered transactions — itemset mining is pointer chasing, not GPU work, and
the transaction lists of a hospital network fit host memory easily.
"""
from __future__ import annotations

import math
from collections import defaultdict
from typing import Dict, List, Optional, Tuple

from ..sql import types as T
from . import util as U
from .base import Estimator, Model

_FP_PARAMS = {
    "itemsCol": ("items", "items column name", str),
    "minSupport": (0.3, "minimal support level of a frequent pattern, in [0, 1]", float),
    "minConfidence": (0.8, "minimal confidence for generating association rules, in [0, 1]", float),
    "predictionCol": ("prediction", "prediction column name", str),
    "numPartitions": (None, "number of partitions used by parallel FP-growth", None),
}


def _gather_lists(df, col: str) -> List[list]:
    from ..sql.dataframe import column_to_python
    local = [list(v) if v is not None else [] for v in column_to_python(df._column_data(col))]
    out = []
    for part in df._comm.allgather_object(local):
        out += part
    return out


class _FPNode:
    __slots__ = ("item", "count", "parent", "children", "link")

    def __init__(self, item, parent):
        self.item, self.count, self.parent, self.children, self.link = item, 0, parent, {}, None


def _fp_growth(transactions: List[Tuple[list, int]], min_count: int) -> List[Tuple[tuple, int]]:
    """(itemset, count) of every itemset with count >= min_count; transactions carry multiplicities."""
    counts: Dict = defaultdict(int)
    for items, c in transactions:
        for it in set(items):
            counts[it] += c
    freq = {it: c for it, c in counts.items() if c >= min_count}
    if not freq:
        return []
    rank = {it: i for i, (it, _) in enumerate(sorted(freq.items(), key=lambda kv: (-kv[1], str(kv[0]))))}
    root = _FPNode(None, None)
    heads: Dict = {}
    for items, c in transactions:
        path = sorted({it for it in items if it in freq}, key=lambda it: rank[it])
        node = root
        for it in path:
            ch = node.children.get(it)
            if ch is None:
                ch = _FPNode(it, node)
                node.children[it] = ch
                ch.link = heads.get(it)
                heads[it] = ch
            ch.count += c
            node = ch
    out = []
    for it in sorted(freq, key=lambda i: -rank[i]):  # least frequent first
        out.append(((it,), freq[it]))
        cond = []
        node = heads.get(it)
        while node is not None:
            path, p = [], node.parent
            while p is not None and p.item is not None:
                path.append(p.item)
                p = p.parent
            if path:
                cond.append((path, node.count))
            node = node.link
        for sub, c in _fp_growth(cond, min_count):
            out.append((tuple(sub) + (it,), c))
    return out


class FPGrowth(Estimator):
    """Parallel FP-growth (Spark semantics): itemsets with support >= minSupport; rules X => {y}
    with confidence >= minConfidence. Items of one transaction must be unique."""
    _params = _FP_PARAMS

    def __init__(self, **kwargs):
        super().__init__(**kwargs)
        self._defaultParamMap.pop("numPartitions", None)

    def _fit(self, df):
        trans = _gather_lists(df, self.getItemsCol())
        for t in trans:
            if len(set(t)) != len(t):
                raise ValueError("FPGrowth: items in a transaction must be unique")
        n = len(trans)
        min_count = int(math.ceil(self.getMinSupport() * n))
        sets = _fp_growth([(t, 1) for t in trans], max(min_count, 1)) if n else []
        model = FPGrowthModel([(sorted(s, key=str), c) for s, c in sets], n, self._item_type(df))
        self._copyValues(model)
        return model

    def _item_type(self, df):
        dt = df.schema[self.getItemsCol()].dataType
        return dt.elementType if isinstance(dt, T.ArrayType) else T.StringType()


class FPGrowthModel(Model):
    _params = _FP_PARAMS

    def __init__(self, itemsets: Optional[List[Tuple[list, int]]] = None, numTrainingRecords: int = 0,
                 itemType: Optional[T.DataType] = None):
        super().__init__()
        self._sets = list(itemsets or [])
        self._n = int(numTrainingRecords)
        self._itype = itemType or T.StringType()

    def _session(self):
        from ..sql.session import SparkSession
        return SparkSession.builder.getOrCreate()

    @property
    def freqItemsets(self):
        from ..sql.builder import rows_round_robin
        schema = T.StructType([T.StructField("items", T.ArrayType(self._itype), False),
                               T.StructField("freq", T.LongType(), False)])
        return rows_round_robin(self._session(), schema, [[list(s), int(c)] for s, c in self._sets])

    def _rules(self) -> List[Tuple[list, list, float, float, float]]:
        freq = {frozenset(s): c for s, c in self._sets}
        single = {next(iter(k)): c for k, c in freq.items() if len(k) == 1}
        out = []
        minc = self.getMinConfidence()
        for s, c in self._sets:
            if len(s) < 2:
                continue
            for y in s:
                ante = frozenset(s) - {y}
                ca = freq.get(ante)
                if not ca:
                    continue
                conf = c / ca
                if conf >= minc:
                    lift = conf / (single[y] / self._n) if self._n else None
                    out.append((sorted(ante, key=str), [y], conf, lift, c / self._n if self._n else None))
        return out

    @property
    def associationRules(self):
        from ..sql.builder import rows_round_robin
        schema = T.StructType([T.StructField("antecedent", T.ArrayType(self._itype), False),
                               T.StructField("consequent", T.ArrayType(self._itype), False),
                               T.StructField("confidence", T.DoubleType(), False),
                               T.StructField("lift", T.DoubleType(), True),
                               T.StructField("support", T.DoubleType(), False)])
        return rows_round_robin(self._session(), schema, [list(r) for r in self._rules()])

    def _transform(self, df):
        from ..sql.builder import column_from_values
        from ..sql.dataframe import column_to_python
        from .feature import _replace_col
        rules = [(set(a), c[0]) for a, c, *_ in self._rules()]
        vals = column_to_python(df._column_data(self.getItemsCol()))
        out = []
        for v in vals:
            if v is None:
                out.append([])
                continue
            have = set(v)
            pred = []
            for a, y in rules:
                if a <= have and y not in have and y not in pred:
                    pred.append(y)
            out.append(pred)
        return _replace_col(df, self.getPredictionCol(),
                            column_from_values(out, T.ArrayType(self._itype), df._device))

    def _save_impl(self, path):
        import pyarrow as pa
        U.write_metadata(self, path, extra={"numTrainingRecords": self._n,
                                            "cmlItemType": self._itype.simpleString()})
        at = pa.list_(pa.string()) if isinstance(self._itype, T.StringType) else pa.list_(pa.int64())
        U.write_parquet(path, "data", pa.Table.from_pylist(
            [{"items": list(s), "freq": int(c)} for s, c in self._sets],
            schema=pa.schema([("items", at), pa.field("freq", pa.int64(), False)])))

    @classmethod
    def _load_impl(cls, path, md):
        rows = U.read_parquet(path, "data").to_pylist()
        it = T.parse_type(md.get("cmlItemType", "string"))
        m = cls([(r["items"], r["freq"]) for r in rows], md.get("numTrainingRecords", 0), it)
        U.apply_params(m, md)
        return m


# --------------------------------------------------------------------------------------------- PrefixSpan

def _contains(seq: List[frozenset], pat: List[frozenset]) -> bool:
    """Greedy leftmost embedding: each pattern itemset in the first later itemset that holds it
    (a leftmost embedding exists whenever any embedding does)."""
    pos = 0
    for iset in pat:
        while pos < len(seq) and not iset <= seq[pos]:
            pos += 1
        if pos == len(seq):
            return False
        pos += 1
    return True


def _prefixspan(db: List[List[frozenset]], min_count: int, max_len: int):
    """Frequent sequential patterns by depth-first prefix growth: a pattern grows by a new itemset
    {x} (s-extension) or by an item x ordered after the last itemset's items (i-extension), and only
    the sequences supporting the prefix are tested for its extensions (support is anti-monotone).
    ``max_len`` bounds the total item count of a pattern (Spark's maxPatternLength)."""
    key = str
    cnt: Dict = defaultdict(int)
    for seq in db:
        for it in set().union(*seq) if seq else set():
            cnt[it] += 1
    items = sorted((it for it, c in cnt.items() if c >= min_count), key=key)
    out = []

    def grow(pat: List[frozenset], ids: List[int], length: int):
        if length >= max_len:
            return
        for x in items:  # s-extensions
            newp = pat + [frozenset([x])]
            sup = [i for i in ids if _contains(db[i], newp)]
            if len(sup) >= min_count:
                out.append((newp, len(sup)))
                grow(newp, sup, length + 1)
        if pat:
            last = pat[-1]
            top = max((key(i) for i in last))
            for x in items:  # i-extensions
                if key(x) <= top:
                    continue
                newp = pat[:-1] + [last | {x}]
                sup = [i for i in ids if _contains(db[i], newp)]
                if len(sup) >= min_count:
                    out.append((newp, len(sup)))
                    grow(newp, sup, length + 1)

    grow([], list(range(len(db))), 0)
    return out


class PrefixSpan:
    """pyspark.ml.fpm.PrefixSpan: ``findFrequentSequentialPatterns(df)`` over a column of sequences
    (arrays of itemsets) -> DataFrame(sequence, freq)."""

    def __init__(self, minSupport: float = 0.1, maxPatternLength: int = 10, maxLocalProjDBSize: int = 32000000,
                 sequenceCol: str = "sequence"):
        self.minSupport, self.maxPatternLength = float(minSupport), int(maxPatternLength)
        self.maxLocalProjDBSize, self.sequenceCol = int(maxLocalProjDBSize), sequenceCol

    def setMinSupport(self, v):
        self.minSupport = float(v)
        return self

    def setMaxPatternLength(self, v):
        self.maxPatternLength = int(v)
        return self

    def setSequenceCol(self, v):
        self.sequenceCol = v
        return self

    def findFrequentSequentialPatterns(self, dataset):
        from ..sql.builder import rows_round_robin
        seqs = _gather_lists(dataset, self.sequenceCol)
        db = [[frozenset(s) for s in seq] for seq in seqs]
        n = len(db)
        min_count = max(int(math.ceil(self.minSupport * n)), 1)
        pats = _prefixspan(db, min_count, self.maxPatternLength)
        et = dataset.schema[self.sequenceCol].dataType
        it = et.elementType.elementType if isinstance(et, T.ArrayType) and isinstance(et.elementType, T.ArrayType) \
            else T.StringType()
        schema = T.StructType([T.StructField("sequence", T.ArrayType(T.ArrayType(it)), False),
                               T.StructField("freq", T.LongType(), False)])
        rows = [[[sorted(s, key=str) for s in p], int(c)] for p, c in pats]
        return rows_round_robin(dataset._session, schema, rows)


__all__ = ["FPGrowth", "FPGrowthModel", "PrefixSpan"]
