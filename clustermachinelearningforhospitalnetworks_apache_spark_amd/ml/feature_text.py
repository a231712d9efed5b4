"""Text features (pyspark.ml.feature) for free-text columns such as triage notes or discharge
summaries: Tokenizer, RegexTokenizer, StopWordsRemover, NGram, HashingTF, CountVectorizer, IDF.

Tokenising is string work and runs on the host per shard; the term-frequency vectors are dense
[n, numFeatures] device tensors (the frame's vector layout), built with one ``index_put_`` scatter
per shard, and IDF is one all-reduce of document frequencies plus a broadcast multiply. Dense rows
make numFeatures a memory knob here: HashingTF refuses a shard whose dense matrix would exceed
``cml.ml.text.maxDenseBytes`` (default 8 GiB) — lower numFeatures (Spark's default 2^18 is a
sparse-vector default).

HashingTF hashes UTF-8 terms with MurmurHash3 x86_32, seed 42 (Spark 3's corrected
``hashUnsafeBytes2``), index = non-negative hash mod numFeatures, so indices match Spark's.
"""
from __future__ import annotations

import re
from typing import Dict, List, Optional

import numpy as np
import torch

from ..sql import types as T
from ..sql.column import ColumnData
from . import util as U
from .base import Estimator, Model, Transformer
from .colutil import _auto_output, _replace_col
from .linalg import DenseVector
from .param import NO_DEFAULT

ENGLISH_STOP_WORDS = (
    "i me my myself we our ours ourselves you your yours yourself yourselves he him his himself she her hers herself "
    "it its itself they them their theirs themselves what which who whom this that these those am is are was were be "
    "been being have has had having do does did doing a an the and but if or because as until while of at by for "
    "with about against between into through during before after above below to from up down in out on off over "
    "under again further then once here there when where why how all any both each few more most other some such no "
    "nor not only own same so than too very s t can will just don should now i'll you'll he'll she'll we'll they'll "
    "i'd you'd he'd she'd we'd they'd i'm you're he's she's it's we're they're i've we've you've they've isn't "
    "aren't wasn't weren't haven't hasn't hadn't don't doesn't didn't won't wouldn't shan't shouldn't mustn't can't "
    "couldn't cannot could here's how's let's ought that's there's what's when's where's who's why's would").split()


def _texts(df, col: str) -> List:
    from ..sql.dataframe import column_to_python
    return column_to_python(df._column_data(col))


def _set_array(df, name: str, vals: List, elem=T.StringType()):
    out = np.empty(len(vals), dtype=object)
    for i, v in enumerate(vals):
        out[i] = v
    return _replace_col(df, name, ColumnData(out, None, T.ArrayType(elem)))


class Tokenizer(Transformer):
    """Lower-cases and splits on whitespace."""
    _params = {"inputCol": (NO_DEFAULT, "input column name", str),
               "outputCol": ("__auto__", "output column name", str)}

    def __init__(self, inputCol=None, outputCol=None):
        super().__init__(inputCol=inputCol, outputCol=outputCol)
        _auto_output(self)

    def _transform(self, df):
        return _set_array(df, self.getOutputCol(), [None if s is None else str(s).lower().split()
                                                    for s in _texts(df, self.getInputCol())])


class RegexTokenizer(Transformer):
    """Splits on ``pattern`` (gaps=True) or extracts its matches (gaps=False); drops tokens shorter
    than minTokenLength."""
    _params = {"inputCol": (NO_DEFAULT, "input column name", str),
               "outputCol": ("__auto__", "output column name", str),
               "minTokenLength": (1, "minimum token length (>= 0)", int),
               "gaps": (True, "whether regex splits on gaps (True) or matches tokens (False)", bool),
               "pattern": ("\\s+", "regex pattern used for tokenizing", str),
               "toLowercase": (True, "whether to convert all characters to lowercase before tokenizing", bool)}

    def __init__(self, minTokenLength=None, gaps=None, pattern=None, inputCol=None, outputCol=None,
                 toLowercase=None):
        super().__init__(minTokenLength=minTokenLength, gaps=gaps, pattern=pattern, inputCol=inputCol,
                         outputCol=outputCol, toLowercase=toLowercase)
        _auto_output(self)

    def _transform(self, df):
        rx = re.compile(self.getPattern())
        low, gaps, mn = self.getToLowercase(), self.getGaps(), self.getMinTokenLength()
        out = []
        for s in _texts(df, self.getInputCol()):
            if s is None:
                out.append(None)
                continue
            s = str(s).lower() if low else str(s)
            toks = rx.split(s) if gaps else rx.findall(s)
            out.append([t for t in toks if len(t) >= mn])
        return _set_array(df, self.getOutputCol(), out)


class StopWordsRemover(Transformer):
    _params = {"inputCol": (NO_DEFAULT, "input column name", str),
               "outputCol": ("__auto__", "output column name", str),
               "stopWords": (list(ENGLISH_STOP_WORDS), "the words to be filtered out", "liststr"),
               "caseSensitive": (False, "whether to do a case sensitive comparison over the stop words", bool),
               "locale": ("en_US", "locale of the input for case insensitive matching", str)}

    def __init__(self, inputCol=None, outputCol=None, stopWords=None, caseSensitive=None, locale=None):
        super().__init__(inputCol=inputCol, outputCol=outputCol, stopWords=stopWords, caseSensitive=caseSensitive,
                         locale=locale)
        _auto_output(self)

    @staticmethod
    def loadDefaultStopWords(language: str) -> List[str]:
        if language.lower() != "english":
            raise ValueError("only the english stop-word list ships with this build")
        return list(ENGLISH_STOP_WORDS)

    def _transform(self, df):
        cs = self.getCaseSensitive()
        stop = set(self.getStopWords()) if cs else {w.lower() for w in self.getStopWords()}
        out = []
        for toks in _texts(df, self.getInputCol()):
            if toks is None:
                out.append(None)
            else:
                out.append([t for t in toks if (t if cs else str(t).lower()) not in stop])
        return _set_array(df, self.getOutputCol(), out)


class NGram(Transformer):
    _params = {"inputCol": (NO_DEFAULT, "input column name", str),
               "outputCol": ("__auto__", "output column name", str),
               "n": (2, "number of elements per n-gram (>= 1)", int)}

    def __init__(self, n=None, inputCol=None, outputCol=None):
        super().__init__(n=n, inputCol=inputCol, outputCol=outputCol)
        _auto_output(self)

    def _transform(self, df):
        n = self.getN()
        out = []
        for toks in _texts(df, self.getInputCol()):
            out.append(None if toks is None else [" ".join(toks[i:i + n]) for i in range(len(toks) - n + 1)])
        return _set_array(df, self.getOutputCol(), out)


# ------------------------------------------------------------------------------------------ hashing

def murmur3_32(data: bytes, seed: int = 42) -> int:
    """MurmurHash3 x86_32 (signed 32-bit result, as Java ints)."""
    c1, c2 = 0xCC9E2D51, 0x1B873593
    h = seed & 0xFFFFFFFF
    n = len(data)
    nb = n // 4
    for i in range(nb):
        k = int.from_bytes(data[4 * i:4 * i + 4], "little")
        k = (k * c1) & 0xFFFFFFFF
        k = ((k << 15) | (k >> 17)) & 0xFFFFFFFF
        k = (k * c2) & 0xFFFFFFFF
        h ^= k
        h = ((h << 13) | (h >> 19)) & 0xFFFFFFFF
        h = (h * 5 + 0xE6546B64) & 0xFFFFFFFF
    tail = data[4 * nb:]
    k = 0
    if len(tail) >= 3:
        k ^= tail[2] << 16
    if len(tail) >= 2:
        k ^= tail[1] << 8
    if len(tail) >= 1:
        k ^= tail[0]
        k = (k * c1) & 0xFFFFFFFF
        k = ((k << 15) | (k >> 17)) & 0xFFFFFFFF
        k = (k * c2) & 0xFFFFFFFF
        h ^= k
    h ^= n
    h ^= h >> 16
    h = (h * 0x85EBCA6B) & 0xFFFFFFFF
    h ^= h >> 13
    h = (h * 0xC2B2AE35) & 0xFFFFFFFF
    h ^= h >> 16
    return h - (1 << 32) if h >= (1 << 31) else h


def _term_bytes(t) -> bytes:
    return str(t).encode("utf-8")


def _dense_budget(df, n: int, d: int, what: str) -> None:
    cap = float(df._session.conf.get("cml.ml.text.maxDenseBytes", str(8 << 30)))
    if n * d * 8 > cap:
        raise MemoryError(f"{what}: a dense [{n}, {d}] shard needs {n * d * 8 / 2**30:.1f} GiB "
                          f"(cml.ml.text.maxDenseBytes = {cap / 2**30:.1f} GiB); lower numFeatures / vocabSize")


def _scatter_counts(df, rows: List[List[int]], d: int, binary: bool, weights: Optional[List[List[float]]] = None):
    n = len(rows)
    _dense_budget(df, n, d, "term frequencies")
    x = torch.zeros((n, d), dtype=torch.float64, device=df._device)
    ri = [i for i, r in enumerate(rows) for _ in r]
    ci = [c for r in rows for c in r]
    if ci:
        vals = torch.ones(len(ci), dtype=torch.float64) if weights is None else torch.as_tensor(
            [w for r in weights for w in r], dtype=torch.float64)
        x.index_put_((torch.as_tensor(ri, device=df._device), torch.as_tensor(ci, device=df._device)),
                     vals.to(df._device), accumulate=True)
    if binary:
        x = (x > 0).to(torch.float64)
    return x


class HashingTF(Transformer):
    _params = {"inputCol": (NO_DEFAULT, "input column name", str),
               "outputCol": ("__auto__", "output column name", str),
               "numFeatures": (1 << 18, "number of features (> 0)", int),
               "binary": (False, "if True, all non zero counts are set to 1", bool)}

    def __init__(self, numFeatures=None, binary=None, inputCol=None, outputCol=None):
        super().__init__(numFeatures=numFeatures, binary=binary, inputCol=inputCol, outputCol=outputCol)
        _auto_output(self)

    def indexOf(self, term) -> int:
        return murmur3_32(_term_bytes(term), 42) % self.getNumFeatures()

    def _transform(self, df):
        d = self.getNumFeatures()
        cache: Dict = {}
        rows = []
        for toks in _texts(df, self.getInputCol()):
            r = []
            for t in toks or []:
                i = cache.get(t)
                if i is None:
                    i = cache[t] = murmur3_32(_term_bytes(t), 42) % d
                r.append(i)
            rows.append(r)
        x = _scatter_counts(df, rows, d, self.getBinary())
        return _replace_col(df, self.getOutputCol(), ColumnData(x, None, T.VectorUDT()))


class CountVectorizer(Estimator):
    """Vocabulary of the vocabSize most frequent terms (corpus term counts, ties by term) that occur in
    at least minDF and at most maxDF documents (counts, or fractions when < 1)."""
    _params = {"inputCol": (NO_DEFAULT, "input column name", str),
               "outputCol": ("__auto__", "output column name", str),
               "vocabSize": (1 << 18, "max size of the vocabulary", int),
               "minDF": (1.0, "minimum number (or fraction, < 1) of documents a term must appear in", float),
               "maxDF": (float(2 ** 63 - 1), "maximum number (or fraction, < 1) of documents a term may appear in",
                         float),
               "minTF": (1.0, "per-document minimum count (or fraction of the document's tokens, < 1)", float),
               "binary": (False, "binary toggle to control the output vector values", bool)}

    def __init__(self, minTF=None, minDF=None, maxDF=None, vocabSize=None, binary=None, inputCol=None,
                 outputCol=None):
        super().__init__(minTF=minTF, minDF=minDF, maxDF=maxDF, vocabSize=vocabSize, binary=binary,
                         inputCol=inputCol, outputCol=outputCol)
        _auto_output(self)

    def _fit(self, df):
        tc: Dict = {}
        dc: Dict = {}
        nd = 0
        for toks in _texts(df, self.getInputCol()):
            if toks is None:
                continue
            nd += 1
            for t in toks:
                tc[t] = tc.get(t, 0) + 1
            for t in set(toks):
                dc[t] = dc.get(t, 0) + 1
        TC: Dict = {}
        DC: Dict = {}
        N = 0
        for a, b, n in df._comm.allgather_object((tc, dc, nd)):
            N += n
            for k, v in a.items():
                TC[k] = TC.get(k, 0) + v
            for k, v in b.items():
                DC[k] = DC.get(k, 0) + v
        mn, mx = self.getMinDF(), self.getMaxDF()
        mn = mn * N if mn < 1.0 else mn
        mx = mx * N if mx < 1.0 else mx
        terms = [t for t in TC if mn <= DC[t] <= mx]
        terms.sort(key=lambda t: (-TC[t], str(t)))
        m = CountVectorizerModel(terms[: self.getVocabSize()])
        self._copyValues(m)
        return m


class CountVectorizerModel(Model):
    _params = CountVectorizer._params

    def __init__(self, vocabulary: Optional[List[str]] = None):
        super().__init__()
        self.vocabulary = list(vocabulary or [])

    @classmethod
    def from_vocabulary(cls, vocabulary, inputCol, outputCol=None, minTF=None, binary=None):
        m = cls(vocabulary)
        m._set(inputCol=inputCol)
        if outputCol is not None:
            m._set(outputCol=outputCol)
        if minTF is not None:
            m._set(minTF=minTF)
        if binary is not None:
            m._set(binary=binary)
        if m.getOutputCol() == "__auto__":
            m._defaultParamMap["outputCol"] = m.uid + "__output"
        return m

    def _transform(self, df):
        idx = {t: i for i, t in enumerate(self.vocabulary)}
        min_tf = self.getMinTF()
        rows = []
        for toks in _texts(df, self.getInputCol()):
            cnt: Dict[int, int] = {}
            for t in toks or []:
                i = idx.get(t)
                if i is not None:
                    cnt[i] = cnt.get(i, 0) + 1
            lim = min_tf * len(toks) if (toks and min_tf < 1.0) else min_tf
            rows.append([(i, c) for i, c in cnt.items() if c >= lim])
        x = _scatter_counts(df, [[i for i, _ in r] for r in rows], len(self.vocabulary), self.getBinary(),
                            [[float(c) for _, c in r] for r in rows])
        return _replace_col(df, self.getOutputCol(), ColumnData(x, None, T.VectorUDT()))

    def _save_impl(self, path):
        import pyarrow as pa
        U.write_metadata(self, path)
        U.write_parquet(path, "data", pa.table({"vocabulary": pa.array([self.vocabulary],
                                                                       type=pa.list_(pa.string()))}))

    @classmethod
    def _load_impl(cls, path, md):
        m = cls(U.read_parquet(path, "data").to_pylist()[0]["vocabulary"])
        U.apply_params(m, md)
        return m


class IDF(Estimator):
    """idf = log((m + 1) / (df + 1)) over m documents; terms in fewer than minDocFreq documents get 0."""
    _params = {"inputCol": (NO_DEFAULT, "input column name", str),
               "outputCol": ("__auto__", "output column name", str),
               "minDocFreq": (0, "minimum number of documents in which a term should appear for filtering", int)}

    def __init__(self, minDocFreq=None, inputCol=None, outputCol=None):
        super().__init__(minDocFreq=minDocFreq, inputCol=inputCol, outputCol=outputCol)
        _auto_output(self)

    def _fit(self, df):
        x = df._feature_matrix(self.getInputCol())
        dfreq = (x != 0).sum(0).to(torch.float64)
        msg = torch.cat([dfreq, torch.tensor([float(x.shape[0])], dtype=torch.float64, device=x.device)])
        df._comm.allreduce_(msg)
        o = msg.cpu().numpy()
        docf, m = o[:-1], o[-1]
        idf = np.where(docf >= self.getMinDocFreq(), np.log((m + 1.0) / (docf + 1.0)), 0.0)
        model = IDFModel(idf, docf.astype(np.int64), int(m))
        self._copyValues(model)
        return model


class IDFModel(Model):
    _params = IDF._params

    def __init__(self, idf=None, docFreq=None, numDocs: int = 0):
        super().__init__()
        self._idf = np.asarray(idf if idf is not None else [], dtype=np.float64)
        self._df = np.asarray(docFreq if docFreq is not None else [], dtype=np.int64)
        self._m = int(numDocs)

    @property
    def idf(self) -> DenseVector:
        return DenseVector(self._idf)

    @property
    def docFreq(self) -> List[int]:
        return self._df.tolist()

    @property
    def numDocs(self) -> int:
        return self._m

    def _transform(self, df):
        x = df._feature_matrix(self.getInputCol()).to(torch.float64)
        y = x * torch.as_tensor(self._idf, device=x.device)
        return _replace_col(df, self.getOutputCol(), ColumnData(y, None, T.VectorUDT()))

    def _save_impl(self, path):
        import pyarrow as pa
        U.write_metadata(self, path)
        U.write_parquet(path, "data", pa.Table.from_pylist(
            [{"idf": U.vector_struct(self._idf), "docFreq": self._df.tolist(), "numDocs": self._m}],
            schema=pa.schema([("idf", U.vector_arrow_type()), ("docFreq", pa.list_(pa.int64())),
                              pa.field("numDocs", pa.int64(), False)])))

    @classmethod
    def _load_impl(cls, path, md):
        r = U.read_parquet(path, "data").to_pylist()[0]
        m = cls(U.vector_from_struct(r["idf"]), r["docFreq"], r["numDocs"])
        U.apply_params(m, md)
        return m


__all__ = ["Tokenizer", "RegexTokenizer", "StopWordsRemover", "NGram", "HashingTF", "CountVectorizer",
           "CountVectorizerModel", "IDF", "IDFModel", "murmur3_32", "ENGLISH_STOP_WORDS"]
