"""Word2Vec (pyspark.ml.feature.Word2Vec / Word2VecModel): skip-gram with hierarchical softmax
over a Huffman tree of the vocabulary, as in Spark's mllib Word2Vec (itself word2vec.c).

Spark semantics kept: vocabulary = words with count >= minCount ordered by count (descending; ties
by word, where Spark's order is partition dependent), sentences split into chunks of at most
maxSentenceLength in-vocabulary words, a random window shrink b ∈ [0, windowSize) per position,
the Huffman codes / inner-node points of word2vec.c, σ evaluated only for |f| < 6, linear
learning-rate decay to 1e-4·stepSize over maxIter passes, syn0 initialised uniform in
[−0.5, 0.5)/vectorSize and syn1 at zero. ``transform`` averages the vectors of a sentence's
words over its full length (out-of-vocabulary words count in the denominator), like Spark.

Device design: training runs on batches of (word, context) pairs instead of one pair at a time —
the dot products with the ≤ 40 inner nodes on each pair's path are one batched [B, L, D]
contraction, and the syn0 / syn1 updates are two ``index_add_`` scatters per batch (Hogwild-style
summation of concurrent updates, the same relaxation Spark's multi-partition training makes when it
averages partition models). The corpus is gathered to every rank and every rank trains the same
model from the same counter-based random stream (hash of (seed, pass, token position)), so the
result does not depend on the number of ranks and training needs no collectives; Word2Vec corpora
are tiny next to a device's HBM. Exact vectors are parity unpinned (Spark's XORShift stream).
"""
from __future__ import annotations

import math
from typing import Dict, List, Optional, Sequence

import numpy as np
import torch

from ..sql import types as T
from ..sql.column import ColumnData
from ..utils import rng as R
from . import util as U
from .base import Estimator, Model
from .colutil import _auto_output, _replace_col
from .linalg import DenseVector, as_array
from .param import NO_DEFAULT

MAX_EXP = 6.0
_BATCH_TOKENS = 4096

_W2V_PARAMS = {
    "inputCol": (NO_DEFAULT, "input column name", str),
    "outputCol": ("__auto__", "output column name", str),
    "vectorSize": (100, "the dimension of codes after transforming from words. Should be > 0.", int),
    "minCount": (5, "the minimum number of times a token must appear to be included in the word2vec model's "
                    "vocabulary. Should be >= 0.", int),
    "numPartitions": (1, "number of partitions for sentences of words. Should be > 0.", int),
    "stepSize": (0.025, "Step size to be used for each iteration of optimization (>= 0).", float),
    "maxIter": (1, "max number of iterations (>= 0)", int),
    "seed": (None, "random seed", None),
    "windowSize": (5, "the window size (context words from [-window, window]). Should be > 0.", int),
    "maxSentenceLength": (1000, "Maximum length (in words) of each sentence in the input data. Any sentence "
                                "longer than this threshold will be divided into chunks up to the size. Should be "
                                "> 0.", int),
}


def huffman(counts: Sequence[int]):
    """word2vec.c's CreateBinaryTree over counts sorted descending: per word its code bits and the
    inner-node points (root first), as lists."""
    V = len(counts)
    if V == 0:
        return [], []
    if V == 1:
        return [[0]], [[0]]
    cnt = np.concatenate([np.asarray(counts, dtype=np.int64), np.full(V, 10 ** 15, dtype=np.int64)])
    parent = np.zeros(2 * V, dtype=np.int64)
    binary = np.zeros(2 * V, dtype=np.int64)
    pos1, pos2 = V - 1, V
    for a in range(V - 1):
        mins = []
        for _ in range(2):
            if pos1 >= 0 and cnt[pos1] < cnt[pos2]:
                mins.append(pos1)
                pos1 -= 1
            else:
                mins.append(pos2)
                pos2 += 1
        cnt[V + a] = cnt[mins[0]] + cnt[mins[1]]
        parent[mins[0]] = V + a
        parent[mins[1]] = V + a
        binary[mins[1]] = 1
    codes, points = [], []
    root = 2 * V - 2
    for a in range(V):
        code, point = [], []
        b = a
        while True:
            code.append(int(binary[b]))
            point.append(int(b))
            b = int(parent[b])
            if b == root:
                break
        n = len(code)
        c = [0] * n
        p = [0] * (n + 1)
        p[0] = V - 2
        for i in range(n):
            c[n - i - 1] = code[i]
            p[n - i] = point[i] - V
        codes.append(c)
        points.append(p[:n])
    return codes, points


class Word2Vec(Estimator):
    _params = _W2V_PARAMS

    def __init__(self, vectorSize=None, minCount=None, numPartitions=None, stepSize=None, maxIter=None, seed=None,
                 inputCol=None, outputCol=None, windowSize=None, maxSentenceLength=None):
        super().__init__(vectorSize=vectorSize, minCount=minCount, numPartitions=numPartitions, stepSize=stepSize,
                         maxIter=maxIter, seed=seed, inputCol=inputCol, outputCol=outputCol, windowSize=windowSize,
                         maxSentenceLength=maxSentenceLength)
        self._defaultParamMap.pop("seed", None)
        _auto_output(self)

    def _fit(self, df):
        from ..sql.dataframe import column_to_python
        from .tree_models import _default_seed
        seed = int(self.getOrDefault("seed")) if self.isSet("seed") else _default_seed(U.jvm_class(self))
        D, window, alpha0 = self.getVectorSize(), self.getWindowSize(), self.getStepSize()
        iters, max_len = self.getMaxIter(), self.getMaxSentenceLength()
        local = [s for s in column_to_python(df._column_data(self.getInputCol())) if s]
        sents: List[List[str]] = [w for part in df._comm.allgather_object(local) for w in part]
        counts: Dict[str, int] = {}
        for s in sents:
            for w in s:
                counts[w] = counts.get(w, 0) + 1
        vocab = sorted((w for w, c in counts.items() if c >= self.getMinCount()), key=lambda w: (-counts[w], w))
        if not vocab:
            raise ValueError("Word2Vec: the vocabulary is empty (lower minCount)")
        index = {w: i for i, w in enumerate(vocab)}
        V = len(vocab)
        codes, points = huffman([counts[w] for w in vocab])
        L = max(len(c) for c in codes)
        dev = df._device
        code_t = torch.zeros((V, L), dtype=torch.float64)
        point_t = torch.zeros((V, L), dtype=torch.int64)
        mask_t = torch.zeros((V, L), dtype=torch.float64)
        for i, (c, p) in enumerate(zip(codes, points)):
            code_t[i, :len(c)] = torch.as_tensor(c, dtype=torch.float64)
            point_t[i, :len(p)] = torch.as_tensor(p)
            mask_t[i, :len(c)] = 1.0
        code_t, point_t, mask_t = code_t.to(dev), point_t.to(dev), mask_t.to(dev)
        # token stream: in-vocabulary words, sentences chunked to maxSentenceLength
        toks = [index[w] for s in sents for w in s if w in index]
        # sentence-chunk boundaries as per-token (start, end) offsets
        starts, ends = self._bounds(sents, index, max_len)
        tok = torch.as_tensor(np.asarray(toks, dtype=np.int64), device=dev)
        st = torch.as_tensor(starts, device=dev)
        en = torch.as_tensor(ends, device=dev)
        ntok = int(tok.shape[0])
        gen = np.random.default_rng(seed & 0xFFFFFFFF)
        syn0 = torch.as_tensor((gen.random((V, D)) - 0.5) / D, device=dev)
        syn1 = torch.zeros((max(V - 1, 1), D), dtype=torch.float64, device=dev)
        total = iters * ntok + 1
        done = 0
        pos_all = torch.arange(ntok, device=dev)
        for it in range(iters):
            shrink = torch.floor(R.uniform(pos_all, seed, 7919 + it) * window).to(torch.int64)
            for a in range(0, ntok, _BATCH_TOKENS):
                pos = pos_all[a:a + _BATCH_TOKENS]
                alpha = max(alpha0 * (1.0 - done / total), alpha0 * 1e-4)
                word, ctx = [], []
                for off in range(-window, window + 1):
                    if off == 0:
                        continue
                    c = pos + off
                    ok = (abs(off) <= window - shrink[pos]) & (c >= st[pos]) & (c < en[pos])
                    word.append(tok[pos[ok]])
                    ctx.append(tok[c[ok]])
                done += int(pos.shape[0])
                if not word:
                    continue
                w = torch.cat(word)
                cx = torch.cat(ctx)
                if w.numel() == 0:
                    continue
                self._step(syn0, syn1, w, cx, code_t, point_t, mask_t, alpha)
        model = Word2VecModel(vocab, syn0.to(torch.float32).cpu().numpy())
        self._copyValues(model)
        return model

    @staticmethod
    def _bounds(sents, index, max_len):
        starts, ends = [], []
        at = 0
        for s in sents:
            n = sum(1 for w in s if w in index)
            for a in range(0, n, max_len):
                m = min(max_len, n - a)
                starts.extend([at] * m)
                ends.extend([at + m] * m)
                at += m
        return np.asarray(starts, dtype=np.int64), np.asarray(ends, dtype=np.int64)

    @staticmethod
    def _step(syn0, syn1, word, ctx, code_t, point_t, mask_t, alpha):
        """One batched hierarchical-softmax update for the pairs (word, context word)."""
        l1 = syn0[ctx]                                  # [B, D]
        pts = point_t[word]                             # [B, L]
        s1 = syn1[pts]                                  # [B, L, D]
        f = torch.einsum("bd,bld->bl", l1, s1)
        m = mask_t[word] * ((f > -MAX_EXP) & (f < MAX_EXP)).to(f.dtype)
        g = (1.0 - code_t[word] - torch.sigmoid(f)) * alpha * m   # [B, L]
        neu1e = torch.einsum("bl,bld->bd", g, s1)
        syn1.index_add_(0, pts.reshape(-1), (g[:, :, None] * l1[:, None, :]).reshape(-1, l1.shape[1]))
        syn0.index_add_(0, ctx, neu1e)


class Word2VecModel(Model):
    _params = _W2V_PARAMS

    def __init__(self, vocab: Optional[List[str]] = None, vectors=None):
        super().__init__()
        self._vocab = list(vocab or [])
        self._vec = np.asarray(vectors if vectors is not None else np.zeros((0, 0)), dtype=np.float32)
        self._index = {w: i for i, w in enumerate(self._vocab)}

    def getVectors(self):
        from ..sql.builder import rows_round_robin
        from ..sql.session import SparkSession
        schema = T.StructType([T.StructField("word", T.StringType(), True), T.StructField("vector", T.VectorUDT(), True)])
        return rows_round_robin(SparkSession.builder.getOrCreate(), schema,
                                [[w, DenseVector(self._vec[i].astype(np.float64))] for i, w in enumerate(self._vocab)])

    def _synonyms(self, word, num: int):
        if isinstance(word, str):
            if word not in self._index:
                raise ValueError(f"{word} not in vocabulary")
            q = self._vec[self._index[word]].astype(np.float64)
            exclude = word
        else:
            q = np.asarray(as_array(word), dtype=np.float64)
            exclude = None
        M = self._vec.astype(np.float64)
        norms = np.linalg.norm(M, axis=1)
        qn = np.linalg.norm(q)
        sim = (M @ q) / np.where(norms * qn == 0, 1.0, norms * qn)
        order = np.argsort(-sim, kind="stable")
        out = []
        for i in order:
            if self._vocab[i] == exclude:
                continue
            out.append((self._vocab[i], float(sim[i])))
            if len(out) == num:
                break
        return out

    def findSynonymsArray(self, word, num: int):
        return self._synonyms(word, num)

    def findSynonyms(self, word, num: int):
        from ..sql.builder import rows_round_robin
        from ..sql.session import SparkSession
        schema = T.StructType([T.StructField("word", T.StringType(), True),
                               T.StructField("similarity", T.DoubleType(), True)])
        return rows_round_robin(SparkSession.builder.getOrCreate(), schema, [list(r) for r in self._synonyms(word, num)])

    def _transform(self, df):
        from ..sql.dataframe import column_to_python
        sents = column_to_python(df._column_data(self.getInputCol()))
        D = self._vec.shape[1] if self._vec.ndim == 2 else self.getVectorSize()
        n = len(sents)
        rows, cols, w = [], [], []
        for r, s in enumerate(sents):
            if not s:
                continue
            inv = 1.0 / len(s)
            for word in s:
                i = self._index.get(word)
                if i is not None:
                    rows.append(r)
                    cols.append(i)
                    w.append(inv)
        dev = df._device
        E = torch.as_tensor(self._vec.astype(np.float64), device=dev)
        out = torch.zeros((n, D), dtype=torch.float64, device=dev)
        if rows:
            r_t = torch.as_tensor(rows, device=dev)
            out.index_add_(0, r_t, E[torch.as_tensor(cols, device=dev)] * torch.as_tensor(w, dtype=torch.float64,
                                                                                          device=dev)[:, None])
        return _replace_col(df, self.getOutputCol(), ColumnData(out, None, T.VectorUDT()))

    def _save_impl(self, path):
        import pyarrow as pa
        U.write_metadata(self, path)
        U.write_parquet(path, "data", pa.table({"word": pa.array(self._vocab, type=pa.string()),
                                                "vector": pa.array([v.tolist() for v in self._vec],
                                                                   type=pa.list_(pa.float32()))}))

    @classmethod
    def _load_impl(cls, path, md):
        t = U.read_parquet(path, "data").to_pydict()
        m = cls(t["word"], np.asarray(t["vector"], dtype=np.float32))
        U.apply_params(m, md)
        return m


__all__: List[str] = ["Word2Vec", "Word2VecModel", "huffman"]
