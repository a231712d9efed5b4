"""Evaluators (ref.py:31, ref.py:33, ref.py:162-169, ref.py:192-198).

Every metric is a handful of sums computed on the rank's shard (K23: fused
device reductions) and combined with ONE all-reduce (C8) — no collect to a driver.
"""
from __future__ import annotations

import math

import numpy as np
import torch

from .base import Evaluator
from .param import NO_DEFAULT


def reg_sums_torch(y, p, w=None):
    """[Σw, Σw e², Σw |e|, Σw y, Σw y², Σw p, Σw p²] — CPU path and K23 oracle."""
    if w is None:
        w = torch.ones_like(y)
    e = y - p
    if not y.numel():
        return torch.zeros(7, dtype=torch.float64, device=y.device)
    return torch.stack([w.sum(), (w * e * e).sum(), (w * e.abs()).sum(), (w * y).sum(), (w * y * y).sum(),
                        (w * p).sum(), (w * p * p).sum()])


def _col(df, name, dtype=torch.float64):
    cd = df._column_data(name)
    if cd.is_host:
        raise TypeError(f"column {name!r} must be numeric")
    v = cd.values
    return v.to(dtype) if v.dim() == 1 else v


class RegressionEvaluator(Evaluator):
    """metricName: rmse (default) | mse | r2 | mae | var."""
    _params = {
        "predictionCol": ("prediction", "prediction column name", str),
        "labelCol": ("label", "label column name", str),
        "weightCol": (None, "weight column name", None),
        "metricName": ("rmse", "metric name in evaluation (mse|rmse|r2|mae|var)", str),
        "throughOrigin": (False, "whether the regression is through the origin", bool),
    }

    def __init__(self, predictionCol=None, labelCol=None, metricName=None, weightCol=None, throughOrigin=None):
        super().__init__(predictionCol=predictionCol, labelCol=labelCol, metricName=metricName, weightCol=weightCol,
                         throughOrigin=throughOrigin)
        self._defaultParamMap.pop("weightCol", None)

    def _evaluate(self, df) -> float:
        y = _col(df, self.getLabelCol())
        p = _col(df, self.getPredictionCol())
        w = _col(df, self.getOrDefault("weightCol")) if self.isSet("weightCol") else None
        if y.is_cuda and y.numel():
            from ..ops import frame_ops  # K23: one fused pass for all seven sums
            stats = frame_ops.reg_metric_sums(y, p, w)
        else:
            stats = reg_sums_torch(y, p, w)
        df._comm.allreduce_(stats)
        n, sse, sae, sy, syy, sp, spp = stats.tolist()
        if n == 0:
            return float("nan")
        m = self.getMetricName()
        mse = sse / n
        if m == "rmse":
            return math.sqrt(mse)
        if m == "mse":
            return mse
        if m == "mae":
            return sae / n
        if m == "r2":
            if self.getThroughOrigin():
                sst = syy
            else:
                sst = syy - sy * sy / n
            return 1.0 - sse / sst if sst > 0 else float("nan")
        if m == "var":
            return spp / n - (sp / n) ** 2
        raise ValueError(f"unknown metric {m}")

    def isLargerBetter(self) -> bool:
        return self.getMetricName() in ("r2", "var")


class MulticlassClassificationEvaluator(Evaluator):
    """metricName: f1 (default) | accuracy | weightedPrecision | weightedRecall | weightedTruePositiveRate |
    weightedFalsePositiveRate | weightedFMeasure | truePositiveRateByLabel | falsePositiveRateByLabel |
    precisionByLabel | recallByLabel | fMeasureByLabel | logLoss | hammingLoss."""
    _params = {
        "predictionCol": ("prediction", "prediction column name", str),
        "labelCol": ("label", "label column name", str),
        "weightCol": (None, "weight column name", None),
        "probabilityCol": ("probability", "probability column name", str),
        "metricName": ("f1", "metric name in evaluation", str),
        "metricLabel": (0.0, "the class whose metric will be computed in *ByLabel", float),
        "beta": (1.0, "the beta value used in fMeasureByLabel/weightedFMeasure", float),
        "eps": (1e-15, "log-loss clipping epsilon", float),
    }

    def __init__(self, predictionCol=None, labelCol=None, metricName=None, weightCol=None, metricLabel=None,
                 beta=None, probabilityCol=None, eps=None):
        super().__init__(predictionCol=predictionCol, labelCol=labelCol, metricName=metricName, weightCol=weightCol,
                         metricLabel=metricLabel, beta=beta, probabilityCol=probabilityCol, eps=eps)
        self._defaultParamMap.pop("weightCol", None)

    def _confusion(self, df):
        y = _col(df, self.getLabelCol()).to(torch.int64)
        p = _col(df, self.getPredictionCol()).to(torch.int64)
        w = _col(df, self.getOrDefault("weightCol")) if self.isSet("weightCol") else torch.ones(
            y.shape[0], dtype=torch.float64, device=y.device)
        local_max = int(max(y.max().item() if y.numel() else 0, p.max().item() if p.numel() else 0))
        C = int(df._comm.max_scalar(float(local_max))) + 1
        if y.is_cuda and y.numel() and C <= 64:
            from ..ops import frame_ops  # K23: weighted confusion counts in one pass
            cm = frame_ops.confusion(y, p, C, None if not self.isSet("weightCol") else w).reshape(-1)
        else:
            cm = torch.zeros(C * C, dtype=torch.float64, device=y.device)
            if y.numel():
                cm.index_add_(0, y * C + p, w)
        df._comm.allreduce_(cm)
        return cm.reshape(C, C).cpu().numpy()  # rows = label, cols = prediction

    def _evaluate(self, df) -> float:
        m = self.getMetricName()
        if m == "logLoss":
            return self._logloss(df)
        cm = self._confusion(df)
        total = cm.sum()
        if total == 0:
            return float("nan")
        tp = np.diag(cm)
        lab = cm.sum(1)
        pred = cm.sum(0)
        with np.errstate(divide="ignore", invalid="ignore"):
            prec = np.where(pred > 0, tp / np.where(pred > 0, pred, 1), 0.0)
            rec = np.where(lab > 0, tp / np.where(lab > 0, lab, 1), 0.0)
            fpr = np.where(total - lab > 0, (pred - tp) / np.where(total - lab > 0, total - lab, 1), 0.0)
        beta = self.getBeta()
        b2 = beta * beta
        with np.errstate(divide="ignore", invalid="ignore"):
            fm = np.where(prec + rec > 0, (1 + b2) * prec * rec / np.where(b2 * prec + rec > 0, b2 * prec + rec, 1),
                          0.0)
        wts = lab / total
        if m == "accuracy":
            return float(tp.sum() / total)
        if m in ("f1", "weightedFMeasure"):
            return float((wts * fm).sum())
        if m == "weightedPrecision":
            return float((wts * prec).sum())
        if m in ("weightedRecall", "weightedTruePositiveRate"):
            return float((wts * rec).sum())
        if m == "weightedFalsePositiveRate":
            return float((wts * fpr).sum())
        if m == "hammingLoss":
            return float(1.0 - tp.sum() / total)
        li = int(self.getMetricLabel())
        if li >= len(tp):
            return 0.0
        if m == "truePositiveRateByLabel" or m == "recallByLabel":
            return float(rec[li])
        if m == "falsePositiveRateByLabel":
            return float(fpr[li])
        if m == "precisionByLabel":
            return float(prec[li])
        if m == "fMeasureByLabel":
            return float(fm[li])
        raise ValueError(f"unknown metric {m}")

    def _logloss(self, df) -> float:
        y = _col(df, self.getLabelCol()).to(torch.int64)
        prob = df._feature_matrix(self.getProbabilityCol()).to(torch.float64)
        eps = self.getEps()
        if y.numel():
            p = prob.gather(1, y.reshape(-1, 1)).reshape(-1).clamp(eps, 1 - eps)
            s = torch.stack([-torch.log(p).sum(), torch.tensor(float(y.numel()), device=y.device,
                                                               dtype=torch.float64)])
        else:
            s = torch.zeros(2, dtype=torch.float64, device=y.device)
        df._comm.allreduce_(s)
        return float(s[0] / s[1]) if s[1] > 0 else float("nan")

    def isLargerBetter(self) -> bool:
        return self.getMetricName() not in ("weightedFalsePositiveRate", "falsePositiveRateByLabel", "logLoss",
                                            "hammingLoss")


class BinaryClassificationEvaluator(Evaluator):
    """areaUnderROC (default) | areaUnderPR, from rawPrediction/probability scores."""
    _params = {
        "rawPredictionCol": ("rawPrediction", "raw prediction (score) column", str),
        "labelCol": ("label", "label column name", str),
        "weightCol": (None, "weight column name", None),
        "metricName": ("areaUnderROC", "areaUnderROC|areaUnderPR", str),
        "numBins": (1000, "number of bins to down-sample the curves (0 = exact)", int),
    }

    def __init__(self, rawPredictionCol=None, labelCol=None, metricName=None, weightCol=None, numBins=None):
        super().__init__(rawPredictionCol=rawPredictionCol, labelCol=labelCol, metricName=metricName,
                         weightCol=weightCol, numBins=numBins)
        self._defaultParamMap.pop("weightCol", None)

    def _evaluate(self, df) -> float:
        cd = df._column_data(self.getRawPredictionCol())
        s = cd.values.to(torch.float64)
        score = s[:, -1] if s.dim() == 2 else s
        y = _col(df, self.getLabelCol())
        w = _col(df, self.getOrDefault("weightCol")) if self.isSet("weightCol") else torch.ones_like(y)
        # exact curves from the gathered (score, label, weight) triples — sorted once on the host
        parts = df._comm.allgather_object((score.cpu().numpy(), y.cpu().numpy(), w.cpu().numpy()))
        sc = np.concatenate([p[0] for p in parts])
        yy = np.concatenate([p[1] for p in parts])
        ww = np.concatenate([p[2] for p in parts])
        order = np.argsort(-sc, kind="stable")
        sc, yy, ww = sc[order], yy[order], ww[order]
        pos = (yy > 0.5) * ww
        neg = (yy <= 0.5) * ww
        # group ties
        uniq = np.r_[True, sc[1:] != sc[:-1]]
        idx = np.cumsum(uniq) - 1
        tp = np.bincount(idx, pos)
        fp = np.bincount(idx, neg)
        ctp, cfp = np.cumsum(tp), np.cumsum(fp)
        P, N = ctp[-1] if len(ctp) else 0.0, cfp[-1] if len(cfp) else 0.0
        if self.getMetricName() == "areaUnderROC":
            if P == 0 or N == 0:
                return float("nan")
            tpr = np.r_[0.0, ctp / P]
            fpr = np.r_[0.0, cfp / N]
            return float(np.trapezoid(tpr, fpr))
        if P == 0:
            return float("nan")
        rec = np.r_[0.0, ctp / P]
        prec = np.r_[1.0, ctp / np.maximum(ctp + cfp, 1e-300)]
        return float(np.trapezoid(prec, rec))


class ClusteringEvaluator(Evaluator):
    """Silhouette with squared euclidean distance (Spark's default), computed from per-cluster sums."""
    _params = {
        "predictionCol": ("prediction", "prediction column name", str),
        "featuresCol": ("features", "features column name", str),
        "metricName": ("silhouette", "metric name", str),
        "distanceMeasure": ("squaredEuclidean", "squaredEuclidean|cosine", str),
        "weightCol": (None, "weight column name", None),
    }

    def __init__(self, predictionCol=None, featuresCol=None, metricName=None, distanceMeasure=None, weightCol=None):
        super().__init__(predictionCol=predictionCol, featuresCol=featuresCol, metricName=metricName,
                         distanceMeasure=distanceMeasure, weightCol=weightCol)
        self._defaultParamMap.pop("weightCol", None)

    def _evaluate(self, df) -> float:
        x = df._feature_matrix(self.getFeaturesCol()).to(torch.float64)
        lab = _col(df, self.getPredictionCol()).to(torch.int64)
        K = int(df._comm.max_scalar(float(lab.max().item()) if lab.numel() else 0.0)) + 1
        d = x.shape[1]
        sums = torch.zeros(K, d, dtype=torch.float64, device=x.device)
        cnt = torch.zeros(K, dtype=torch.float64, device=x.device)
        sq = torch.zeros(K, dtype=torch.float64, device=x.device)
        if lab.numel():
            from ..ops.group_ops import group_reduce, group_sum_rows  # K25 on the GPU (few clusters)
            sums = group_sum_rows(lab, x, K)
            cnt = group_reduce(lab, torch.ones_like(lab, dtype=torch.uint8), K, "sum", floating=True)
            sq = group_reduce(lab, (x * x).sum(1), K, "sum")
        msg = torch.cat([sums.reshape(-1), cnt, sq])
        df._comm.allreduce_(msg)
        sums = msg[: K * d].reshape(K, d)
        cnt = msg[K * d: K * d + K]
        sq = msg[K * d + K:]
        if lab.numel() == 0:
            part = torch.zeros(2, dtype=torch.float64, device=x.device)
        else:
            xx = (x * x).sum(1, keepdim=True)
            # mean squared distance from each point to every cluster: (N_c|x|² − 2x·S_c + Q_c)/N_c
            dist = (cnt[None, :] * xx - 2 * x @ sums.T + sq[None, :]) / cnt.clamp(min=1)[None, :]
            own = dist.gather(1, lab.reshape(-1, 1)).reshape(-1)
            nc = cnt[lab]
            a = torch.where(nc > 1, own * nc / (nc - 1).clamp(min=1), torch.zeros_like(own))
            other = dist.clone()
            other[torch.arange(len(lab), device=x.device), lab] = float("inf")
            other[:, cnt == 0] = float("inf")
            b = other.min(1).values
            s = torch.where(nc > 1, (b - a) / torch.maximum(a, b).clamp(min=1e-300), torch.zeros_like(a))
            part = torch.stack([s.sum(), torch.tensor(float(len(lab)), dtype=torch.float64, device=x.device)])
        df._comm.allreduce_(part)
        return float(part[0] / part[1]) if part[1] > 0 else float("nan")


# ------------------------------------------------------------------------- multilabel / ranking

def _array_pairs(df, pred_col: str, label_col: str):
    """This rank's (prediction list, label list) pairs; metrics merge per-rank sums."""
    from ..sql.dataframe import column_to_python
    p = column_to_python(df._column_data(pred_col))
    lab = column_to_python(df._column_data(label_col))
    return [(list(a or []), list(b or [])) for a, b in zip(p, lab)]


class MultilabelClassificationEvaluator(Evaluator):
    """Spark's MultilabelMetrics over array columns of predicted and true labels: subsetAccuracy,
    accuracy, hammingLoss, precision, recall, f1Measure (default), micro*, and *ByLabel for
    ``metricLabel``. Per-rank sums, one all-gather of the small count maps."""
    _params = {
        "predictionCol": ("prediction", "prediction column name", str),
        "labelCol": ("label", "label column name", str),
        "metricName": ("f1Measure", "metric name in evaluation", str),
        "metricLabel": (0.0, "the class whose metric will be computed in *ByLabel", float),
    }

    def __init__(self, predictionCol=None, labelCol=None, metricName=None, metricLabel=None):
        super().__init__(predictionCol=predictionCol, labelCol=labelCol, metricName=metricName,
                         metricLabel=metricLabel)

    def _evaluate(self, df) -> float:
        pairs = _array_pairs(df, self.getPredictionCol(), self.getLabelCol())
        s = np.zeros(8)  # n, subset, acc, prec, rec, f1, sumTp, sumFp (sumFn below)
        fn = 0.0
        by: dict = {}
        labels = set()
        for p, lab in pairs:
            P, L = set(p), set(lab)
            inter = len(P & L)
            s[0] += 1
            s[1] += P == L
            den = len(P) + len(L) - inter
            s[2] += inter / den if den else float("nan")
            s[3] += inter / len(P) if P else 0.0
            s[4] += inter / len(L) if L else float("nan")
            s[5] += 2.0 * inter / (len(P) + len(L)) if (P or L) else float("nan")
            s[6] += inter
            s[7] += len(P - L)
            fn += len(L - P)
            labels |= L
            for x in P | L:
                t = by.setdefault(x, [0, 0, 0])
                t[0] += x in P and x in L
                t[1] += x in P and x not in L
                t[2] += x in L and x not in P
        parts = df._comm.allgather_object((s.tolist(), fn, by, sorted(labels, key=str)))
        S = np.sum([np.asarray(q[0]) for q in parts], 0)
        FN = sum(q[1] for q in parts)
        allby: dict = {}
        all_labels = set()
        for _, _, b, labs in parts:
            all_labels |= set(labs)
            for k, v in b.items():
                t = allby.setdefault(k, [0, 0, 0])
                for i in range(3):
                    t[i] += v[i]
        n = S[0]
        m = self.getMetricName()
        if m == "subsetAccuracy":
            return S[1] / n
        if m == "accuracy":
            return S[2] / n
        if m == "hammingLoss":
            return (S[7] + FN) / (n * max(len(all_labels), 1))
        if m == "precision":
            return S[3] / n
        if m == "recall":
            return S[4] / n
        if m == "f1Measure":
            return S[5] / n
        tp, fp = S[6], S[7]
        if m == "microPrecision":
            return tp / (tp + fp)
        if m == "microRecall":
            return tp / (tp + FN)
        if m == "microF1Measure":
            return 2 * tp / (2 * tp + fp + FN)
        t = allby.get(self.getMetricLabel(), [0, 0, 0])
        prec = t[0] / (t[0] + t[1]) if t[0] + t[1] else 0.0
        rec = t[0] / (t[0] + t[2]) if t[0] + t[2] else 0.0
        if m == "precisionByLabel":
            return prec
        if m == "recallByLabel":
            return rec
        if m == "f1MeasureByLabel":
            return 2 * prec * rec / (prec + rec) if prec + rec else 0.0
        raise ValueError(f"unknown multilabel metric {m!r}")

    def isLargerBetter(self) -> bool:
        return self.getMetricName() != "hammingLoss"


class RankingEvaluator(Evaluator):
    """Spark's RankingMetrics with binary relevance: meanAveragePrecision (default),
    meanAveragePrecisionAtK, precisionAtK, ndcgAtK, recallAtK over ranked prediction arrays and
    ground-truth label arrays."""
    _params = {
        "predictionCol": ("prediction", "prediction column name", str),
        "labelCol": ("label", "label column name", str),
        "metricName": ("meanAveragePrecision", "metric name in evaluation", str),
        "k": (10, "the ranking position value used in the *AtK metrics (> 0)", int),
    }

    def __init__(self, predictionCol=None, labelCol=None, metricName=None, k=None):
        super().__init__(predictionCol=predictionCol, labelCol=labelCol, metricName=metricName, k=k)

    def _evaluate(self, df) -> float:
        pairs = _array_pairs(df, self.getPredictionCol(), self.getLabelCol())
        m, k = self.getMetricName(), self.getK()
        tot = 0.0
        for pred, lab in pairs:
            L = set(lab)
            if m == "meanAveragePrecision":
                hits, acc = 0, 0.0
                for i, x in enumerate(pred):
                    if x in L:
                        hits += 1
                        acc += hits / (i + 1)
                tot += acc / len(L) if L else 0.0
            elif m == "meanAveragePrecisionAtK":
                hits, acc = 0, 0.0
                for i, x in enumerate(pred[:k]):
                    if x in L:
                        hits += 1
                        acc += hits / (i + 1)
                tot += acc / min(len(L), k) if L else 0.0
            elif m == "precisionAtK":
                tot += sum(1 for x in pred[:k] if x in L) / k if L else 0.0
            elif m == "recallAtK":
                tot += sum(1 for x in pred[:k] if x in L) / len(L) if L else 0.0
            elif m == "ndcgAtK":
                if not L:
                    continue
                dcg = sum(1.0 / math.log2(i + 2) for i, x in enumerate(pred[:k]) if x in L)
                idcg = sum(1.0 / math.log2(i + 2) for i in range(min(k, len(L))))
                tot += dcg / idcg
            else:
                raise ValueError(f"unknown ranking metric {m!r}")
        t = torch.tensor([tot, float(len(pairs))], dtype=torch.float64, device=df._device)
        df._comm.allreduce_(t)
        return float(t[0] / t[1]) if t[1] > 0 else float("nan")
