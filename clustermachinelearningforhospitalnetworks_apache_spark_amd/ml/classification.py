"""Classifiers: DecisionTreeClassifier / RandomForestClassifier (ref.py:32,
ref.py:182-190) and LogisticRegression ([NS]; the reference's dead per-batch hook
names it, ref.py:95).

LogisticRegression follows Spark's defaults (maxIter=100, regParam=0,
elasticNetParam=0, tol=1e-6, fitIntercept=True, standardization=True,
threshold=0.5, family="auto").  Binomial fits run L-BFGS (OWL-QN with L1) whose
every function evaluation is ONE fused device pass over the shard (K13: margin,
sigmoid, gradient and loss, X read once) + one all-reduce of the (d+3)-vector.
``solver="sgd"`` (cml extension for the [NS] mini-batch SGD config) keeps the
coefficients on the device and runs K13 on mini-batch slices + RCCL all-reduce +
an on-device update per step, with no host synchronisation inside an epoch.
Multinomial fits run K13m (glm.hip multinomial_grad_kernel): the C margins, the softmax and the
C×d gradient in one pass over X, f64 partials; L1 through OWL-QN.
"""
from __future__ import annotations

import math
from typing import List, Optional

import numpy as np
import torch

from ..models.optim import lbfgs
from ..ops import glm_ops
from ..sql import types as T
from ..sql.column import ColumnData
from . import util as U
from .base import Estimator, Model
from .evaluation import BinaryClassificationEvaluator, MulticlassClassificationEvaluator
from .feature import _replace_col
from .linalg import DenseMatrix, DenseVector, as_array
from .tree_models import (CLASSIF_PARAMS, FOREST_PARAMS, GBT_PARAMS, TREE_PARAMS, GBTEstimatorMixin, GBTModelMixin,
                          TreeEstimatorMixin, TreeModelMixin, _default_seed)

_LOGREG_PARAMS = {
    "featuresCol": ("features", "features column name", str),
    "labelCol": ("label", "label column name", str),
    "predictionCol": ("prediction", "prediction column name", str),
    "probabilityCol": ("probability", "column name for predicted class conditional probabilities", str),
    "rawPredictionCol": ("rawPrediction", "raw prediction (a.k.a. confidence) column name", str),
    "maxIter": (100, "max number of iterations (>= 0)", int),
    "regParam": (0.0, "regularization parameter (>= 0)", float),
    "elasticNetParam": (0.0, "ElasticNet mixing parameter in [0, 1]", float),
    "tol": (1e-6, "convergence tolerance for iterative algorithms (>= 0)", float),
    "fitIntercept": (True, "whether to fit an intercept term", bool),
    "threshold": (0.5, "threshold in binary classification prediction, in range [0, 1]", float),
    "thresholds": (None, "thresholds in multi-class classification", None),
    "standardization": (True, "whether to standardize the training features before fitting", bool),
    "weightCol": (None, "weight column name", None),
    "aggregationDepth": (2, "suggested depth for treeAggregate (>= 2)", int),
    "family": ("auto", "auto | binomial | multinomial", str),
    "maxBlockSizeInMB": (0.0, "maximum memory in MB for stacking input data into blocks", float),
    # cml extensions for the [NS] data-parallel mini-batch SGD configuration
    "solver": ("lbfgs", "cml: 'lbfgs' (Spark's optimizer) or 'sgd' (mini-batch, device-resident)", str),
    "stepSize": (1.0, "cml: SGD step size", float),
    "batchSize": (65536, "cml: SGD rows per rank per step", int),
    "momentum": (0.9, "cml: SGD momentum", float),
}


class LogisticRegression(Estimator):
    _params = _LOGREG_PARAMS

    def __init__(self, **kwargs):
        super().__init__(**kwargs)
        for k in ("thresholds", "weightCol"):
            self._defaultParamMap.pop(k, None)

    # ------------------------------------------------------------------ fit
    def _fit(self, df):
        x = df._feature_matrix(self.getFeaturesCol())
        d = x.shape[1]
        y = df._column_data(self.getLabelCol()).values.to(torch.float64)
        w = df._column_data(self.getOrDefault("weightCol")).values.to(torch.float64) \
            if self.isSet("weightCol") else None
        comm = df._comm
        ymax = comm.max_scalar(float(y.max().item()) if y.numel() else 0.0)
        num_classes = max(2, int(ymax) + 1)
        family = self.getFamily()
        multinomial = family == "multinomial" or (family == "auto" and num_classes > 2)
        if family == "binomial" and num_classes > 2:
            raise ValueError("binomial family only supports 1 or 2 outcome classes")
        # feature standard deviations (K7 + all-reduce)
        n, s1, s2, shift = glm_ops.moments(x, d)
        msg = torch.cat([torch.tensor([float(n)], dtype=torch.float64, device=x.device), s1 + n * shift,
                         s2 + 2 * shift * s1 + n * shift * shift])
        comm.allreduce_(msg)
        N = msg[0].item()
        mean = msg[1:1 + d] / max(N, 1)
        var = torch.clamp((msg[1 + d:] - N * mean * mean) / max(N - 1, 1), min=0.0)
        std = torch.sqrt(var).cpu().numpy()
        # L-BFGS state checkpoints (cml.ml.checkpointDir): x, f, g and the s/y history every
        # cml.ml.checkpointInterval iterations; a restarted fit resumes and ends bit for bit where the
        # uninterrupted one does
        from ..utils.checkpoint import FitCheckpoint
        sgd = self.getSolver() == "sgd" and not multinomial
        ck = None
        if not sgd:
            key = (f"{'multinomial' if multinomial else 'binomial'}|d={d}|C={num_classes}|reg={self.getRegParam()}|"
                   f"en={self.getElasticNetParam()}|fi={self.getFitIntercept()}|std={self.getStandardization()}|"
                   f"tol={self.getTol()}")
            ck = FitCheckpoint(df, "logreg", key, (x, y, w))
        if multinomial:
            coef, icpt, hist, iters = self._fit_multinomial(x, y, w, d, num_classes, std, comm, ck)
        elif sgd:
            coef, icpt, hist, iters = self._fit_sgd(x, y, w, d, std, comm)
            coef, icpt = coef[None, :], np.array([icpt])
        else:
            coef, icpt, hist, iters = self._fit_binomial(x, y, w, d, std, comm, ck)
            coef, icpt = coef[None, :], np.array([icpt])
        if ck is not None:
            ck.clear()
        model = LogisticRegressionModel(coef, icpt, num_classes, multinomial)
        self._copyValues(model)
        model._attach_summary(LogisticRegressionTrainingSummary(model, df, hist, iters))
        return model

    def _reg(self):
        lam, a = self.getRegParam(), self.getElasticNetParam()
        return lam * (1.0 - a), lam * a

    def _lbfgs(self, fg, p0, l1v, ck):
        """models/optim.lbfgs with the fit's checkpoint (resume + periodic saves) and crash point."""
        from ..models.optim import lbfgs_state_arrays, lbfgs_state_from_arrays
        state = None
        if ck is not None:
            got = ck.load()
            if got is not None:
                state = lbfgs_state_from_arrays(got[1])

        def on_iter(it, st):
            if ck is not None and ck.due(it):
                ck.save(it, lbfgs_state_arrays(st))
        return lbfgs(fg, p0, self.getMaxIter(), self.getTol(), l1=l1v, state=state, on_iter=on_iter,
                     fault="logreg.iteration")

    def _fit_binomial(self, x, y, w, d, std, comm, ck=None):
        l2, l1 = self._reg()
        sd = np.where(std > 0, std, 1.0)
        active = std > 0
        fi = self.getFitIntercept()
        standardize = self.getStandardization()
        dev = x.device

        def fg(p):
            wp, b = p[:d], (p[d] if fi else 0.0)
            coef = np.where(active, wp / sd, 0.0)
            out = glm_ops.logreg_grad(x, d, y, torch.as_tensor(np.r_[coef, b], device=dev), w)
            comm.allreduce_(out)
            o = out.cpu().numpy()
            wsum = max(o[d + 2], 1e-300)
            g = np.zeros(d + 1)
            g[:d] = np.where(active, o[:d] / sd, 0.0) / wsum
            g[d] = o[d] / wsum if fi else 0.0
            f = o[d + 1] / wsum
            if l2 > 0:
                pen = wp if standardize else wp / sd
                f += 0.5 * l2 * float(np.sum(np.where(active, pen * pen, 0.0)))
                g[:d] += l2 * np.where(active, pen if standardize else pen / sd, 0.0)
            return f, g

        p0 = np.zeros(d + 1)
        if fi:
            # Spark's warm start: intercept = log(p / (1 - p)) of the (weighted) positive rate
            pos = (y * (w if w is not None else 1.0)).sum()
            tot = (w.sum() if w is not None else torch.tensor(float(y.numel()), dtype=torch.float64))
            pt = torch.stack([pos.to(torch.float64).to(dev), tot.to(torch.float64).to(dev)])
            comm.allreduce_(pt)
            pr = float(pt[0] / max(float(pt[1]), 1e-300))
            if 0.0 < pr < 1.0:
                p0[d] = math.log(pr / (1.0 - pr))
        l1v = None
        if l1 > 0:
            l1v = np.r_[np.full(d, l1) if standardize else l1 / sd, 0.0]
        p, hist, iters = self._lbfgs(fg, p0, l1v, ck)
        coef = np.where(active, p[:d] / sd, 0.0)
        return coef, float(p[d]) if fi else 0.0, hist, iters

    def _fit_sgd(self, x, y, w, d, std, comm):
        """Data-parallel mini-batch SGD with momentum (models/sgd.py): coefficients and velocity stay
        on the device; on one GPU each step is a replayed HIP graph."""
        from ..models.sgd import LogisticSGD
        l2, _ = self._reg()
        n = x.shape[0]
        bs = max(1, min(self.getBatchSize(), max(n, 1)))
        steps_per_epoch = max(1, max(c // max(1, min(bs, c)) if c else 0 for c in comm.allgather_object(n)))
        opt = LogisticSGD(x, d, y, w, comm, bs, self.getStepSize(), self.getMomentum(), l2, self.getFitIntercept())
        hist = []
        for epoch in range(self.getMaxIter()):
            hist.append(opt.epoch(epoch, self.getStepSize(), steps_per_epoch))
            if len(hist) > 1 and abs(hist[-2] - hist[-1]) < self.getTol() * max(abs(hist[-1]), 1.0):
                break
        c = opt.coef.cpu().numpy()
        return c[:d], float(c[d]), hist, opt.steps

    def _fit_multinomial(self, x, y, w, d, C, std, comm, ck=None):
        """Softmax regression (Spark's multinomial family): L-BFGS / OWL-QN over the standardized
        coefficients; every evaluation is one K13m pass over the local rows (glm_ops.multinomial_grad: X
        read once, no f64 copy) and one all-reduce of the [C·d | C | loss | weight] message."""
        l2, l1 = self._reg()
        sd = np.where(std > 0, std, 1.0)
        active = std > 0
        fi = self.getFitIntercept()
        standardize = self.getStandardization()
        dev = x.device

        def fg(p):
            P = p.reshape(C, d + 1)
            coef = np.zeros((C, d + 1))
            coef[:, :d] = np.where(active[None, :], P[:, :d] / sd[None, :], 0.0)
            if fi:
                coef[:, d] = P[:, d]
            msg = glm_ops.multinomial_grad(x, d, y, torch.as_tensor(coef, device=dev), w)
            comm.allreduce_(msg)
            o = msg.cpu().numpy()
            wsum = max(o[-1], 1e-300)
            G = np.zeros((C, d + 1))
            G[:, :d] = np.where(active[None, :], o[: C * d].reshape(C, d) / sd[None, :], 0.0) / wsum
            if fi:
                G[:, d] = o[C * d: C * d + C] / wsum
            f = o[-2] / wsum
            if l2 > 0:
                Wn = P[:, :d]
                pen = Wn if standardize else Wn / sd[None, :]
                f += 0.5 * l2 * float(np.sum(np.where(active[None, :], pen * pen, 0.0)))
                G[:, :d] += l2 * np.where(active[None, :], pen if standardize else pen / sd[None, :], 0.0)
            return f, G.reshape(-1)

        p0 = np.zeros(C * (d + 1))
        l1v = None
        if l1 > 0:  # OWL-QN on the coefficients (intercepts unpenalised), as Spark's multinomial elastic net
            l1v = np.zeros((C, d + 1))
            l1v[:, :d] = np.full(d, l1)[None, :] if standardize else (l1 / sd)[None, :]
            l1v = l1v.reshape(-1)
        p, hist, iters = self._lbfgs(fg, p0, l1v, ck)
        P = p.reshape(C, d + 1)
        coef = np.where(active[None, :], P[:, :d] / sd[None, :], 0.0)
        icpt = P[:, d].copy() if fi else np.zeros(C)
        if self.getRegParam() == 0.0:
            coef -= coef.mean(0, keepdims=True)
        if fi:
            icpt -= icpt.mean()
        return coef, icpt, hist, iters


class LogisticRegressionModel(Model):
    _params = _LOGREG_PARAMS

    def __init__(self, coefficientMatrix=None, interceptVector=None, numClasses: int = 2,
                 isMultinomial: bool = False):
        super().__init__()
        self._W = np.atleast_2d(np.asarray(coefficientMatrix if coefficientMatrix is not None else np.zeros((1, 0)),
                                           dtype=np.float64))
        self._b = np.asarray(interceptVector if interceptVector is not None else np.zeros(1), dtype=np.float64)
        self._num_classes = int(numClasses)
        self._multinomial = bool(isMultinomial)
        self._summary = None

    @property
    def coefficients(self) -> DenseVector:
        if self._multinomial:
            raise RuntimeError("Multinomial models contain a matrix of coefficients, use coefficientMatrix instead")
        return DenseVector(self._W[0])

    @property
    def intercept(self) -> float:
        if self._multinomial:
            raise RuntimeError("Multinomial models contain a vector of intercepts, use interceptVector instead")
        return float(self._b[0])

    @property
    def coefficientMatrix(self) -> DenseMatrix:
        return DenseMatrix(self._W.shape[0], self._W.shape[1], self._W.T.reshape(-1), False)

    @property
    def interceptVector(self) -> DenseVector:
        return DenseVector(self._b)

    @property
    def numClasses(self) -> int:
        return self._num_classes

    @property
    def numFeatures(self) -> int:
        return int(self._W.shape[1])

    def _scores(self, x: torch.Tensor):
        dev = x.device
        d = x.shape[1]
        if not self._multinomial:
            coef = torch.as_tensor(np.r_[self._W[0], self._b[0]], device=dev)
            m = glm_ops.linear_predict(x, d, coef, "identity")
            raw = torch.stack([-m, m], 1)
            p1 = torch.sigmoid(m)
            prob = torch.stack([1 - p1, p1], 1)
            return raw, prob
        W = torch.as_tensor(self._W, device=dev)
        b = torch.as_tensor(self._b, device=dev)
        if x.is_cuda:  # K13t: one pass, f64 MFMAs (bf16 / f32 rows, d <= 256, C <= 64)
            out = glm_ops.multinomial_predict(x, d, torch.cat([W, b[:, None]], 1))
            if out is not None:
                return out
        # row chunks: the C-class margins without an f64 copy of the whole feature matrix
        raw = torch.empty((x.shape[0], W.shape[0]), dtype=torch.float64, device=dev)
        for r0 in range(0, int(x.shape[0]), 1 << 20):
            raw[r0:r0 + (1 << 20)] = x[r0:r0 + (1 << 20), :d].to(torch.float64) @ W.T + b[None, :]
        return raw, torch.softmax(raw, 1)

    def _predict_from_prob(self, prob: torch.Tensor) -> torch.Tensor:
        thr = self.getOrDefault("thresholds") if self.isSet("thresholds") else None
        if thr:
            t = torch.as_tensor(np.asarray(thr, dtype=np.float64), device=prob.device)
            return torch.argmax(prob / t.clamp(min=1e-300), 1).to(torch.float64)
        if not self._multinomial:
            return (prob[:, 1] > self.getThreshold()).to(torch.float64)
        return torch.argmax(prob, 1).to(torch.float64)

    def _transform(self, df):
        x = df._feature_matrix(self.getFeaturesCol())
        raw, prob = self._scores(x)
        out = df
        if self.getRawPredictionCol():
            out = _replace_col(out, self.getRawPredictionCol(), ColumnData(raw, None, T.VectorUDT()))
        if self.getProbabilityCol():
            out = _replace_col(out, self.getProbabilityCol(), ColumnData(prob, None, T.VectorUDT()))
        return _replace_col(out, self.getPredictionCol(),
                            ColumnData(self._predict_from_prob(prob), None, T.DoubleType()))

    def predict(self, value) -> float:
        v = torch.as_tensor(as_array(value), dtype=torch.float64).reshape(1, -1)
        _, prob = self._scores(v)
        return float(self._predict_from_prob(prob)[0])

    def predictProbability(self, value) -> DenseVector:
        v = torch.as_tensor(as_array(value), dtype=torch.float64).reshape(1, -1)
        return DenseVector(self._scores(v)[1][0].cpu().numpy())

    def predictRaw(self, value) -> DenseVector:
        v = torch.as_tensor(as_array(value), dtype=torch.float64).reshape(1, -1)
        return DenseVector(self._scores(v)[0][0].cpu().numpy())

    def evaluate(self, df):
        return LogisticRegressionSummary(self, df)

    def _save_impl(self, path):
        import pyarrow as pa
        U.write_metadata(self, path)
        row = {"numClasses": self._num_classes, "numFeatures": self.numFeatures,
               "interceptVector": U.vector_struct(self._b), "coefficientMatrix": U.matrix_struct(self._W),
               "isMultinomial": self._multinomial}
        U.write_parquet(path, "data", pa.Table.from_pylist([row], schema=pa.schema([
            pa.field("numClasses", pa.int32(), nullable=False), pa.field("numFeatures", pa.int32(), nullable=False),
            ("interceptVector", U.vector_arrow_type()), ("coefficientMatrix", U.matrix_arrow_type()),
            pa.field("isMultinomial", pa.bool_(), nullable=False)])))

    @classmethod
    def _load_impl(cls, path, md):
        r = U.read_parquet(path, "data").to_pylist()[0]
        m = cls(U.matrix_from_struct(r["coefficientMatrix"]), U.vector_from_struct(r["interceptVector"]),
                r["numClasses"], r["isMultinomial"])
        U.apply_params(m, md)
        return m


class LogisticRegressionSummary:
    def __init__(self, model, df):
        self._model = model
        self._df = df
        self.labelCol = model.getLabelCol()
        self.predictionCol = model.getPredictionCol()
        self.probabilityCol = model.getProbabilityCol()
        self.featuresCol = model.getFeaturesCol()
        self._pred = None

    @property
    def predictions(self):
        if self._pred is None:
            self._pred = self._model.transform(self._df)
        return self._pred

    def _mc(self, metric, label=0.0):
        return MulticlassClassificationEvaluator(labelCol=self.labelCol, predictionCol=self.predictionCol,
                                                 metricName=metric, metricLabel=label).evaluate(self.predictions)

    @property
    def accuracy(self):
        return self._mc("accuracy")

    @property
    def weightedPrecision(self):
        return self._mc("weightedPrecision")

    @property
    def weightedRecall(self):
        return self._mc("weightedRecall")

    @property
    def weightedFMeasure(self):
        return self._mc("weightedFMeasure")

    @property
    def areaUnderROC(self):
        return BinaryClassificationEvaluator(rawPredictionCol=self._model.getRawPredictionCol(),
                                             labelCol=self.labelCol).evaluate(self.predictions)


class LogisticRegressionTrainingSummary(LogisticRegressionSummary):
    def __init__(self, model, df, hist, iters):
        super().__init__(model, df)
        self.objectiveHistory = list(hist)
        self.totalIterations = int(iters)


BinaryLogisticRegressionTrainingSummary = LogisticRegressionTrainingSummary


# ------------------------------------------------------------------------------------------------ trees

class DecisionTreeClassifier(TreeEstimatorMixin, Estimator):
    _task = "classification"
    _params = dict(TREE_PARAMS, **CLASSIF_PARAMS,
                   impurity=("gini", "criterion used for information gain (gini, entropy)", str),
                   seed=(_default_seed("org.apache.spark.ml.classification.DecisionTreeClassifier"), "random seed",
                         int))

    def __init__(self, **kwargs):
        super().__init__(**kwargs)
        for k in ("weightCol", "thresholds"):
            self._defaultParamMap.pop(k, None)

    def _fit(self, df):
        trees, d, nc = self._tree_fit(df)
        m = DecisionTreeClassificationModel()
        self._copyValues(m)
        m._init_trees(trees, d, nc)
        return m


class DecisionTreeClassificationModel(TreeModelMixin, Model):
    _task = "classification"
    _params = DecisionTreeClassifier._params

    def __init__(self):
        super().__init__()
        self._init_trees([], 0)

    @property
    def numClasses(self) -> int:
        return self._num_classes

    @staticmethod
    def _single_tree_class():
        return DecisionTreeClassificationModel


class RandomForestClassifier(TreeEstimatorMixin, Estimator):
    _task = "classification"
    _forest = True
    _params = dict(TREE_PARAMS, **CLASSIF_PARAMS, **FOREST_PARAMS,
                   impurity=("gini", "criterion used for information gain (gini, entropy)", str),
                   seed=(_default_seed("org.apache.spark.ml.classification.RandomForestClassifier"), "random seed",
                         int))

    def __init__(self, **kwargs):
        super().__init__(**kwargs)
        for k in ("weightCol", "thresholds"):
            self._defaultParamMap.pop(k, None)

    def _fit(self, df):
        trees, d, nc = self._tree_fit(df)
        m = RandomForestClassificationModel()
        self._copyValues(m)
        m._init_trees(trees, d, nc)
        return m


class RandomForestClassificationModel(TreeModelMixin, Model):
    _task = "classification"
    _forest = True
    _params = RandomForestClassifier._params

    def __init__(self):
        super().__init__()
        self._init_trees([], 0)

    @property
    def numClasses(self) -> int:
        return self._num_classes

    @staticmethod
    def _single_tree_class():
        return DecisionTreeClassificationModel


class GBTClassifier(GBTEstimatorMixin, Estimator):
    """Gradient-boosted trees for binary labels (Spark ``GBTClassifier``, LogLoss on labels mapped
    to {-1,+1}; rawPrediction [-F, F], probability 1/(1+exp(-2F)))."""
    _classification = True
    _params = dict(TREE_PARAMS, **CLASSIF_PARAMS, **GBT_PARAMS,
                   lossType=("logistic", "loss function which GBT tries to minimize (logistic)", str),
                   seed=(_default_seed("org.apache.spark.ml.classification.GBTClassifier"), "random seed", int))

    def __init__(self, **kwargs):
        super().__init__(**kwargs)
        self._defaultParamMap.pop("thresholds", None)

    def _fit(self, df):
        trees, tw, d = self._gbt_fit(df)
        m = GBTClassificationModel()
        self._copyValues(m)
        m._init_trees(trees, d, 2, tw)
        return m


class GBTClassificationModel(GBTModelMixin, Model):
    _classification = True
    _params = GBTClassifier._params

    def __init__(self):
        super().__init__()
        self._init_trees([], 0)

    @property
    def numClasses(self) -> int:
        return 2

    @staticmethod
    def _single_tree_class():
        from .regression import DecisionTreeRegressionModel
        return DecisionTreeRegressionModel


from .naive_bayes import NaiveBayes, NaiveBayesModel  # noqa: E402,F401
from .classification_more import (LinearSVC, LinearSVCModel, LinearSVCSummary,  # noqa: E402,F401
                                  LinearSVCTrainingSummary, MultilayerPerceptronClassificationModel,
                                  MultilayerPerceptronClassifier, OneVsRest, OneVsRestModel)
from .fm import FMClassificationModel, FMClassifier  # noqa: E402,F401
