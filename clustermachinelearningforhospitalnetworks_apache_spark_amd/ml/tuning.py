"""Model selection (pyspark.ml.tuning-compatible): ParamGridBuilder, CrossValidator, TrainValidationSplit.

The reference fits each of its three regressors and two classifiers once with fixed hyper-parameters
(ref.py:145-158, ref.py:182-190) and compares them by RMSE / accuracy (ref.py:160-198). These
classes run that comparison over a parameter grid, the way a Spark user would.

MI355X-first notes:
  * folds come from ``DataFrame.randomSplit`` — a hash of (seed, global row id) — so fold membership,
    and with it every metric, is the same on 1..8 GPUs and on the CPU;
  * every fold stays HBM-resident: the training complement is a row-mask view (``union`` of the
    other folds' shards, no host round trip), and each candidate fit runs the normal distributed
    kernels (histograms / Gram / gradients all-reduced over RCCL);
  * ``parallelism`` is accepted for API parity; fits run one after another because each one already
    fills the GPU (and the collectives must be issued in the same order on every rank).
"""
from __future__ import annotations

import itertools
import os
from typing import Any, Dict, List, Optional

import numpy as np

from . import util as U
from .base import Estimator, Model
from .param import NO_DEFAULT, Param


class ParamGridBuilder:
    """Cartesian product of parameter values -> list of ``{Param: value}`` maps."""

    def __init__(self):
        self._grid: Dict[Param, List[Any]] = {}

    def addGrid(self, param: Param, values) -> "ParamGridBuilder":
        self._grid[param] = list(values)
        return self

    def baseOn(self, *args) -> "ParamGridBuilder":
        if len(args) == 1 and isinstance(args[0], dict):
            items = list(args[0].items())
        else:
            items = list(args)
        for p, v in items:
            self.addGrid(p, [v])
        return self

    def build(self) -> List[Dict[Param, Any]]:
        keys = list(self._grid)
        return [dict(zip(keys, combo)) for combo in itertools.product(*(self._grid[k] for k in keys))]


class _ValidatorParams:
    """estimator / estimatorParamMaps / evaluator (objects, not JSON-serialisable params)."""

    def _init_validator(self, estimator, estimatorParamMaps, evaluator):
        self._estimator = estimator
        self._epm = list(estimatorParamMaps) if estimatorParamMaps is not None else None
        self._evaluator = evaluator

    def setEstimator(self, value):
        self._estimator = value
        return self

    def getEstimator(self):
        return self._estimator

    def setEstimatorParamMaps(self, value):
        self._epm = list(value)
        return self

    def getEstimatorParamMaps(self):
        return self._epm

    def setEvaluator(self, value):
        self._evaluator = value
        return self

    def getEvaluator(self):
        return self._evaluator

    def _check(self):
        if self._estimator is None or self._evaluator is None:
            raise ValueError(f"{type(self).__name__}: estimator and evaluator must be set")
        return self._epm if self._epm else [{}]

    def _evaluate_maps(self, train, valid, maps, keep_models: bool):
        """Fit one model per param map on ``train`` and score it on ``valid``."""
        metrics, models = [], []
        for pm in maps:
            model = self._estimator.fit(train, pm)
            metrics.append(float(self._evaluator.evaluate(model.transform(valid))))
            if keep_models:
                models.append(model)
        return metrics, models

    def _best_index(self, metrics) -> int:
        m = np.asarray(metrics, dtype=np.float64)
        return int(np.argmax(m) if self._evaluator.isLargerBetter() else np.argmin(m))


def _param_map_json(pm: Dict) -> List[Dict[str, Any]]:
    return [{"parent": p.parent if isinstance(p, Param) else "", "name": p.name if isinstance(p, Param) else str(p),
             "value": U._json_value(v), "isJson": True} for p, v in pm.items()]


def _save_validator_model(inst, path: str, metrics_key: str, metrics: List[float], extra: Dict[str, Any]) -> None:
    U.write_metadata(inst, path, extra={metrics_key: metrics,
                                        "estimatorParamMaps": [_param_map_json(pm) for pm in (inst._epm or [])],
                                        **extra})
    d = os.path.join(path, "bestModel")
    os.makedirs(d, exist_ok=True)
    inst.bestModel._save_impl(d)


class CrossValidator(Estimator, _ValidatorParams):
    """k-fold cross validation: for each param map, the mean metric over ``numFolds`` (train on
    k-1 folds, evaluate on the held-out one); the best map is refit on the whole dataset."""
    _pause_gc = False  # meta-estimator: the collector runs between the inner fits (ml/base.py)

    _params = {
        "numFolds": (3, "number of folds for cross validation (>= 2)", int),
        "seed": (-1289195219, "random seed", int),
        "parallelism": (1, "number of threads to use when running parallel algorithms (>= 1)", int),
        "collectSubModels": (False, "whether to collect a list of sub-models trained during tuning", bool),
        "foldCol": ("", "integer column in [0, numFolds) naming each row's fold; empty = random folds", str),
    }

    def __init__(self, estimator=None, estimatorParamMaps=None, evaluator=None, numFolds=None, seed=None,
                 parallelism=None, collectSubModels=None, foldCol=None):
        super().__init__(numFolds=numFolds, seed=seed, parallelism=parallelism, collectSubModels=collectSubModels,
                         foldCol=foldCol)
        self._init_validator(estimator, estimatorParamMaps, evaluator)

    def _folds(self, df):
        k = self.getNumFolds()
        if k < 2:
            raise ValueError("numFolds must be >= 2")
        fc = self.getFoldCol()
        if fc:
            from ..sql import functions as F
            folds = [df.filter(F.col(fc) == i) for i in range(k)]
        else:
            folds = df.randomSplit([1.0] * k, seed=self.getSeed())
        out = []
        for i in range(k):
            train = None
            for j in range(k):
                if j != i:
                    train = folds[j] if train is None else train.union(folds[j])
            out.append((train, folds[i]))
        return out

    def _fit(self, df):
        maps = self._check()
        keep = bool(self.getCollectSubModels())
        per_fold, sub = [], []
        for train, valid in self._folds(df):
            m, models = self._evaluate_maps(train, valid, maps, keep)
            per_fold.append(m)
            sub.append(models)
        arr = np.asarray(per_fold, dtype=np.float64)  # [folds, maps]
        avg, std = arr.mean(axis=0), arr.std(axis=0)
        best = self._best_index(avg)
        best_model = self._estimator.fit(df, maps[best])
        m = CrossValidatorModel(best_model, avg.tolist(), sub if keep else None, std.tolist())
        self._copyValues(m)
        m._init_validator(self._estimator, self._epm, self._evaluator)
        return m


class CrossValidatorModel(Model, _ValidatorParams):
    _params = CrossValidator._params

    def __init__(self, bestModel=None, avgMetrics: Optional[List[float]] = None, subModels=None,
                 stdMetrics: Optional[List[float]] = None):
        super().__init__()
        self.bestModel = bestModel
        self.avgMetrics = list(avgMetrics or [])
        self.stdMetrics = list(stdMetrics or [])
        self.subModels = subModels
        self._init_validator(None, None, None)

    def _transform(self, df):
        return self.bestModel.transform(df)

    def _save_impl(self, path):
        _save_validator_model(self, path, "avgMetrics", self.avgMetrics, {"stdMetrics": self.stdMetrics})

    @classmethod
    def _load_impl(cls, path, md):
        m = cls(U.load(os.path.join(path, "bestModel")), md.get("avgMetrics"), None, md.get("stdMetrics"))
        U.apply_params(m, md)
        return m


class TrainValidationSplit(Estimator, _ValidatorParams):
    """One train/validation split (``trainRatio``) per param map; the best map is refit on all rows."""
    _pause_gc = False  # meta-estimator: the collector runs between the inner fits (ml/base.py)

    _params = {
        "trainRatio": (0.75, "ratio between training set and validation set (>= 0, <= 1)", float),
        "seed": (-1103429291, "random seed", int),
        "parallelism": (1, "number of threads to use when running parallel algorithms (>= 1)", int),
        "collectSubModels": (False, "whether to collect a list of sub-models trained during tuning", bool),
    }

    def __init__(self, estimator=None, estimatorParamMaps=None, evaluator=None, trainRatio=None, seed=None,
                 parallelism=None, collectSubModels=None):
        super().__init__(trainRatio=trainRatio, seed=seed, parallelism=parallelism,
                         collectSubModels=collectSubModels)
        self._init_validator(estimator, estimatorParamMaps, evaluator)

    def _fit(self, df):
        maps = self._check()
        r = float(self.getTrainRatio())
        if not 0.0 < r < 1.0:
            raise ValueError("trainRatio must be in (0, 1)")
        train, valid = df.randomSplit([r, 1.0 - r], seed=self.getSeed())
        keep = bool(self.getCollectSubModels())
        metrics, models = self._evaluate_maps(train, valid, maps, keep)
        best = self._best_index(metrics)
        best_model = self._estimator.fit(df, maps[best])
        m = TrainValidationSplitModel(best_model, metrics, models if keep else None)
        self._copyValues(m)
        m._init_validator(self._estimator, self._epm, self._evaluator)
        return m


class TrainValidationSplitModel(Model, _ValidatorParams):
    _params = TrainValidationSplit._params

    def __init__(self, bestModel=None, validationMetrics: Optional[List[float]] = None, subModels=None):
        super().__init__()
        self.bestModel = bestModel
        self.validationMetrics = list(validationMetrics or [])
        self.subModels = subModels
        self._init_validator(None, None, None)

    def _transform(self, df):
        return self.bestModel.transform(df)

    def _save_impl(self, path):
        _save_validator_model(self, path, "validationMetrics", self.validationMetrics, {})

    @classmethod
    def _load_impl(cls, path, md):
        m = cls(U.load(os.path.join(path, "bestModel")), md.get("validationMetrics"))
        U.apply_params(m, md)
        return m


__all__ = ["ParamGridBuilder", "CrossValidator", "CrossValidatorModel", "TrainValidationSplit",
           "TrainValidationSplitModel"]
