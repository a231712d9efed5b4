"""Estimator / Transformer / Model / Evaluator (pyspark.ml-compatible).

``Estimator.fit(df) -> Model`` and ``Model.transform(df) -> df`` are the only
contracts the reference relies on (ref.py:147-190).  Streaming DataFrames are
accepted by ``transform`` too: the transformation is recorded and replayed on
every micro-batch.
"""
from __future__ import annotations

import contextlib
import copy
from typing import Any, Dict, List, Optional, Union

import torch

from .param import Params
from ..utils.device import gc_paused
from ..utils.trace import trace
from .util import MLReadable, MLWritable


class Transformer(Params, MLWritable, MLReadable):
    def transform(self, dataset, params: Optional[Dict] = None):
        inst = self.copy(params) if params else self
        if dataset.isStreaming:
            return dataset._lazy("_apply_transformer", inst)
        with trace(f"{type(self).__name__}.transform"):
            return inst._transform(dataset)

    def _transform(self, dataset):
        raise NotImplementedError


class Estimator(Params, MLWritable, MLReadable):
    # leaf estimators pause the cycle collector over their hot loops; meta-estimators (Pipeline, CrossValidator,
    # TrainValidationSplit, OneVsRest) do not, so it runs between their inner fits and reclaims an inner fit's
    # engine buffers held in reference cycles before the next fold allocates its own
    _pause_gc = True

    def fit(self, dataset, params: Optional[Union[Dict, List[Dict]]] = None):
        if isinstance(params, (list, tuple)):
            return [self.fit(dataset, p) for p in params]
        if dataset.isStreaming:
            raise RuntimeError("fit() on a streaming DataFrame: use writeStream.foreachBatch to train per batch")
        inst = self.copy(params) if params else self
        with trace(f"{type(self).__name__}.fit"), (gc_paused() if inst._pause_gc else contextlib.nullcontext()):
            model = inst._fit(dataset)
        if model is not None and getattr(model, "parent", None) is None:
            model.parent = inst
            model.uid = inst.uid  # Spark models carry their estimator's uid
        return model

    def fitMultiple(self, dataset, paramMaps):
        for i, pm in enumerate(paramMaps):
            yield i, self.fit(dataset, pm)

    def _fit(self, dataset):
        raise NotImplementedError


class Model(Transformer):
    parent = None

    def hasSummary(self) -> bool:
        return getattr(self, "_summary", None) is not None

    @property
    def summary(self):
        s = getattr(self, "_summary", None)
        if s is None:
            raise RuntimeError("No training summary available for this model")
        if hasattr(s, "_model") and s._model is None:
            # stored detached (no model <-> summary reference cycle, which would keep the training
            # DataFrame's HBM alive until Python's cycle collector happened to run); hand out a
            # shallow copy bound to this model
            b = copy.copy(s)
            b._model = self
            return b
        return s

    def _attach_summary(self, s) -> None:
        if hasattr(s, "_model"):
            s._model = None
        self._summary = s


class Evaluator(Params, MLWritable, MLReadable):
    def evaluate(self, dataset, params: Optional[Dict] = None) -> float:
        inst = self.copy(params) if params else self
        with trace(f"{type(self).__name__}.evaluate"):
            return inst._evaluate(dataset)

    def _evaluate(self, dataset) -> float:
        raise NotImplementedError

    def isLargerBetter(self) -> bool:
        return True


def session_of(df):
    return df._session


def feature_matrix(df, col: str) -> torch.Tensor:
    return df._feature_matrix(col)
