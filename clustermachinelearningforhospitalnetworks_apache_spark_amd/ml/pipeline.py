"""Pipeline / PipelineModel ([NS]: VectorAssembler -> StandardScaler -> KMeans -> LogReg).

Persistence follows Spark: ``metadata`` with ``paramMap.stageUids`` and one
sub-directory ``stages/<idx>_<uid>`` per stage.
"""
from __future__ import annotations

import os
from typing import List, Optional

from . import util as U
from .base import Estimator, Model, Transformer


class Pipeline(Estimator):
    _pause_gc = False  # meta-estimator: the collector runs between the inner fits (ml/base.py)
    _params = {"stages": ([], "a list of pipeline stages", None)}

    def __init__(self, stages: Optional[List] = None):
        super().__init__(stages=stages)

    def getStages(self) -> List:
        return list(self.getOrDefault("stages"))

    def _fit(self, df):
        stages = self.getStages()
        last_est = max([i for i, s in enumerate(stages) if isinstance(s, Estimator)], default=-1)
        fitted = []
        cur = df
        for i, st in enumerate(stages):
            if isinstance(st, Estimator):
                m = st.fit(cur)
                fitted.append(m)
                if i < last_est:
                    cur = m.transform(cur)
            elif isinstance(st, Transformer):
                fitted.append(st)
                if i < last_est:
                    cur = st.transform(cur)
            else:
                raise TypeError(f"pipeline stage {st!r} is neither an Estimator nor a Transformer")
        return PipelineModel(fitted)

    def _save_impl(self, path):
        _save_stages(self, self.getStages(), path)

    @classmethod
    def _load_impl(cls, path, md):
        p = cls(_load_stages(path, md))
        p.uid = md["uid"]
        return p


class PipelineModel(Model):
    _params = {}

    def __init__(self, stages: Optional[List] = None):
        super().__init__()
        self.stages = list(stages or [])

    def _transform(self, df):
        for st in self.stages:
            df = st.transform(df)
        return df

    def _save_impl(self, path):
        _save_stages(self, self.stages, path)

    @classmethod
    def _load_impl(cls, path, md):
        m = cls(_load_stages(path, md))
        m.uid = md["uid"]
        return m


def _stage_dir(path: str, i: int, n: int, uid: str) -> str:
    width = len(str(max(n - 1, 0)))
    return os.path.join(path, "stages", f"{str(i).zfill(width)}_{uid}")


def _save_stages(inst, stages, path):
    U.write_metadata(inst, path, param_map={"stageUids": [s.uid for s in stages]})
    for i, s in enumerate(stages):
        d = _stage_dir(path, i, len(stages), s.uid)
        os.makedirs(d, exist_ok=True)
        s._save_impl(d)


def _load_stages(path, md) -> List:
    uids = md["paramMap"]["stageUids"]
    out = []
    for i, uid in enumerate(uids):
        d = _stage_dir(path, i, len(uids), uid)
        out.append(U.load(d))
    return out
