"""Model persistence in Spark's on-disk ML format (ref.py:241-243).

``path/metadata/part-00000``: one JSON line ``{"class", "timestamp", "sparkVersion",
"uid", "paramMap", "defaultParamMap"}`` (+ ``_SUCCESS``); ``path/data/part-*.parquet``
holds the model data with Spark's schemas (VectorUDT / MatrixUDT structs).  The
layouts come from Spark 3.x knowledge and could not be verified offline (no JVM
here) — they are kept in this one module.

``model.save(p)`` refuses an existing path (Spark semantics, the reference's dead
per-batch save ref.py:103); ``model.write().overwrite().save(p)`` replaces it
(ref.py:241-243).  Only rank 0 writes; all ranks meet at a barrier.
"""
from __future__ import annotations

import importlib
import json
import math
import os
import re
import shutil
import time
import uuid
from typing import Any, Dict, List, Optional

import numpy as np

SPARK_VERSION = "3.5.1"

# python class  <->  Spark JVM class names
_JVM = {
    "LinearRegression": "org.apache.spark.ml.regression.LinearRegression",
    "LinearRegressionModel": "org.apache.spark.ml.regression.LinearRegressionModel",
    "DecisionTreeRegressor": "org.apache.spark.ml.regression.DecisionTreeRegressor",
    "DecisionTreeRegressionModel": "org.apache.spark.ml.regression.DecisionTreeRegressionModel",
    "RandomForestRegressor": "org.apache.spark.ml.regression.RandomForestRegressor",
    "RandomForestRegressionModel": "org.apache.spark.ml.regression.RandomForestRegressionModel",
    "DecisionTreeClassifier": "org.apache.spark.ml.classification.DecisionTreeClassifier",
    "DecisionTreeClassificationModel": "org.apache.spark.ml.classification.DecisionTreeClassificationModel",
    "RandomForestClassifier": "org.apache.spark.ml.classification.RandomForestClassifier",
    "RandomForestClassificationModel": "org.apache.spark.ml.classification.RandomForestClassificationModel",
    "LogisticRegression": "org.apache.spark.ml.classification.LogisticRegression",
    "LogisticRegressionModel": "org.apache.spark.ml.classification.LogisticRegressionModel",
    "KMeans": "org.apache.spark.ml.clustering.KMeans",
    "KMeansModel": "org.apache.spark.ml.clustering.KMeansModel",
    "StandardScaler": "org.apache.spark.ml.feature.StandardScaler",
    "StandardScalerModel": "org.apache.spark.ml.feature.StandardScalerModel",
    "VectorAssembler": "org.apache.spark.ml.feature.VectorAssembler",
    "StringIndexer": "org.apache.spark.ml.feature.StringIndexer",
    "StringIndexerModel": "org.apache.spark.ml.feature.StringIndexerModel",
    "Binarizer": "org.apache.spark.ml.feature.Binarizer",
    "MinMaxScaler": "org.apache.spark.ml.feature.MinMaxScaler",
    "MinMaxScalerModel": "org.apache.spark.ml.feature.MinMaxScalerModel",
    "Pipeline": "org.apache.spark.ml.Pipeline",
    "PipelineModel": "org.apache.spark.ml.PipelineModel",
    "RegressionEvaluator": "org.apache.spark.ml.evaluation.RegressionEvaluator",
    "MulticlassClassificationEvaluator": "org.apache.spark.ml.evaluation.MulticlassClassificationEvaluator",
    "BinaryClassificationEvaluator": "org.apache.spark.ml.evaluation.BinaryClassificationEvaluator",
    "ClusteringEvaluator": "org.apache.spark.ml.evaluation.ClusteringEvaluator",
    "CrossValidator": "org.apache.spark.ml.tuning.CrossValidator",
    "CrossValidatorModel": "org.apache.spark.ml.tuning.CrossValidatorModel",
    "TrainValidationSplit": "org.apache.spark.ml.tuning.TrainValidationSplit",
    "TrainValidationSplitModel": "org.apache.spark.ml.tuning.TrainValidationSplitModel",
    "OneHotEncoder": "org.apache.spark.ml.feature.OneHotEncoder",
    "OneHotEncoderModel": "org.apache.spark.ml.feature.OneHotEncoderModel",
    "Imputer": "org.apache.spark.ml.feature.Imputer",
    "ImputerModel": "org.apache.spark.ml.feature.ImputerModel",
    "Bucketizer": "org.apache.spark.ml.feature.Bucketizer",
    "QuantileDiscretizer": "org.apache.spark.ml.feature.QuantileDiscretizer",
    "Normalizer": "org.apache.spark.ml.feature.Normalizer",
    "PCA": "org.apache.spark.ml.feature.PCA",
    "PCAModel": "org.apache.spark.ml.feature.PCAModel",
    "GeneralizedLinearRegression": "org.apache.spark.ml.regression.GeneralizedLinearRegression",
    "GeneralizedLinearRegressionModel": "org.apache.spark.ml.regression.GeneralizedLinearRegressionModel",
    "NaiveBayes": "org.apache.spark.ml.classification.NaiveBayes",
    "NaiveBayesModel": "org.apache.spark.ml.classification.NaiveBayesModel",
    "BisectingKMeans": "org.apache.spark.ml.clustering.BisectingKMeans",
    "BisectingKMeansModel": "org.apache.spark.ml.clustering.BisectingKMeansModel",
    "GBTRegressor": "org.apache.spark.ml.regression.GBTRegressor",
    "GBTRegressionModel": "org.apache.spark.ml.regression.GBTRegressionModel",
    "GBTClassifier": "org.apache.spark.ml.classification.GBTClassifier",
    "GBTClassificationModel": "org.apache.spark.ml.classification.GBTClassificationModel",
    "MaxAbsScaler": "org.apache.spark.ml.feature.MaxAbsScaler",
    "MaxAbsScalerModel": "org.apache.spark.ml.feature.MaxAbsScalerModel",
    "RobustScaler": "org.apache.spark.ml.feature.RobustScaler",
    "RobustScalerModel": "org.apache.spark.ml.feature.RobustScalerModel",
    "ElementwiseProduct": "org.apache.spark.ml.feature.ElementwiseProduct",
    "PolynomialExpansion": "org.apache.spark.ml.feature.PolynomialExpansion",
    "Interaction": "org.apache.spark.ml.feature.Interaction",
    "VectorSlicer": "org.apache.spark.ml.feature.VectorSlicer",
    "VectorIndexer": "org.apache.spark.ml.feature.VectorIndexer",
    "VectorIndexerModel": "org.apache.spark.ml.feature.VectorIndexerModel",
    "SQLTransformer": "org.apache.spark.ml.feature.SQLTransformer",
    "DCT": "org.apache.spark.ml.feature.DCT",
    "FeatureHasher": "org.apache.spark.ml.feature.FeatureHasher",
    "VectorSizeHint": "org.apache.spark.ml.feature.VectorSizeHint",
    "Word2Vec": "org.apache.spark.ml.feature.Word2Vec",
    "Word2VecModel": "org.apache.spark.ml.feature.Word2VecModel",
    "LDA": "org.apache.spark.ml.clustering.LDA",
    "LocalLDAModel": "org.apache.spark.ml.clustering.LocalLDAModel",
    "DistributedLDAModel": "org.apache.spark.ml.clustering.DistributedLDAModel",
    "PowerIterationClustering": "org.apache.spark.ml.clustering.PowerIterationClustering",
    "VarianceThresholdSelector": "org.apache.spark.ml.feature.VarianceThresholdSelector",
    "VarianceThresholdSelectorModel": "org.apache.spark.ml.feature.VarianceThresholdSelectorModel",
    "UnivariateFeatureSelector": "org.apache.spark.ml.feature.UnivariateFeatureSelector",
    "UnivariateFeatureSelectorModel": "org.apache.spark.ml.feature.UnivariateFeatureSelectorModel",
    "ChiSqSelector": "org.apache.spark.ml.feature.ChiSqSelector",
    "ChiSqSelectorModel": "org.apache.spark.ml.feature.ChiSqSelectorModel",
    "RFormula": "org.apache.spark.ml.feature.RFormula",
    "CountVectorizer": "org.apache.spark.ml.feature.CountVectorizer",
    "CountVectorizerModel": "org.apache.spark.ml.feature.CountVectorizerModel",
    "HashingTF": "org.apache.spark.ml.feature.HashingTF",
    "IDF": "org.apache.spark.ml.feature.IDF",
    "IDFModel": "org.apache.spark.ml.feature.IDFModel",
    "NGram": "org.apache.spark.ml.feature.NGram",
    "RegexTokenizer": "org.apache.spark.ml.feature.RegexTokenizer",
    "StopWordsRemover": "org.apache.spark.ml.feature.StopWordsRemover",
    "Tokenizer": "org.apache.spark.ml.feature.Tokenizer",
    "MultilabelClassificationEvaluator": "org.apache.spark.ml.evaluation.MultilabelClassificationEvaluator",
    "RankingEvaluator": "org.apache.spark.ml.evaluation.RankingEvaluator",
    "BucketedRandomProjectionLSH": "org.apache.spark.ml.feature.BucketedRandomProjectionLSH",
    "BucketedRandomProjectionLSHModel": "org.apache.spark.ml.feature.BucketedRandomProjectionLSHModel",
    "MinHashLSH": "org.apache.spark.ml.feature.MinHashLSH",
    "MinHashLSHModel": "org.apache.spark.ml.feature.MinHashLSHModel",
    "ALS": "org.apache.spark.ml.recommendation.ALS",
    "ALSModel": "org.apache.spark.ml.recommendation.ALSModel",
    "FPGrowth": "org.apache.spark.ml.fpm.FPGrowth",
    "FPGrowthModel": "org.apache.spark.ml.fpm.FPGrowthModel",
    "FMRegressor": "org.apache.spark.ml.regression.FMRegressor",
    "FMRegressionModel": "org.apache.spark.ml.regression.FMRegressionModel",
    "FMClassifier": "org.apache.spark.ml.classification.FMClassifier",
    "FMClassificationModel": "org.apache.spark.ml.classification.FMClassificationModel",
    "AFTSurvivalRegression": "org.apache.spark.ml.regression.AFTSurvivalRegression",
    "AFTSurvivalRegressionModel": "org.apache.spark.ml.regression.AFTSurvivalRegressionModel",
    "IsotonicRegression": "org.apache.spark.ml.regression.IsotonicRegression",
    "IsotonicRegressionModel": "org.apache.spark.ml.regression.IsotonicRegressionModel",
    "GaussianMixture": "org.apache.spark.ml.clustering.GaussianMixture",
    "GaussianMixtureModel": "org.apache.spark.ml.clustering.GaussianMixtureModel",
    "LinearSVC": "org.apache.spark.ml.classification.LinearSVC",
    "LinearSVCModel": "org.apache.spark.ml.classification.LinearSVCModel",
    "OneVsRest": "org.apache.spark.ml.classification.OneVsRest",
    "OneVsRestModel": "org.apache.spark.ml.classification.OneVsRestModel",
    "MultilayerPerceptronClassifier": "org.apache.spark.ml.classification.MultilayerPerceptronClassifier",
    "MultilayerPerceptronClassificationModel": "org.apache.spark.ml.classification.MultilayerPerceptronClassificationModel",
    "RFormulaModel": "org.apache.spark.ml.feature.RFormulaModel",
    "IndexToString": "org.apache.spark.ml.feature.IndexToString",
}
_PY = {
    "LinearRegression": "regression", "LinearRegressionModel": "regression",
    "DecisionTreeRegressor": "regression", "DecisionTreeRegressionModel": "regression",
    "RandomForestRegressor": "regression", "RandomForestRegressionModel": "regression",
    "DecisionTreeClassifier": "classification", "DecisionTreeClassificationModel": "classification",
    "RandomForestClassifier": "classification", "RandomForestClassificationModel": "classification",
    "LogisticRegression": "classification", "LogisticRegressionModel": "classification",
    "KMeans": "clustering", "KMeansModel": "clustering",
    "StandardScaler": "feature", "StandardScalerModel": "feature", "VectorAssembler": "feature",
    "StringIndexer": "feature", "StringIndexerModel": "feature", "Binarizer": "feature",
    "MinMaxScaler": "feature", "MinMaxScalerModel": "feature",
    "Pipeline": "pipeline", "PipelineModel": "pipeline",
    "RegressionEvaluator": "evaluation", "MulticlassClassificationEvaluator": "evaluation",
    "BinaryClassificationEvaluator": "evaluation", "ClusteringEvaluator": "evaluation",
    "CrossValidator": "tuning", "CrossValidatorModel": "tuning",
    "TrainValidationSplit": "tuning", "TrainValidationSplitModel": "tuning",
    "OneHotEncoder": "feature", "OneHotEncoderModel": "feature", "Imputer": "feature", "ImputerModel": "feature",
    "Bucketizer": "feature", "QuantileDiscretizer": "feature", "Normalizer": "feature", "PCA": "feature",
    "PCAModel": "feature",
    "GeneralizedLinearRegression": "regression", "GeneralizedLinearRegressionModel": "regression",
    "NaiveBayes": "classification", "NaiveBayesModel": "classification",
    "BisectingKMeans": "clustering", "BisectingKMeansModel": "clustering",
    "GBTRegressor": "regression", "GBTRegressionModel": "regression",
    "GBTClassifier": "classification", "GBTClassificationModel": "classification",
    "MaxAbsScaler": "feature",
    "MaxAbsScalerModel": "feature",
    "RobustScaler": "feature",
    "RobustScalerModel": "feature",
    "ElementwiseProduct": "feature",
    "PolynomialExpansion": "feature",
    "Interaction": "feature",
    "VectorSlicer": "feature",
    "VectorIndexer": "feature",
    "VectorIndexerModel": "feature",
    "SQLTransformer": "feature",
    "DCT": "feature",
    "FeatureHasher": "feature",
    "VectorSizeHint": "feature",
    "Word2Vec": "feature",
    "Word2VecModel": "feature",
    "LDA": "clustering",
    "LocalLDAModel": "clustering",
    "DistributedLDAModel": "clustering",
    "PowerIterationClustering": "clustering",
    "VarianceThresholdSelector": "feature",
    "VarianceThresholdSelectorModel": "feature",
    "UnivariateFeatureSelector": "feature",
    "UnivariateFeatureSelectorModel": "feature",
    "ChiSqSelector": "feature",
    "ChiSqSelectorModel": "feature",
    "RFormula": "feature",
    "CountVectorizer": "feature",
    "CountVectorizerModel": "feature",
    "HashingTF": "feature",
    "IDF": "feature",
    "IDFModel": "feature",
    "NGram": "feature",
    "RegexTokenizer": "feature",
    "StopWordsRemover": "feature",
    "Tokenizer": "feature",
    "MultilabelClassificationEvaluator": "evaluation", "RankingEvaluator": "evaluation",
    "BucketedRandomProjectionLSH": "feature",
    "BucketedRandomProjectionLSHModel": "feature",
    "MinHashLSH": "feature",
    "MinHashLSHModel": "feature",
    "ALS": "recommendation", "ALSModel": "recommendation",
    "FPGrowth": "fpm", "FPGrowthModel": "fpm",
    "FMRegressor": "regression", "FMRegressionModel": "regression",
    "FMClassifier": "classification", "FMClassificationModel": "classification",
    "AFTSurvivalRegression": "regression",
    "AFTSurvivalRegressionModel": "regression",
    "IsotonicRegression": "regression",
    "IsotonicRegressionModel": "regression",
    "GaussianMixture": "clustering",
    "GaussianMixtureModel": "clustering",
    "LinearSVC": "classification",
    "LinearSVCModel": "classification",
    "OneVsRest": "classification",
    "OneVsRestModel": "classification",
    "MultilayerPerceptronClassifier": "classification",
    "MultilayerPerceptronClassificationModel": "classification",
    "RFormulaModel": "feature",
    "IndexToString": "feature",
}


class JavaRandom:
    """``java.util.Random``: the 48-bit LCG and nextDouble, bit-exact."""

    _MUL, _ADD, _MASK = 0x5DEECE66D, 0xB, (1 << 48) - 1

    def __init__(self, seed: int):
        self._s = (int(seed) ^ self._MUL) & self._MASK

    def _next(self, bits: int) -> int:
        self._s = (self._s * self._MUL + self._ADD) & self._MASK
        return self._s >> (48 - bits)

    def next_double(self) -> float:
        return ((self._next(26) << 27) + self._next(27)) * (1.0 / (1 << 53))

    def next_int(self, bound: int) -> int:
        """``nextInt(bound)`` including Java's 32-bit overflow test in the rejection loop."""
        r = self._next(31)
        m = bound - 1
        if bound & m == 0:
            return (bound * r) >> 31
        u = r
        while True:
            r = u % bound
            v = (u - r + m) & 0xFFFFFFFF
            if v < 0x80000000:  # non-negative as a Java int
                return r
            u = self._next(31)

    def next_gaussian(self) -> float:
        """``nextGaussian``: Marsaglia's polar method, the second deviate cached."""
        g = getattr(self, "_gauss", None)
        if g is not None:
            self._gauss = None
            return g
        while True:
            v1 = 2.0 * self.next_double() - 1.0
            v2 = 2.0 * self.next_double() - 1.0
            s = v1 * v1 + v2 * v2
            if 0.0 < s < 1.0:
                break
        mul = math.sqrt(-2.0 * math.log(s) / s)
        self._gauss = v2 * mul
        return v1 * mul


def java_hash(s: str) -> int:
    """``java.lang.String.hashCode`` (Spark seeds default to the estimator class name's hash)."""
    h = 0
    for ch in s:
        h = (31 * h + ord(ch)) & 0xFFFFFFFF
    return h - (1 << 32) if h >= (1 << 31) else h


def jvm_class(obj) -> str:
    name = type(obj).__name__
    return _JVM.get(name, f"cml.{type(obj).__module__}.{name}")


def py_class_from_jvm(jvm: str):
    short = jvm.rsplit(".", 1)[-1]
    mod = _PY.get(short)
    if mod is None:
        raise ValueError(f"unknown model class {jvm}")
    m = importlib.import_module(f"clustermachinelearningforhospitalnetworks_apache_spark_amd.ml.{mod}")
    return getattr(m, short)


def _json_value(v):
    if isinstance(v, (np.integer,)):
        return int(v)
    if isinstance(v, (np.floating,)):
        return float(v)
    if isinstance(v, np.ndarray):
        return v.tolist()
    return v


def _comm():
    from ..sql.session import SparkSession
    s = SparkSession.getActiveSession()
    if s is None:
        from ..parallel.comm import local_comm
        return local_comm()
    return s._comm


def _is_extension_param(instance, name: str) -> bool:
    """Params that Spark's class does not have (docs start with "cml") — kept out of Spark's
    paramMap/defaultParamMap, whose readers reject unknown names, and stored under cml keys."""
    spec = getattr(type(instance), "_all_params", {}).get(name)
    return bool(spec) and str(spec[1]).startswith("cml")


def write_metadata(instance, path: str, extra: Optional[Dict[str, Any]] = None, param_map=None) -> None:
    pm = param_map if param_map is not None else instance._paramMap
    dm = instance._defaultParamMap
    md = {"class": jvm_class(instance), "timestamp": int(time.time() * 1000), "sparkVersion": SPARK_VERSION,
          "uid": instance.uid,
          "paramMap": {k: _json_value(v) for k, v in pm.items() if not _is_extension_param(instance, k)},
          "defaultParamMap": {k: _json_value(v) for k, v in dm.items() if not _is_extension_param(instance, k)}}
    ext = {k: _json_value(v) for k, v in pm.items() if _is_extension_param(instance, k)}
    ext_d = {k: _json_value(v) for k, v in dm.items() if _is_extension_param(instance, k)}
    if ext:
        md["cmlParamMap"] = ext
    if ext_d:
        md["cmlDefaultParamMap"] = ext_d
    if extra:
        md.update(extra)
    d = os.path.join(path, "metadata")
    os.makedirs(d, exist_ok=True)
    with open(os.path.join(d, "part-00000"), "w") as fh:
        fh.write(json.dumps(md, separators=(",", ":")) + "\n")
    open(os.path.join(d, "_SUCCESS"), "w").close()
    from ..utils.fault import maybe_fail
    maybe_fail("ml.save")  # crash point: metadata written, data not yet


def read_metadata(path: str) -> Dict[str, Any]:
    with open(os.path.join(path, "metadata", "part-00000")) as fh:
        return json.loads(fh.readline())


def apply_params(instance, md: Dict[str, Any]) -> None:
    instance.uid = md.get("uid", instance.uid)
    for key in ("defaultParamMap", "cmlDefaultParamMap"):
        for k, v in md.get(key, {}).items():
            if instance.hasParam(k):
                instance._defaultParamMap[k] = v
    for key in ("paramMap", "cmlParamMap"):
        for k, v in md.get(key, {}).items():
            if instance.hasParam(k):
                instance._paramMap[k] = v


def write_parquet(path: str, sub: str, table) -> None:
    import pyarrow.parquet as pq
    d = os.path.join(path, sub)
    os.makedirs(d, exist_ok=True)
    pq.write_table(table, os.path.join(d, f"part-00000-{uuid.uuid4()}-c000.snappy.parquet"), compression="snappy")
    open(os.path.join(d, "_SUCCESS"), "w").close()


def read_parquet(path: str, sub: str):
    import pyarrow as pa
    import pyarrow.parquet as pq
    d = os.path.join(path, sub)
    files = sorted(f for f in os.listdir(d) if f.endswith(".parquet"))
    return pa.concat_tables([pq.read_table(os.path.join(d, f)) for f in files])


# ---------------------------------------------------------------------------------------------- UDT encoders

def vector_struct(v) -> Dict[str, Any]:
    """VectorUDT row value (dense)."""
    arr = np.asarray(v.toArray() if hasattr(v, "toArray") else v, dtype=np.float64)
    return {"type": 1, "size": None, "indices": None, "values": arr.tolist()}


def vector_from_struct(s) -> np.ndarray:
    if s is None:
        return None
    if s["type"] == 0:
        a = np.zeros(s["size"])
        a[np.asarray(s["indices"], dtype=np.int64)] = s["values"]
        return a
    return np.asarray(s["values"], dtype=np.float64)


def matrix_struct(m: np.ndarray) -> Dict[str, Any]:
    """MatrixUDT row value (dense, column-major, isTransposed=false)."""
    m = np.asarray(m, dtype=np.float64)
    return {"type": 1, "numRows": int(m.shape[0]), "numCols": int(m.shape[1]), "colPtrs": None,
            "rowIndices": None, "values": m.T.reshape(-1).tolist(), "isTransposed": False}


def matrix_from_struct(s) -> np.ndarray:
    vals = np.asarray(s["values"], dtype=np.float64)
    if s.get("isTransposed"):
        return vals.reshape(s["numRows"], s["numCols"])
    return vals.reshape(s["numCols"], s["numRows"]).T


def vector_arrow_type():
    from ..io.arrow import vector_udt_arrow
    return vector_udt_arrow()


def matrix_arrow_type():
    import pyarrow as pa
    return pa.struct([pa.field("type", pa.int8(), nullable=False), pa.field("numRows", pa.int32(), nullable=False),
                      pa.field("numCols", pa.int32(), nullable=False),
                      pa.field("colPtrs", pa.list_(pa.field("element", pa.int32(), nullable=False))),
                      pa.field("rowIndices", pa.list_(pa.field("element", pa.int32(), nullable=False))),
                      pa.field("values", pa.list_(pa.field("element", pa.float64(), nullable=False))),
                      pa.field("isTransposed", pa.bool_(), nullable=False)])


# ---------------------------------------------------------------------------------------------- writer/reader

def _pid_alive(pid: int) -> bool:
    try:
        os.kill(pid, 0)
    except ProcessLookupError:
        return False
    except (PermissionError, OSError):
        return True
    return True


def recover_save(path: str) -> None:
    """Finish or roll back a save that crashed between its two renames. MLWriter.save moves the
    previous model to ``.<name>.old-<pid>`` only after the new one is complete in
    ``.<name>.tmp-<pid>``, so when ``path`` is missing, a complete new model (the tmp of the same
    writer) is promoted, else the old model is restored. Leftovers of dead writers are removed.
    Writers that are still alive are left alone (they finish their own renames)."""
    parent = os.path.dirname(os.path.abspath(path)) or "."
    base = os.path.basename(path)
    try:
        entries = os.listdir(parent)
    except FileNotFoundError:
        return
    pat = re.compile(r"^\." + re.escape(base) + r"\.(tmp|old)-(\d+)$")
    dead = {}
    for e in entries:
        m = pat.match(e)
        if m and not _pid_alive(int(m.group(2))):
            dead.setdefault(int(m.group(2)), {})[m.group(1)] = os.path.join(parent, e)
    for pid, parts in sorted(dead.items()):
        if not os.path.exists(path) and "old" in parts:
            os.replace(parts.pop("tmp") if "tmp" in parts else parts.pop("old"), path)
        for leftover in parts.values():
            shutil.rmtree(leftover, ignore_errors=True)


class MLWriter:
    def __init__(self, instance):
        self.instance = instance
        self._overwrite = False

    def overwrite(self) -> "MLWriter":
        self._overwrite = True
        return self

    def option(self, key, value) -> "MLWriter":
        return self

    def session(self, spark) -> "MLWriter":
        return self

    def save(self, path: str) -> None:
        """Crash-consistent save: the model is written into a sibling temp directory and renamed
        into place, so a failure mid-save never leaves a half-written model and,
        with overwrite, the previous model survives until the new one is complete."""
        from ..utils.trace import trace
        with trace("MLWriter.save"):
            self._save(path)

    def _save(self, path: str) -> None:
        from ..io.reader import strip_scheme
        path = strip_scheme(path).rstrip("/")
        comm = _comm()
        if comm.is_root:
            recover_save(path)
        comm.barrier()
        if os.path.exists(path) and not self._overwrite:
            raise FileExistsError(f"Path {path} already exists. To overwrite it, use write().overwrite().save(path)")
        comm.barrier()
        err = None
        if comm.is_root:
            parent = os.path.dirname(os.path.abspath(path))
            os.makedirs(parent, exist_ok=True)
            tmp = os.path.join(parent, f".{os.path.basename(path)}.tmp-{os.getpid()}")
            if os.path.exists(tmp):
                shutil.rmtree(tmp)
            os.makedirs(tmp)
            try:
                self.instance._save_impl(tmp)
                if os.path.exists(path):
                    old = os.path.join(parent, f".{os.path.basename(path)}.old-{os.getpid()}")
                    os.replace(path, old)
                    os.replace(tmp, path)
                    shutil.rmtree(old, ignore_errors=True)
                else:
                    os.replace(tmp, path)
            except BaseException as e:  # keep the previous model; drop the partial one
                shutil.rmtree(tmp, ignore_errors=True)
                err = e
        comm.barrier()
        if err is not None:
            raise err


class MLWritable:
    def write(self) -> MLWriter:
        return MLWriter(self)

    def save(self, path: str) -> None:
        self.write().save(path)

    def _save_impl(self, path: str) -> None:
        write_metadata(self, path)


class MLReader:
    def __init__(self, cls):
        self.cls = cls

    def load(self, path: str):
        from ..io.reader import strip_scheme
        path = strip_scheme(path)
        if not os.path.exists(path):
            recover_save(path.rstrip("/"))
        md = read_metadata(path)
        cls = py_class_from_jvm(md["class"]) if self.cls is None else self.cls
        return cls._load_impl(path, md)

    def session(self, spark) -> "MLReader":
        return self


class MLReadable:
    @classmethod
    def read(cls) -> MLReader:
        return MLReader(cls)

    @classmethod
    def load(cls, path: str):
        return cls.read().load(path)

    @classmethod
    def _load_impl(cls, path: str, md: Dict[str, Any]):
        inst = cls()
        apply_params(inst, md)
        return inst


DefaultParamsWritable = MLWritable
DefaultParamsReadable = MLReadable


def load(path: str):
    """Load any saved estimator/model/pipeline by its metadata class."""
    return MLReader(None).load(path)


def java_double_str(v: float) -> str:
    """``java.lang.Double.toString``: shortest round-trip digits, plain notation for
    1e-3 <= |v| < 1e7 (at least one fractional digit), ``d.dddE±n`` otherwise."""
    import decimal
    v = float(v)
    if math.isnan(v):
        return "NaN"
    if math.isinf(v):
        return "Infinity" if v > 0 else "-Infinity"
    if v == 0.0:
        return "-0.0" if math.copysign(1.0, v) < 0 else "0.0"
    sign, digits, exp = decimal.Decimal(repr(v)).as_tuple()
    ds = "".join(map(str, digits)).rstrip("0") or "0"
    point = len(digits) + exp          # decimal point position relative to the digit string
    a = abs(v)
    neg = "-" if sign else ""
    if 1e-3 <= a < 1e7:
        if point <= 0:
            return f"{neg}0.{'0' * -point}{ds}"
        if point >= len(ds):
            return f"{neg}{ds}{'0' * (point - len(ds))}.0"
        return f"{neg}{ds[:point]}.{ds[point:]}"
    return f"{neg}{ds[0]}.{ds[1:] or '0'}E{point - 1}"
