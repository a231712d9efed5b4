"""pyspark.ml-compatible estimators, transformers, evaluators and persistence."""
from .base import Estimator, Evaluator, Model, Transformer
from .pipeline import Pipeline, PipelineModel

__all__ = ["Estimator", "Evaluator", "Model", "Transformer", "Pipeline", "PipelineModel"]
