"""MI355X-native distributed tabular-ML engine with a pyspark-compatible API.

Capabilities of alexv879/ClusterMachineLearningForHospitalNetworks-Apache-Spark
(streaming ingest -> unbounded table -> windowed SQL -> VectorAssembler ->
LinearRegression / DecisionTree / RandomForest regressors and classifiers ->
RMSE / accuracy evaluation -> feature importances -> Spark-format model save),
plus KMeans, StandardScaler, LogisticRegression and Pipeline, running on
hand-written gfx950 HIP kernels with RCCL data parallelism over xGMI.

    from clustermachinelearningforhospitalnetworks_apache_spark_amd.sql import SparkSession
    from clustermachinelearningforhospitalnetworks_apache_spark_amd.ml.clustering import KMeans
"""
__version__ = "0.1.0"

from . import sql  # noqa: E402,F401
