#!/usr/bin/env python3
"""The reference workflow (alexv879/...-Apache-Spark, mllearnforhospitalnetwork.py), end to end,
with its INTENDED semantics on this engine:

  CSV uploads --readStream(+watermark, ingest_time)--> unbounded append table (checkpointed,
  foreachBatch per-batch retrain hook)  --SQL training window--> na.drop --> VectorAssembler
  --> randomSplit(0.7/0.3, seed 42) --> LinearRegression / DecisionTreeRegressor /
  RandomForestRegressor --> RMSE;  LOS_binary = LOS > 5.0 --> DT / RF classifiers --> accuracy;
  prediction + residual plots (saved, headless); feature importances; model save (Spark
  format, overwrite); operational insights report; stop.

No HDFS here: ``hdfs://namenode:9000/...`` paths map onto ``$CML_HDFS_ROOT`` (default ./hdfs).
Synthetic uploads with the reference schema are generated when the input dir is empty.

    python examples/hospital_resource_prediction.py --master local[2]
    python examples/hospital_resource_prediction.py --master mi355x          # one GPU
    torchrun --nproc-per-node 8 --master-addr 127.0.0.1 examples/hospital_resource_prediction.py --master mi355x[8]
"""
from __future__ import annotations

import argparse
import os
import sys

import numpy as np
import pandas as pd

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from clustermachinelearningforhospitalnetworks_apache_spark_amd.ml.classification import (  # noqa: E402
    DecisionTreeClassifier, RandomForestClassifier)
from clustermachinelearningforhospitalnetworks_apache_spark_amd.ml.evaluation import (  # noqa: E402
    MulticlassClassificationEvaluator, RegressionEvaluator)
from clustermachinelearningforhospitalnetworks_apache_spark_amd.ml.feature import VectorAssembler  # noqa: E402
from clustermachinelearningforhospitalnetworks_apache_spark_amd.ml.regression import (  # noqa: E402
    DecisionTreeRegressor, LinearRegression, RandomForestRegressor)
from clustermachinelearningforhospitalnetworks_apache_spark_amd.sql import SparkSession  # noqa: E402
from clustermachinelearningforhospitalnetworks_apache_spark_amd.sql.functions import current_timestamp, when  # noqa
from clustermachinelearningforhospitalnetworks_apache_spark_amd.sql.types import (  # noqa: E402
    DoubleType, IntegerType, StringType, StructField, StructType, TimestampType)

CONFIG = {
    "appName": "HospitalResourcePredictionExtended",
    "hdfsInputPath": "hdfs://namenode:9000/hospitals/incoming/",
    "checkpointLocation": "hdfs://namenode:9000/checkpoints/hospital_stream/",
    "outputTable": "hospital_unbounded_table",
    "trainingWindowStart": "2025-03-31 22:00:00",
    "trainingWindowEnd": "2025-03-31 23:00:00",
    "hdfsMaster": "spark://master-node-address:7077",
    "modelSavePath": "hdfs://namenode:9000/hospitals/models/latest_model",
    "losThreshold": 5.0,
}


def synth_uploads(path: str, n_files: int = 4, rows: int = 2500, seed: int = 7) -> None:
    """Hospital uploads with the reference schema (ref.py:64-72); a few nulls to exercise na.drop."""
    os.makedirs(path, exist_ok=True)
    rs = np.random.RandomState(seed)
    t0 = pd.Timestamp("2025-03-31 21:30:00")
    for f in range(n_files):
        n = rows
        adm = rs.randint(0, 60, n)
        occ = rs.randint(50, 400, n)
        er = rs.randint(0, 40, n)
        season = rs.rand(n)
        los = 1.5 + 0.04 * adm + 0.008 * occ + 0.06 * er + 2.5 * season + rs.randn(n) * 0.5
        ts = t0 + pd.to_timedelta(rs.randint(0, 7200, n), unit="s")
        pdf = pd.DataFrame({"hospital_id": [f"H{(f * 7 + i) % 12:02d}" for i in range(n)],
                            "event_time": ts.strftime("%Y-%m-%d %H:%M:%S"), "admission_count": adm,
                            "current_occupancy": occ, "emergency_visits": er,
                            "seasonality_index": season.round(4), "length_of_stay": los.round(3)})
        pdf["emergency_visits"] = pdf["emergency_visits"].astype("Int64")  # nullable int: no "12.0" in the CSV
        pdf.loc[rs.rand(n) < 0.01, "emergency_visits"] = pd.NA
        pdf.to_csv(os.path.join(path, f"hospital_upload_{f:03d}.csv"), index=False)


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--master", default=CONFIG["hdfsMaster"])
    ap.add_argument("--out", default=os.environ.get("CML_HDFS_ROOT", os.path.join(os.getcwd(), "hdfs")))
    ap.add_argument("--plots", default=None, help="directory for the two regression plots (headless savefig)")
    ap.add_argument("--synth-files", type=int, default=4, help="synthetic uploads when the input dir is empty")
    ap.add_argument("--synth-rows", type=int, default=2500, help="rows per synthetic upload file")
    ap.add_argument("--trace", action="store_true", help="print per-phase timings (utils.trace)")
    args = ap.parse_args(argv)
    if args.trace:
        from clustermachinelearningforhospitalnetworks_apache_spark_amd.utils.trace import TRACER
        TRACER.enable(sync=True)
    os.environ["CML_HDFS_ROOT"] = args.out

    spark = (SparkSession.builder.appName(CONFIG["appName"]).master(args.master)
             .config("spark.sql.warehouse.dir", os.path.join(args.out, "warehouse")).getOrCreate())
    root = spark.rank == 0
    from clustermachinelearningforhospitalnetworks_apache_spark_amd.io.reader import strip_scheme
    incoming = strip_scheme(CONFIG["hdfsInputPath"])
    if root and not (os.path.isdir(incoming) and os.listdir(incoming)):
        synth_uploads(incoming, n_files=args.synth_files, rows=args.synth_rows)
    spark._comm.barrier()

    schema = StructType([
        StructField("hospital_id", StringType(), True),
        StructField("event_time", TimestampType(), True),
        StructField("admission_count", IntegerType(), True),
        StructField("current_occupancy", IntegerType(), True),
        StructField("emergency_visits", IntegerType(), True),
        StructField("seasonality_index", DoubleType(), True),
        StructField("length_of_stay", DoubleType(), True),
    ])
    streaming_df = spark.readStream.option("header", True).schema(schema).csv(CONFIG["hdfsInputPath"])
    streaming_df = streaming_df.withWatermark("event_time", "10 minutes")
    streaming_df = streaming_df.withColumn("ingest_time", current_timestamp())

    feature_cols = ["admission_count", "current_occupancy", "emergency_visits", "seasonality_index"]
    assembler = VectorAssembler(inputCols=feature_cols, outputCol="features")
    per_batch_rmse = []

    def train_model_on_batch(batch_df, batch_id):  # the reference's intended per-batch hook (ref.py:91-106)
        data = assembler.transform(batch_df.na.drop())
        if data.count() < 10:
            return
        model = LinearRegression(featuresCol="features", labelCol="length_of_stay").fit(data)
        predictions = model.transform(data)  # ref.py:99
        model.write().overwrite().save(os.path.join(args.out, "models", f"linear_regression_model_batch_{batch_id}"))
        predictions.show()  # ref.py:106 (every rank takes part; rank 0 prints)
        per_batch_rmse.append((batch_id, model.summary.rootMeanSquaredError))

    query_stream = (streaming_df.writeStream.foreachBatch(train_model_on_batch).format("delta")
                    .outputMode("append").option("checkpointLocation", CONFIG["checkpointLocation"])
                    .trigger(availableNow=True).table(CONFIG["outputTable"]))
    query_stream.awaitTermination()  # the reference leaves this commented out (D7); here the batch part waits

    training_window_query = f"""
        SELECT *
        FROM {CONFIG["outputTable"]}
        WHERE event_time BETWEEN '{CONFIG["trainingWindowStart"]}' AND '{CONFIG["trainingWindowEnd"]}'
    """
    training_df = spark.sql(training_window_query).na.drop()

    final_data = assembler.transform(training_df).select("features", "length_of_stay")
    train_data, test_data = final_data.randomSplit([0.7, 0.3], seed=42)

    lr_model = LinearRegression(featuresCol="features", labelCol="length_of_stay").fit(train_data)
    lr_predictions = lr_model.transform(test_data)
    dt_model = DecisionTreeRegressor(featuresCol="features", labelCol="length_of_stay").fit(train_data)
    dt_predictions = dt_model.transform(test_data)
    rf_model = RandomForestRegressor(featuresCol="features", labelCol="length_of_stay").fit(train_data)
    rf_predictions = rf_model.transform(test_data)

    reg_evaluator = RegressionEvaluator(labelCol="length_of_stay", predictionCol="prediction", metricName="rmse")
    lr_rmse = reg_evaluator.evaluate(lr_predictions)
    dt_rmse = reg_evaluator.evaluate(dt_predictions)
    rf_rmse = reg_evaluator.evaluate(rf_predictions)

    training_df = training_df.withColumn(
        "LOS_binary", when(training_df["length_of_stay"] > CONFIG["losThreshold"], 1).otherwise(0))
    classification_data = assembler.transform(training_df).select("features", "LOS_binary")
    class_train, class_test = classification_data.randomSplit([0.7, 0.3], seed=42)
    dt_class_model = DecisionTreeClassifier(featuresCol="features", labelCol="LOS_binary").fit(class_train)
    rf_class_model = RandomForestClassifier(featuresCol="features", labelCol="LOS_binary").fit(class_train)
    class_evaluator = MulticlassClassificationEvaluator(labelCol="LOS_binary", predictionCol="prediction",
                                                        metricName="accuracy")
    dt_accuracy = class_evaluator.evaluate(dt_class_model.transform(class_test))
    rf_accuracy = class_evaluator.evaluate(rf_class_model.transform(class_test))

    predictions_pd = lr_predictions.select("length_of_stay", "prediction").toPandas()
    predictions_pd["residual"] = predictions_pd["length_of_stay"] - predictions_pd["prediction"]
    if args.plots and root:
        from clustermachinelearningforhospitalnetworks_apache_spark_amd.utils.report import regression_plots
        regression_plots(predictions_pd, args.plots, model_name="Linear Regression")

    save = CONFIG["modelSavePath"]
    lr_model.write().overwrite().save(save + "/lr")
    dt_model.write().overwrite().save(save + "/dt")
    rf_model.write().overwrite().save(save + "/rf")

    if root:
        print(f"Training-window rows: {training_df.count()}  (streamed batches retrained: {len(per_batch_rmse)})")
        print(f"Linear Regression RMSE: {lr_rmse}")
        print(f"Decision Tree Regression RMSE: {dt_rmse}")
        print(f"Random Forest Regression RMSE: {rf_rmse}")
        print(f"Decision Tree Classifier Accuracy: {dt_accuracy}")
        print(f"Random Forest Classifier Accuracy: {rf_accuracy}")
        print("\n--- Feature Importances ---")
        print("Decision Tree Regressor Feature Importances:")
        for feature, importance in zip(feature_cols, dt_model.featureImportances):
            print(f"{feature}: {importance}")
        print("Random Forest Regressor Feature Importances:")
        for feature, importance in zip(feature_cols, rf_model.featureImportances):
            print(f"{feature}: {importance}")
        from clustermachinelearningforhospitalnetworks_apache_spark_amd.utils.report import operational_insights
        print(operational_insights(lr_rmse, dt_rmse, rf_rmse, dt_accuracy, rf_accuracy))
        if args.trace:
            from clustermachinelearningforhospitalnetworks_apache_spark_amd.utils.trace import TRACER
            print(TRACER.report())
    spark.stop()
    return {"lr_rmse": lr_rmse, "dt_rmse": dt_rmse, "rf_rmse": rf_rmse, "dt_accuracy": dt_accuracy,
            "rf_accuracy": rf_accuracy, "batches": per_batch_rmse, "n_pred": len(predictions_pd)}


if __name__ == "__main__":
    main()
