import pytest
"""AutoML (SURVEY §2.6 T5; ML 09 - AutoML.py:35-90)."""
import numpy as np
import pandas as pd

from cdnaml import automl
from cdnaml import tracking as mlflow
from cdnaml.ml.evaluation import RegressionEvaluator


@pytest.mark.slow
def test_automl_regress_and_serve(spark, tmp_path):
    mlflow.set_tracking_uri(str(tmp_path / "mlruns"))
    try:
        rng = np.random.default_rng(0)
        n = 1200
        pdf = pd.DataFrame({"room": rng.choice(["a", "b", "c"], n), "acc": rng.integers(1, 8, n),
                            "x": rng.normal(size=n)})
        pdf["price"] = 30 * pdf.acc + (pdf.room == "a") * 50 + 5 * pdf.x + rng.normal(0, 3, n)
        train_df, test_df = spark.createDataFrame(pdf).randomSplit([.8, .2], seed=42)
        summary = automl.regress(train_df, target_col="price", primary_metric="rmse", timeout_minutes=5,
                                 max_trials=3)
        best = summary.best_trial
        assert best.metrics["val_rmse"] == min(t.metrics["val_rmse"] for t in summary.trials)
        predict = mlflow.pyfunc.spark_udf(spark, f"runs:/{best.mlflow_run_id}/model")
        pred_df = test_df.withColumn("prediction", predict(*test_df.drop("price").columns))
        rmse = RegressionEvaluator(labelCol="price").evaluate(pred_df)
        assert rmse < 0.5 * float(np.std(pdf.price))
    finally:
        mlflow.set_tracking_uri(None)


def test_automl_classify(spark, tmp_path):
    mlflow.set_tracking_uri(str(tmp_path / "mlruns"))
    try:
        rng = np.random.default_rng(1)
        n = 1000
        pdf = pd.DataFrame({"a": rng.normal(size=n), "b": rng.normal(size=n), "c": rng.choice(["u", "v"], n)})
        pdf["label"] = ((pdf.a + (pdf.c == "u")) > 0.5).astype(int)
        s = automl.classify(spark.createDataFrame(pdf), target_col="label", primary_metric="accuracy",
                            timeout_minutes=5, max_trials=2)
        assert s.best_trial.metrics["val_accuracy"] > 0.85
    finally:
        mlflow.set_tracking_uri(None)
