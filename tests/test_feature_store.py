"""Feature store (ML 10 - Feature Store.py:45-348)."""
import numpy as np
import pandas as pd
import pytest

from cdnaml import tracking as mlflow
from cdnaml.feature_store import FeatureLookup, FeatureStoreClient, feature_table
from cdnaml.sql import functions as F
from cdnaml.sql import types as T


@pytest.fixture
def airbnb(spark, tmp_path):
    rng = np.random.default_rng(0)
    n = 400
    pdf = pd.DataFrame({"bedrooms": rng.integers(0, 4, n).astype(float),
                        "accommodates": rng.integers(1, 8, n).astype(float),
                        "review_scores_accuracy": rng.uniform(5, 10, n),
                        "review_scores_value": rng.uniform(5, 10, n),
                        "room_type": rng.choice(["Entire", "Private"], n)})
    pdf["price"] = 40 * pdf.bedrooms + 10 * pdf.accommodates + rng.normal(0, 5, n)
    path = str(tmp_path / "clean.delta")
    spark.createDataFrame(pdf).write.format("delta").save(path)
    mlflow.set_tracking_uri(str(tmp_path / "mlruns"))
    yield spark.read.format("delta").load(path).coalesce(1).withColumn("index", F.monotonically_increasing_id()), path
    while mlflow.active_run():
        mlflow.end_run()
    mlflow.set_tracking_uri(None)


def test_feature_store_end_to_end(spark, airbnb):
    from sklearn.ensemble import RandomForestRegressor
    from sklearn.model_selection import train_test_split

    df, src = airbnb
    spark.sql("CREATE DATABASE IF NOT EXISTS fsdb")
    table = "fsdb.airbnb_abc123"
    fs = FeatureStoreClient()
    numeric = [f.name for f in df.schema.fields if f.dataType == T.DoubleType() and f.name != "price"]

    @feature_table
    def select_numeric_features(data):
        return data.select(["index"] + numeric)

    feats = select_numeric_features(df)
    fs.create_feature_table(name=table, keys=["index"], features_df=feats, schema=feats.schema,
                            description="Numeric features of airbnb data")
    ft = fs.get_feature_table(table)
    assert ft.description == "Numeric features of airbnb data"
    assert any(src.rstrip("/") in p for p in ft.path_data_sources)
    assert fs.read_table(table).count() == 400
    with pytest.raises(ValueError):
        fs.create_feature_table(name=table, keys=["index"], features_df=feats)

    inference = df.select("index", "price", (F.rand() * 0.5 - 0.25).alias("score_diff_from_last_month"))
    ts = fs.create_training_set(inference, [FeatureLookup(table_name=table, lookup_key="index")], label="price",
                                exclude_columns="index")
    pdf = ts.load_df().toPandas()
    assert "index" not in pdf.columns and set(numeric) <= set(pdf.columns)
    assert len(pdf) == 400
    X = pdf.drop("price", axis=1)
    y = pdf["price"]
    Xtr, Xte, ytr, yte = train_test_split(X, y, test_size=0.2, random_state=42)
    with mlflow.start_run():
        rf = RandomForestRegressor(max_depth=3, n_estimators=20, random_state=42).fit(Xtr, ytr)
        fs.log_model(model=rf, artifact_path="feature-store-model", flavor=mlflow.sklearn, training_set=ts,
                     registered_model_name="feature_store_airbnb", input_example=Xtr[:5],
                     signature=mlflow.models.infer_signature(Xtr, ytr))
    scored = fs.score_batch("models:/feature_store_airbnb/1", inference.drop("price"), result_type="double")
    out = scored.toPandas().sort_values("index")
    ref = rf.predict(out[list(X.columns)])
    np.testing.assert_allclose(out.prediction.values, ref, rtol=1e-6)

    # overwrite with a condensed schema: dropped columns read back as nulls (ML 10:299-348)
    reviews = ["review_scores_accuracy", "review_scores_value"]

    @feature_table
    def condensed(data):
        return (data.select(["index"] + numeric)
                .withColumn("average_review_score", F.expr("+".join(reviews)) / F.lit(len(reviews)))
                .drop(*reviews))

    fs.write_table(name=table, df=condensed(df), mode="overwrite")
    latest = fs.read_table(name=table).toPandas()
    assert "average_review_score" in latest.columns
    assert latest["review_scores_accuracy"].isna().all()


def test_feature_store_merge_upsert(spark, tmp_path):
    fs = FeatureStoreClient()
    a = spark.createDataFrame(pd.DataFrame({"id": [1, 2, 3], "f": [1.0, 2.0, 3.0]}))
    fs.create_table("default.t_merge", primary_keys="id", df=a)
    b = spark.createDataFrame(pd.DataFrame({"id": [3, 4], "f": [30.0, 40.0]}))
    fs.write_table("default.t_merge", b, mode="merge")
    out = fs.read_table("default.t_merge").orderBy("id").toPandas()
    assert out.id.tolist() == [1, 2, 3, 4]
    assert out.f.tolist() == [1.0, 2.0, 30.0, 40.0]
    with pytest.raises(ValueError):
        fs.write_table("default.t_merge", b.drop("id"), mode="merge")
    fs.drop_table("default.t_merge")
    with pytest.raises(ValueError):
        fs.get_table("default.t_merge")
