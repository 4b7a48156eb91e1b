"""ML 13 many-models flow, timed four ways (10 IoT devices x 10k rows by default):

  sklearn-serial    groupBy().applyInPandas(sklearn forest per device), one group at a time
  sklearn-threads   the same with the concurrent group dispatch (cdnaml.applyInPandas.parallelism)
  engine-serial     this engine's RandomForestRegressor fitted per device (filter + fit, one by one)
  engine-batched    GroupedEstimator: every device's forest in one batched pass over shared bins

    python bench/many_models.py [--groups 10] [--rows-per-group 10000] [--trees 10]
"""
import argparse
import os
import sys
import time

import numpy as np
import pandas as pd

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--groups", type=int, default=10)
    ap.add_argument("--rows-per-group", type=int, default=10000)
    ap.add_argument("--trees", type=int, default=10)
    ap.add_argument("--depth", type=int, default=5)
    args = ap.parse_args()
    import torch

    import cdnaml
    from cdnaml.ml.feature import VectorAssembler
    from cdnaml.ml.grouped import GroupedEstimator
    from cdnaml.ml.regression import RandomForestRegressor
    from cdnaml.sql import functions as F
    spark = cdnaml.SparkSession.builder.getOrCreate()
    G, n = args.groups, args.groups * args.rows_per_group
    rng = np.random.default_rng(0)
    ids = np.arange(n)
    pdf = pd.DataFrame({"record_id": ids, "device_id": ids % G})
    for k in (1, 2, 3):
        pdf[f"feature_{k}"] = rng.random(n) * k
    pdf["label"] = pdf[["feature_1", "feature_2", "feature_3"]].sum(1) + rng.random(n)
    df = VectorAssembler(inputCols=["feature_1", "feature_2", "feature_3"], outputCol="features").transform(
        spark.createDataFrame(pdf)).cache()
    df.count()
    schema = "device_id integer, n_used integer, mse float"

    def train_model(p):
        from sklearn.ensemble import RandomForestRegressor as SkRF
        X, y = p[["feature_1", "feature_2", "feature_3"]], p["label"]
        rf = SkRF(n_estimators=args.trees, max_depth=args.depth, random_state=0).fit(X, y)
        return pd.DataFrame([[int(p.device_id.iloc[0]), len(p), float(((rf.predict(X) - y) ** 2).mean())]],
                            columns=["device_id", "n_used", "mse"])

    def sync():
        if spark.device.type == "cuda":
            torch.cuda.synchronize()

    def timed(fn, reps=3):
        fn()
        sync()
        t0 = time.perf_counter()
        for _ in range(reps):
            fn()
        sync()
        return (time.perf_counter() - t0) / reps * 1e3

    res = {}
    spark.conf.set("cdnaml.applyInPandas.parallelism", "1")
    res["sklearn-serial"] = timed(lambda: df.groupby("device_id").applyInPandas(train_model, schema).toPandas(), 1)
    spark.conf.set("cdnaml.applyInPandas.parallelism", str(G))
    res["sklearn-threads"] = timed(lambda: df.groupby("device_id").applyInPandas(train_model, schema).toPandas(), 1)
    est = RandomForestRegressor(numTrees=args.trees, maxDepth=args.depth, seed=1)

    def serial():
        return [est.fit(df.filter(F.col("device_id") == g)) for g in range(G)]
    res["engine-serial"] = timed(serial)
    res["engine-batched"] = timed(lambda: GroupedEstimator(estimator=est, groupCol="device_id").fit(df))
    for k, v in res.items():
        print(f"{k:16s} {v:9.1f} ms", flush=True)
    print(f"batched speed-up over engine-serial: {res['engine-serial'] / res['engine-batched']:.1f}x; "
          f"threads over serial sklearn: {res['sklearn-serial'] / res['sklearn-threads']:.1f}x")


if __name__ == "__main__":
    main()
