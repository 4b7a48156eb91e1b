"""SPMD scenarios run both single-process and under torchrun (gloo, CPU).

    python -m torch.distributed.run --nproc-per-node 2 --master-addr 127.0.0.1 \
        --master-port P tests/dist_worker.py <scenario> <out.json>

Every rank computes the same global results; rank 0 writes them as JSON so the
test can compare the W-rank answers against the 1-process answers.
"""
import json
import os
import sys

import numpy as np
import pandas as pd

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def _session():
    import cdnaml
    return cdnaml.SparkSession.builder.getOrCreate()


def _data(spark, n=6000, d=4, seed=0):
    """Same global table regardless of world size (rows sliced by rank)."""
    rng = np.random.default_rng(seed)
    X = rng.normal(size=(n, d))
    cat = rng.choice(["a", "b", "c"], n)
    y = X @ np.arange(1.0, d + 1) + (cat == "a") * 3.0 + 0.1 * rng.normal(size=n)
    pdf = pd.DataFrame(X, columns=[f"x{i}" for i in range(d)])
    pdf["cat"] = cat
    pdf["label"] = y
    pdf["k"] = np.arange(n) % 7
    return spark.createDataFrame(pdf)


def scenario_frame(spark):
    from cdnaml.sql import functions as F
    df = _data(spark)
    out = {"count": df.count()}
    tr, te = df.randomSplit([0.8, 0.2], seed=42)
    out["train"] = tr.count()
    g = df.groupBy("k").count().orderBy("k").toPandas()
    out["group_counts"] = g["count"].tolist()
    a = df.groupBy("cat").agg(F.avg("label").alias("m")).orderBy("cat").toPandas()
    out["cat_means"] = a.m.round(9).tolist()
    out["distinct_k"] = df.select("k").dropDuplicates().count()
    small = spark.createDataFrame(pd.DataFrame({"k": [0, 1, 2], "name": ["zero", "one", "two"]}))
    out["join"] = df.join(small, on="k").count()
    top = df.orderBy(F.col("label").desc()).limit(3).toPandas()
    out["top"] = top.label.round(9).tolist()
    out["mean_x0"] = round(float(df.describe().toPandas().set_index("summary").loc["mean", "x0"]), 9)
    out["repart"] = df.repartition(5).count()
    return out


def scenario_ml(spark):
    from cdnaml.ml import Pipeline
    from cdnaml.ml.clustering import KMeans
    from cdnaml.ml.evaluation import RegressionEvaluator
    from cdnaml.ml.feature import StringIndexer, VectorAssembler
    from cdnaml.ml.regression import LinearRegression, RandomForestRegressor
    df = _data(spark)
    si = StringIndexer(inputCol="cat", outputCol="ci")
    va = VectorAssembler(inputCols=["x0", "x1", "x2", "x3", "ci"], outputCol="features")
    lr = Pipeline(stages=[si, va, LinearRegression()]).fit(df)
    out = {"lr_coef": np.round(lr.stages[-1].coefficients.toArray(), 8).tolist(),
           "si_labels": list(lr.stages[0].labels)}
    rf = Pipeline(stages=[si, va, RandomForestRegressor(numTrees=5, maxDepth=4, seed=7)]).fit(df)
    pred = rf.transform(df)
    out["rf_rmse"] = round(RegressionEvaluator().evaluate(pred), 6)
    out["rf_nodes"] = int(rf.stages[-1].totalNumNodes)
    out["rf_importances"] = np.round(rf.stages[-1].featureImportances.toArray(), 6).tolist()
    km = KMeans(k=3, seed=1, maxIter=10).fit(va.transform(si.fit(df).transform(df)))
    out["km_cost"] = round(km.summary.trainingCost, 3)
    return out


def scenario_fault(spark):
    """CDNAML_FAULT=1:all_reduce:2 -> rank 1 fails its 2nd all-reduce; every rank must see a
    CommError naming a rank and the collective instead of hanging (watchdog CDNAML_COMM_TIMEOUT)."""
    import time
    from cdnaml.models.regression import LinearRegression
    from cdnaml.models.feature import VectorAssembler
    from cdnaml.parallel.comm import CommError
    df = VectorAssembler(inputCols=["x0", "x1", "x2", "x3"], outputCol="features").transform(_data(spark))
    t0 = time.time()
    try:
        for _ in range(3):
            LinearRegression().fit(df)
        return {"rank": spark.comm.rank, "error": None}
    except CommError as e:
        return {"rank": spark.comm.rank, "error": str(e), "err_rank": e.rank, "op": e.op,
                "seconds": time.time() - t0}


SCENARIOS = {"frame": scenario_frame, "ml": scenario_ml, "fault": scenario_fault}


def run(name):
    spark = _session()
    return SCENARIOS[name](spark)


if __name__ == "__main__":
    res = run(sys.argv[1])
    rank = int(os.environ.get("RANK", "0"))
    if sys.argv[1] == "fault":  # every rank reports (its own failure mode)
        with open(f"{sys.argv[2]}.rank{rank}", "w") as f:
            json.dump(res, f)
    elif rank == 0:
        with open(sys.argv[2], "w") as f:
            json.dump(res, f)
