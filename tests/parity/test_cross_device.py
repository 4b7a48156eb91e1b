"""Cross-device parity of the notebook flows: every flow below runs on the host (cpu) and on
the GPU (cuda) in one test, with the GPU's native-kernel size thresholds set to 0 (HASH_MIN_ROWS, GATHER_MIN,
FUSE_MIN_ROWS) so the course-sized frames go through the HIP kernels, and the outputs are compared:

* row counts, dedup results, group counts, SQL results, bests maps: exactly;
* tree models (int64 fixed-point histograms on both devices): forest digests exactly, predictions bit for bit
  (fp64 leaves and sums in one tree order), avgMetrics / RMSE / AUC to 1e-12 (only the fp64 metric reductions'
  order differs);
* logistic regression (fp64 margins on both devices): the objective to 1e-7, coefficients to 1e-4, the MLE 03
  regParam x elasticNet CV to the same best map;
* models fitted through floating-point reductions whose order differs between the devices (the K1 Gram's fp32
  MFMA partial slabs, L-BFGS on fp64 device vectors, K-means sums): to the tolerance stated per flow.

Each flow also records which native kernels the cuda run called (``_lib.check`` sees every launch by name), and
the test asserts the data flows reach the K16 hash / K18 fused-expression / K19 gather kernels.
Reference flows: S/Labs/ML 00L - Dedup Lab.py:79-147, ML 01 - Data Cleansing.py:135-169, S/Labs/ML 01L,
ML 02 / ML 03 Linear Regression, ML 06 Decision Trees, ML 07 / S/Labs/ML 07L, ML Electives/MLE 01:241-374 (SQL),
MLE 02 K-Means, S/ML Electives/MLE 03 Logistic Regression."""
import collections
import os

import numpy as np
import pytest

from tests.conftest import session_device

pytestmark = pytest.mark.gpu


def _sf(ds, name):
    return os.path.join(ds, "airbnb", "sf-listings", name)


def _airbnb(spark, ds):
    return spark.read.format("delta").load(_sf(ds, "sf-listings-2019-03-06-clean.delta"))


# ------------------------------------------------------------------------------------------------------ flows
def flow_dedup(spark, ds, work):
    from pyspark.sql.functions import col, lower, translate
    from cdnaml.utils import datasets as D
    src = os.path.join(work, "people-with-dups.txt")
    os.makedirs(work, exist_ok=True)
    D.people_with_dups(n_unique=100000, n_dups=3000).to_csv(src, sep=":", index=False)
    spark.conf.set("spark.sql.shuffle.partitions", 8)
    df = spark.read.csv(src, header=True, sep=":", inferSchema=True)
    dedup = (df.select(col("*"), lower(col("firstName")).alias("lcFirstName"),
                       lower(col("lastName")).alias("lcLastName"), lower(col("middleName")).alias("lcMiddleName"),
                       translate(col("ssn"), "-", "").alias("ssnNums"))
             .dropDuplicates(["lcFirstName", "lcMiddleName", "lcLastName", "ssnNums", "gender", "birthDate",
                              "salary"])
             .drop("lcFirstName", "lcMiddleName", "lcLastName", "ssnNums"))
    dest = os.path.join(work, "people.parquet")
    dedup.write.mode("overwrite").parquet(dest)
    back = spark.read.parquet(dest).toPandas()
    rows = sorted(map(tuple, back.astype(str).values.tolist()))
    return {"count": df.count(), "dedup": len(back), "parts": len([f for f in os.listdir(dest)
                                                                   if f.endswith(".parquet")]),
            "rows_hash": hash(tuple(rows))}


def flow_cleansing(spark, ds, work):
    from pyspark.sql.functions import col, translate, when
    from pyspark.ml.feature import Imputer
    raw = spark.read.csv(_sf(ds, "sf-listings-2019-03-06.csv"), header="true", inferSchema="true",
                         multiLine="true", escape='"')
    base = raw.select("host_is_superhost", "neighbourhood_cleansed", "room_type", "accommodates", "bedrooms",
                      "beds", "minimum_nights", "review_scores_rating", "price")
    fixed = base.withColumn("price", translate(col("price"), "$,", "").cast("double"))
    summ = fixed.select("price", "bedrooms", "beds").summary().toPandas().set_index("summary")
    pos = fixed.filter(col("price") > 0)
    counts = pos.groupBy("room_type").count().orderBy(col("count").desc(), col("room_type")).toPandas()
    hood = pos.groupBy("neighbourhood_cleansed").count().orderBy("neighbourhood_cleansed").toPandas()
    nums = [c for c, t in pos.dtypes if t in ("int", "bigint", "double") and c != "price"]
    for c in nums:
        pos = pos.withColumn(c, col(c).cast("double"))
    for c in nums:
        pos = pos.withColumn(c + "_na", when(col(c).isNull(), 1.0).otherwise(0.0))
    imp = Imputer(strategy="median", inputCols=nums, outputCols=nums).fit(pos)
    out = imp.transform(pos)
    def num(v):  # summary() cells are strings; compare their values (fp64 reduction order differs by device)
        try:
            return float(v)
        except (TypeError, ValueError):
            return str(v)
    return {"summary": {k: [num(v) for v in summ.loc[k].tolist()] for k in summ.index},
            "room_counts": list(zip(counts.room_type, counts["count"].astype(int))),
            "hood_counts": list(zip(hood.neighbourhood_cleansed, hood["count"].astype(int))),
            "medians": {c: float(v) for c, v in zip(nums, imp.surrogateDF.toPandas().iloc[0].tolist())},
            "na_sums": [float(out.agg({c + "_na": "sum"}).first()[0]) for c in nums],
            "n": out.count()}


def flow_exploration(spark, ds, work):
    from pyspark.sql.functions import avg, col, lit, log
    from pyspark.ml.evaluation import RegressionEvaluator
    df = _airbnb(spark, ds)
    lp = df.select(log("price").alias("log_price")).toPandas().log_price.values
    top = df.groupBy("neighbourhood_cleansed").count().orderBy(col("count").desc(), "neighbourhood_cleansed") \
        .limit(5).toPandas()
    train, test = df.randomSplit([0.8, 0.2], seed=42)
    mean_price = train.select(avg("price")).first()[0]
    median_price = train.approxQuantile("price", [0.5], 0.0)[0]
    ev = RegressionEvaluator(predictionCol="pred", labelCol="price", metricName="rmse")
    return {"n_train": train.count(), "n_test": test.count(), "mean": mean_price, "median": median_price,
            "log_sum": float(np.sum(lp)),
            "top": list(zip(top.neighbourhood_cleansed, top["count"].astype(int))),
            "rmse_mean": ev.evaluate(test.withColumn("pred", lit(mean_price))),
            "rmse_median": ev.evaluate(test.withColumn("pred", lit(median_price)))}


def flow_sql(spark, ds, work):
    ratings = spark.read.parquet(os.path.join(ds, "movielens", "ratings.parquet"))
    movies = spark.read.parquet(os.path.join(ds, "movielens", "movies.parquet"))
    ratings.createOrReplaceTempView("ratings")
    movies.createOrReplaceTempView("movies")
    q = spark.sql("SELECT m.title, COUNT(*) AS n, AVG(r.rating) AS avg_rating FROM ratings r "
                  "JOIN movies m ON (r.movieId = m.ID) GROUP BY m.title HAVING COUNT(*) > 20 "
                  "ORDER BY avg_rating DESC, m.title LIMIT 100").toPandas()
    d = ratings.select("userId").dropDuplicates().count()
    return {"rows": len(q), "titles": q.title.tolist(), "n": q.n.astype(int).tolist(),
            "avg": q.avg_rating.tolist(), "users": d, "ratings": ratings.count()}


def _split_cols(train, label="price"):
    cats = [c for c, t in train.dtypes if t == "string"]
    nums = [c for c, t in train.dtypes if t == "double" and c not in (label, "price")]
    return cats, [c + "Index" for c in cats], nums


def flow_lr(spark, ds, work):
    from pyspark.ml import Pipeline
    from pyspark.ml.feature import OneHotEncoder, StringIndexer, VectorAssembler
    from pyspark.ml.regression import LinearRegression
    from pyspark.ml.evaluation import RegressionEvaluator
    train, test = _airbnb(spark, ds).randomSplit([0.8, 0.2], seed=42)
    cats, idx, nums = _split_cols(train)
    ohe = [c + "OHE" for c in cats]
    model = Pipeline(stages=[StringIndexer(inputCols=cats, outputCols=idx, handleInvalid="skip"),
                             OneHotEncoder(inputCols=idx, outputCols=ohe),
                             VectorAssembler(inputCols=ohe + nums, outputCol="features"),
                             LinearRegression(labelCol="price", featuresCol="features")]).fit(train)
    ev = RegressionEvaluator(labelCol="price")
    pred = model.transform(test)
    lr = model.stages[-1]
    return {"coef": lr.coefficients.toArray().tolist(), "intercept": lr.intercept,
            "rmse": ev.evaluate(pred), "n_pred": pred.count()}


def flow_dt(spark, ds, work):
    from pyspark.ml import Pipeline
    from pyspark.ml.feature import StringIndexer, VectorAssembler
    from pyspark.ml.regression import DecisionTreeRegressor
    from pyspark.ml.evaluation import RegressionEvaluator
    from cdnaml.utils.synthetic import forest_digest
    train, test = _airbnb(spark, ds).randomSplit([0.8, 0.2], seed=42)
    cats, idx, nums = _split_cols(train)
    model = Pipeline(stages=[StringIndexer(inputCols=cats, outputCols=idx, handleInvalid="skip"),
                             VectorAssembler(inputCols=idx + nums, outputCol="features"),
                             DecisionTreeRegressor(labelCol="price", maxBins=40)]).fit(train)
    return {"digest": forest_digest(model.stages[-1]._forest),
            "importances": model.stages[-1].featureImportances.toArray().tolist(),
            "rmse": RegressionEvaluator(labelCol="price").evaluate(model.transform(test))}


def flow_rf_cv(spark, ds, work):
    from pyspark.ml import Pipeline
    from pyspark.ml.feature import StringIndexer, VectorAssembler
    from pyspark.ml.regression import RandomForestRegressor
    from pyspark.ml.tuning import CrossValidator, ParamGridBuilder
    from pyspark.ml.evaluation import RegressionEvaluator
    from cdnaml.utils.synthetic import forest_digest
    train, test = _airbnb(spark, ds).randomSplit([0.8, 0.2], seed=42)
    cats, idx, nums = _split_cols(train)
    rf = RandomForestRegressor(labelCol="price", maxBins=40, seed=42)
    grid = ParamGridBuilder().addGrid(rf.maxDepth, [2, 5]).addGrid(rf.numTrees, [5, 10]).build()
    ev = RegressionEvaluator(labelCol="price", predictionCol="prediction")
    cv = CrossValidator(estimator=rf, evaluator=ev, estimatorParamMaps=grid, numFolds=3, seed=42, parallelism=4)
    model = Pipeline(stages=[StringIndexer(inputCols=cats, outputCols=idx, handleInvalid="skip"),
                             VectorAssembler(inputCols=idx + nums, outputCol="features"), cv]).fit(train)
    cvm = model.stages[-1]
    return {"avg": list(cvm.avgMetrics), "best": int(np.argmin(cvm.avgMetrics)),
            "digest": forest_digest(cvm.bestModel._forest), "rmse": ev.evaluate(model.transform(test))}


def flow_rf_cls(spark, ds, work):
    """S/Labs/ML 07L:42-209 -- priceClass, RandomForestClassifier grid maxDepth {2, 5, 10} x numTrees {10, 20, 100},
    3-fold CV on areaUnderROC."""
    from pyspark.sql.functions import col, when
    from pyspark.ml import Pipeline
    from pyspark.ml.classification import RandomForestClassifier
    from pyspark.ml.feature import StringIndexer, VectorAssembler
    from pyspark.ml.tuning import CrossValidator, ParamGridBuilder
    from pyspark.ml.evaluation import BinaryClassificationEvaluator
    from cdnaml.utils.synthetic import forest_digest
    df = _airbnb(spark, ds).withColumn("priceClass", when(col("price") >= 150, 1).otherwise(0))
    train, test = df.randomSplit([0.8, 0.2], seed=42)
    cats, idx, nums = _split_cols(train, "priceClass")
    rf = RandomForestClassifier(labelCol="priceClass", maxBins=40, seed=42)
    grid = ParamGridBuilder().addGrid(rf.maxDepth, [2, 5, 10]).addGrid(rf.numTrees, [10, 20, 100]).build()
    ev = BinaryClassificationEvaluator(labelCol="priceClass")
    cv = CrossValidator(estimator=rf, evaluator=ev, estimatorParamMaps=grid, numFolds=3, seed=42)
    model = Pipeline(stages=[StringIndexer(inputCols=cats, outputCols=idx, handleInvalid="skip"),
                             VectorAssembler(inputCols=idx + nums, outputCol="features"), cv]).fit(train)
    cvm = model.stages[-1]
    return {"avg": list(cvm.avgMetrics), "best": int(np.argmax(cvm.avgMetrics)),
            "digest": forest_digest(cvm.bestModel._forest), "auc": ev.evaluate(model.transform(test))}


def flow_kmeans(spark, ds, work):
    from pyspark.ml.clustering import KMeans
    from pyspark.ml.feature import VectorAssembler
    rng = np.random.default_rng(0)
    pts = np.concatenate([rng.normal(c, 0.3, (2000, 2)) for c in ((0, 0), (4, 4), (0, 5))])
    df = spark.createDataFrame([(float(a), float(b)) for a, b in pts], ["x", "y"])
    data = VectorAssembler(inputCols=["x", "y"], outputCol="features").transform(df)
    m = KMeans(k=3, seed=221, maxIter=20).fit(data)
    c0 = np.array(KMeans(k=3, seed=221, maxIter=0).fit(data).clusterCenters())
    lab = m.transform(data).groupBy("prediction").count().orderBy("prediction").toPandas()
    return {"centers": np.array(m.clusterCenters()).tolist(), "init": c0.tolist(),
            "sizes": lab["count"].astype(int).tolist()}


def flow_logistic(spark, ds, work):
    from pyspark.sql.functions import col, when
    from pyspark.ml import Pipeline
    from pyspark.ml.classification import LogisticRegression
    from pyspark.ml.feature import RFormula
    from pyspark.ml.evaluation import BinaryClassificationEvaluator, MulticlassClassificationEvaluator
    data = _airbnb(spark, ds).withColumn("priceClass", when(col("price") >= 150, 1.0).otherwise(0.0))
    train, test = data.randomSplit([0.8, 0.2], seed=42)
    model = Pipeline(stages=[RFormula(formula="priceClass ~ . - price", handleInvalid="skip"),
                             LogisticRegression(labelCol="priceClass", regParam=0.1)]).fit(train)
    pred = model.transform(test)
    lrm = model.stages[-1]
    # fp64 margins and gradients on both devices (K11): the same L-BFGS path up to summation order
    return {"loss": float(lrm.summary.objectiveHistory[-1]), "coef": list(lrm.coefficients.toArray()),
            "intercept": float(lrm.intercept), "iters": int(lrm.summary.totalIterations),
            "acc": MulticlassClassificationEvaluator(labelCol="priceClass", metricName="accuracy").evaluate(pred),
            "auc": BinaryClassificationEvaluator(labelCol="priceClass").evaluate(pred)}


def flow_logistic_cv(spark, ds, work):
    """MLE 03's regParam x elasticNetParam grid in a 3-fold CrossValidator on AUC (S/ML Electives/MLE 03 -
    Logistic Regression Lab.py:143-158): both devices must pick the same map with the same fold metrics."""
    from pyspark.sql.functions import col, when
    from pyspark.ml import Pipeline
    from pyspark.ml.classification import LogisticRegression
    from pyspark.ml.feature import RFormula
    from pyspark.ml.evaluation import BinaryClassificationEvaluator
    from pyspark.ml.tuning import CrossValidator, ParamGridBuilder
    data = _airbnb(spark, ds).withColumn("priceClass", when(col("price") >= 150, 1.0).otherwise(0.0))
    train, _ = data.randomSplit([0.8, 0.2], seed=42)
    lr = LogisticRegression(labelCol="priceClass")
    grid = ParamGridBuilder().addGrid(lr.regParam, [0.1, 0.2]).addGrid(lr.elasticNetParam, [0.0, 0.5, 1.0]).build()
    cv = CrossValidator(estimator=lr, evaluator=BinaryClassificationEvaluator(labelCol="priceClass"),
                        estimatorParamMaps=grid, numFolds=3, seed=42)
    model = Pipeline(stages=[RFormula(formula="priceClass ~ . - price", handleInvalid="skip"), cv]).fit(train)
    cvm = model.stages[-1]
    return {"avg": list(cvm.avgMetrics), "best": int(np.argmax(cvm.avgMetrics))}


FLOWS = {"dedup": flow_dedup, "cleansing": flow_cleansing, "exploration": flow_exploration, "sql": flow_sql,
         "lr": flow_lr, "dt": flow_dt, "rf_cv": flow_rf_cv, "rf_cls": flow_rf_cls, "kmeans": flow_kmeans,
         "logistic": flow_logistic, "logistic_cv": flow_logistic_cv}

# native kernels each data flow must reach on the GPU (any one of each tuple)
HASH = ("cdna_hp_part", "cdna_hp_agg", "cdna_hp_hist", "cdna_la_groups", "cdna_hash_insert", "cdna_pack_keys",
        "cdna_bucket_compact", "cdna_grouped_reduce")
NATIVE = {"dedup": [HASH],
          "cleansing": [HASH, ("cdna_expr_eval",), ("cdna_col_moments",), ("cdna_gather", "cdna_compact_mask")],
          "exploration": [HASH, ("cdna_reg_metrics",)],
          "sql": [("cdna_join_build", "cdna_join_build_dense"), ("cdna_join_probe", "cdna_join_probe_dense"), HASH],
          "lr": [("cdna_reg_metrics",)], "dt": [("cdna_binize",), ("cdna_split_scan", "cdna_split_scan_ex")],
          "rf_cv": [("cdna_binize",), ("cdna_tree_predict_heap", "cdna_tree_predict")],
          "rf_cls": [("cdna_binize",), ("cdna_split_scan_ex",), ("cdna_score_hist", "cdna_tree_predict")],
          "kmeans": [("cdna_kmeans_step",)], "logistic": [("cdna_logistic_grad",)],
          "logistic_cv": [("cdna_logistic_grad",)]}


def _run_all(device, root, monkeypatch=None):
    import cdnaml
    import cdnaml.compat as compat
    from cdnaml.ops import _lib
    from cdnaml.utils import datasets as D
    out, calls = {}, collections.defaultdict(collections.Counter)
    with session_device(device):
        os.environ["CDNAML_DBFS_ROOT"] = str(root / f"dbfs_{device}")
        os.environ["CDNAML_TRACKING_URI"] = str(root / f"mlruns_{device}")
        spark = cdnaml.SparkSession.builder.config("cdnaml.warehouse.dir", str(root / f"wh_{device}")).getOrCreate()
        compat.install()
        ds = D.install_datasets(str(root / "datasets"), spark, scale=0.3)
        orig = _lib.check
        current = {"flow": None}

        def counting(code, name):
            if current["flow"] is not None:
                calls[current["flow"]][name.split("(")[0]] += 1
            return orig(code, name)
        _lib.check = counting
        try:
            for name, fn in FLOWS.items():
                current["flow"] = name
                out[name] = fn(spark, ds, str(root / f"work_{device}_{name}"))
        finally:
            _lib.check = orig
            compat.uninstall()
            spark.stop()
    return out, calls


@pytest.fixture(scope="module")
def results(tmp_path_factory):
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from cdnaml.ops import kernels as K, relops as R
    from cdnaml.sql import fused
    root = tmp_path_factory.mktemp("xdev")
    cpu, _ = _run_all("cpu", root)
    saved = (R.HASH_MIN_ROWS, R.GATHER_MIN, fused.FUSE_MIN_ROWS)
    R.HASH_MIN_ROWS, R.GATHER_MIN, fused.FUSE_MIN_ROWS = 0, 0, 0
    try:
        gpu, calls = _run_all("cuda", root)
    finally:
        R.HASH_MIN_ROWS, R.GATHER_MIN, fused.FUSE_MIN_ROWS = saved
    out = os.environ.get("CDNAML_PARITY_CALLS")
    if out:  # e.g. gpurun_out/parity_calls.json: which native kernels each flow reached on the GPU
        import json
        with open(out, "w") as f:
            json.dump({k: dict(v) for k, v in calls.items()}, f, indent=1, sort_keys=True)
    return cpu, gpu, calls


def _close(a, b, rel, path=""):
    if isinstance(a, dict):
        assert a.keys() == b.keys(), path
        for k in a:
            _close(a[k], b[k], rel, f"{path}.{k}")
    elif isinstance(a, (list, tuple)):
        assert len(a) == len(b), path
        for i, (x, y) in enumerate(zip(a, b)):
            _close(x, y, rel, f"{path}[{i}]")
    elif isinstance(a, float) and not isinstance(a, bool):
        assert b == pytest.approx(a, rel=rel, abs=rel), (path, a, b)
    else:
        assert a == b, (path, a, b)


EXACT = ("dedup", "sql")
# int64 histograms on both devices: identical models (digests compared exactly); their predictions / probabilities
# are fp64 sums over trees in ONE fixed order on both devices (K.ordered_tree_sum), bit-identical; the metrics
# over them are fp64 reductions (the device's in another summation order: RMSE to ~1e-16, AUC from exact counts)
TREES = ("dt", "rf_cv", "rf_cls")
TREE_METRIC_TOL = 1e-12
# fp64 reductions in a different order: 1e-9 (LR: course-sized normal equations take the fp64 Gram on both
# devices -- gramPrecision auto; the K1 fp32 MFMA Gram had moved these ill-conditioned OHE coefficients by
# 2e-3 relative).  Logistic regression: L-BFGS / OWL-QN stops at the same loss tolerance
# from fp32 device gradients vs fp64 host ones: the fitted objectives and the accuracy / AUC compared
TOL = {"cleansing": 1e-9, "exploration": 1e-9, "lr": 1e-8, "kmeans": 1e-6, "logistic": 1e-7, "logistic_cv": 1e-7}


@pytest.mark.parametrize("flow", list(FLOWS))
def test_flow_matches_across_devices(results, flow):
    cpu, gpu, calls = results
    a, b = cpu[flow], gpu[flow]
    if flow in EXACT:
        assert a == b
    elif flow in TREES:
        assert a["digest"] == b["digest"]
        _close(a, b, TREE_METRIC_TOL)
    elif flow == "lr":
        # fp64 normal equations on both devices: coefficients to 1e-8; the RMSE of fp32 device predictions to 1e-5
        _close({k: a[k] for k in ("coef", "intercept", "n_pred")}, {k: b[k] for k in ("coef", "intercept", "n_pred")},
               TOL["lr"])
        _close(a["rmse"], b["rmse"], 1e-5)
    elif flow == "logistic":
        # fp64 margins on both devices (K11): the fitted objective to 1e-7, the coefficients to 1e-4
        _close(a["loss"], b["loss"], TOL["logistic"])
        _close({k: a[k] for k in ("coef", "intercept")}, {k: b[k] for k in ("coef", "intercept")}, 1e-4)
        _close({k: a[k] for k in ("acc", "auc")}, {k: b[k] for k in ("acc", "auc")}, 1e-9)
    else:
        _close(a, b, TOL[flow])
    for group in NATIVE.get(flow, []):
        assert any(calls[flow][k] for k in group), (flow, group, dict(calls[flow]))
