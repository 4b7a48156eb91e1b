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


def _tree_df(spark, n=4000, d=12, seed=3, uneven=None):
    """Partition-invariant regression/classification table (features keyed by global row id)."""
    rng = np.random.default_rng(seed)
    X = rng.normal(size=(n, d))
    y = X[:, 0] * 2.0 - X[:, 1] + np.sin(2 * X[:, 2]) + 0.1 * rng.normal(size=n)
    pdf = pd.DataFrame({"idx": np.arange(n), "label": y, "cls": (y > 0).astype(float),
                        "cls3": (y > -0.5).astype(float) + (y > 0.8).astype(float)})
    from cdnaml.ml.feature import VectorAssembler
    for i in range(d):
        pdf[f"x{i}"] = X[:, i]
    df = spark.createDataFrame(pdf)
    if uneven is not None:
        # keep a prefix of the global rows: rank shards become empty / imbalanced (filter keeps placement)
        from cdnaml.sql import functions as F
        df = df.filter(F.col("idx") < int(n * uneven))
    return VectorAssembler(inputCols=[f"x{i}" for i in range(d)], outputCol="features").transform(df)


def _tree_digests(df):
    from cdnaml.ml.classification import RandomForestClassifier
    from cdnaml.ml.regression import DecisionTreeRegressor, GBTRegressor, RandomForestRegressor
    from cdnaml.ml.xgboost import XgboostClassifier, XgboostRegressor
    from cdnaml.utils.synthetic import forest_digest
    out = {}
    fits = {
        "rf20": RandomForestRegressor(numTrees=20, maxDepth=5, maxBins=40, seed=42),
        "dt": DecisionTreeRegressor(maxDepth=6, maxBins=32),
        "gbt": GBTRegressor(maxIter=5, maxDepth=4, seed=1),
        "xgb_reg": XgboostRegressor(n_estimators=5, max_depth=4, learning_rate=0.3, random_state=42, missing=0.0),
        "xgb_cls": XgboostClassifier(n_estimators=4, max_depth=3, random_state=7, labelCol="cls"),
        "rf_cls": RandomForestClassifier(numTrees=5, maxDepth=4, seed=11, labelCol="cls"),
        # three classes on the packed record path (sums W1 + 2^32 W2 all-reduced as int64)
        "rf_cls3": RandomForestClassifier(numTrees=4, maxDepth=4, seed=13, labelCol="cls3"),
    }
    for k, est in fits.items():
        m = est.fit(df)
        out[k] = forest_digest(m._forest)
        out[k + "_nodes"] = int(sum(len(m._forest.tree_nodes(t)) for t in range(len(m._forest.roots))))
    return out


def scenario_trees(spark):
    """Every tree learner's fitted model is bit-identical at any world size (int64 fixed-point histograms
    all-reduced exactly, scales agreed over ranks, data keyed by global row id)."""
    return _tree_digests(_tree_df(spark))


def scenario_trees_uneven(spark):
    """Same with imbalanced shards: the first 30 % of the global rows only (at W >= 4 some ranks are
    empty): every rank must still issue the same collectives and reach the 1-rank model."""
    return _tree_digests(_tree_df(spark, uneven=0.3))


def scenario_trees_rs(spark):
    """Every level histogram reduce-scattered by feature (RS_MIN_BYTES = 0; RF without the chunked all-reduce
    overlap, so its feature-subset masks are sliced too): 13 features give uneven slices and, at W = 8, ranks
    without features.  The forests must equal the 1-rank (all-reduce-free) fits bit for bit."""
    from cdnaml.models.tree import engine
    engine.RS_MIN_BYTES = 0
    engine.HIST_OVERLAP = 1
    seen = {"rs": 0}
    orig = engine.ForestTrainer._reduce_scatter_features

    def counted(self, Hb, d):
        seen["rs"] += 1
        return orig(self, Hb, d)
    engine.ForestTrainer._reduce_scatter_features = counted
    out = _tree_digests(_tree_df(spark, d=13))
    out["rs_levels"] = seen["rs"]
    return out


def scenario_trees_rs_overlap(spark):
    """Reduce-scatter by feature COMPOSED with the chunked (overlapped) histograms: (a) overlap
    with all-reduce for the shallow levels, reduce-scatter from level 2 on; (b) every level from 0 reduce-scatters
    and the levels past the overlap threshold reduce-scatter chunk by chunk (async, while the next chunk builds,
    the parents cut to the rank's feature slice); (c) every level overlapped + reduce-scattered, with the RF
    headline shape scaled down and a depth-8 / 256-bin GBDT.  All must give the 1-rank forests bit for bit."""
    from cdnaml.models.tree import engine
    seen = {"rs": 0, "ov": 0, "ov_rs": 0}
    o_rs, o_ov = engine.ForestTrainer._reduce_scatter_features, engine.ForestTrainer._hist_overlapped

    def rs(self, *a):
        seen["rs"] += 1
        return o_rs(self, *a)

    def ov(self, *a, **k):
        seen["ov"] += 1
        seen["ov_rs"] += int(bool(k.get("rs")))
        return o_ov(self, *a, **k)
    engine.ForestTrainer._reduce_scatter_features = rs
    engine.ForestTrainer._hist_overlapped = ov
    engine.HIST_OVERLAP = 2
    df = _tree_df(spark, d=13)
    out = {}
    for tag, rs_min, ov_min in (("a", 200000, 100000), ("b", 0, 300000)):
        engine.RS_MIN_BYTES, engine.HIST_OVERLAP_MIN_BYTES = rs_min, ov_min
        seen.update(rs=0, ov=0, ov_rs=0)
        for k, v in _tree_digests(df).items():
            out[f"{tag}_{k}"] = v
        out[f"{tag}_levels"] = dict(seen)
    from cdnaml.ml.regression import RandomForestRegressor
    from cdnaml.ml.xgboost import XgboostRegressor
    from cdnaml.utils.synthetic import forest_digest
    engine.RS_MIN_BYTES, engine.HIST_OVERLAP_MIN_BYTES, engine.HIST_OVERLAP = 0, 0, 4
    seen.update(rs=0, ov=0, ov_rs=0)
    big = _tree_df(spark, n=6000, d=24, seed=5)
    for k, est in (("rf", RandomForestRegressor(numTrees=20, maxDepth=5, maxBins=40, seed=42)),
                   ("gbdt8", XgboostRegressor(n_estimators=3, max_depth=8, max_bin=256, learning_rate=0.3,
                                              random_state=1))):
        m = est.fit(big)
        out[f"c_{k}"] = forest_digest(m._forest)
    out["c_levels"] = dict(seen)
    return out


def scenario_trace_rs_overlap(spark):
    """A traced fit with every multi-slot level overlapped + reduce-scattered: count the tree.reduce_scatter
    spans that are in flight when a later tree.hist_chunk span starts (Chrome trace written next to the result)."""
    from cdnaml.ml.regression import RandomForestRegressor
    from cdnaml.models.tree import engine
    from cdnaml.utils import tracing
    engine.RS_MIN_BYTES, engine.HIST_OVERLAP_MIN_BYTES, engine.HIST_OVERLAP = 0, 0, 4
    df = _tree_df(spark, n=20000, d=24, seed=5)
    RandomForestRegressor(numTrees=8, maxDepth=5, maxBins=40, seed=42).fit(df)   # warm-up
    tracing.reset()
    tracing.enable()
    RandomForestRegressor(numTrees=8, maxDepth=5, maxBins=40, seed=42).fit(df)
    tracing.disable()
    path = os.path.abspath(f"rs_overlap_trace.rank{spark.comm.rank}.json")
    tracing.export_chrome_trace(path)
    with open(path) as f:
        evs = json.load(f)["traceEvents"]
    rs = [e for e in evs if e["name"] == "tree.reduce_scatter"]
    ch = [e for e in evs if e["name"] == "tree.hist_chunk"]
    overl = sum(1 for a in rs for c in ch if a["ts"] < c["ts"] < a["ts"] + a["dur"])
    return {"rs_spans": len(rs), "chunk_spans": len(ch), "overlapping": overl, "trace": path}


def scenario_trees_rs_nccl(spark):
    """the RCCL branches of Comm (reduce_scatter_tensor, all_gather_into_tensor, device
    barriers) driven through tests/fake_nccl.py's recording nccl-over-gloo proxy (installed before the session's
    Comm is built, see run()): direct collective checks, then the trees_rs forests (every level histogram
    reduce-scattered by feature, winners all-gathered) -- which must equal the 1-rank fits bit for bit."""
    import torch
    import fake_nccl
    comm = spark.comm
    W, r = comm.world_size, comm.rank
    out = {"backend": comm.backend}
    # reduce-scatter: [W, 3, 5] int64 -> this rank's [3, 5] slice of the sum, on the caller's device
    t = (torch.arange(W * 15, dtype=torch.int64).reshape(W, 3, 5) + 100 * r)
    got = comm.reduce_scatter(t)
    want = (torch.arange(W * 15, dtype=torch.int64).reshape(W, 3, 5) * W + 100 * sum(range(W)))[r]
    out["rs_ok"] = bool(got.shape == (3, 5) and got.device == t.device and torch.equal(got, want))
    # non-contiguous input is made contiguous before RCCL sees it
    tt = torch.arange(W * 10, dtype=torch.float64).reshape(10, W).T
    out["rs_noncontig_ok"] = bool(torch.equal(comm.reduce_scatter(tt), tt[r] * W))
    g = comm.all_gather_tensor(torch.full((2, 3), float(r)))
    out["ag_ok"] = bool(g.shape == (W, 2, 3) and all(bool((g[k] == k).all()) for k in range(W)))
    a = torch.ones(7, dtype=torch.float64) * (r + 1)
    out["ar_async_ok"] = bool(torch.equal(comm.all_reduce_async(a).wait(), torch.full((7,), W * (W + 1) / 2.0,
                                                                                   dtype=torch.float64)))
    chunks = [torch.full((j + 1, 2), float(r * 10 + j)) for j in range(W)]
    recv = comm.all_to_all_v(chunks)
    out["a2a_ok"] = bool(all(x.shape == (r + 1, 2) and bool((x == k * 10 + r).all()) for k, x in enumerate(recv)))
    # the async reduce-scatter (the overlapped chunks of reduce-scatter levels)
    hs = [comm.reduce_scatter_async(t * (j + 1)) for j in range(3)]
    out["rs_async_ok"] = bool(all(torch.equal(h.wait(), want * (j + 1)) for j, h in enumerate(hs)))
    comm.barrier()
    res = scenario_trees_rs(spark)
    out.update(res)
    from cdnaml.models.tree import engine
    engine.HIST_OVERLAP, engine.HIST_OVERLAP_MIN_BYTES = 3, 0
    ov = _tree_digests(_tree_df(spark, d=13))
    out["overlap_same"] = bool(all(ov[k] == res[k] for k in ov))
    rec = comm.all_gather_object(dict(fake_nccl.RECORD))
    out["record_min"] = {k: min(x.get(k, 0) for x in rec) for k in rec[0]}
    out["violations"] = sorted(set(sum(comm.all_gather_object(list(fake_nccl.VIOLATIONS)), [])))
    return out


def scenario_trees_deep(spark):
    """Forests deeper than 8 levels (binary classification and regression forests switch from the u16 row codes
    to node ids at level 8, then build node-id record histograms): bit-identical at any world size, also with
    every level reduce-scattered by feature."""
    from cdnaml.ml.classification import RandomForestClassifier
    from cdnaml.ml.regression import RandomForestRegressor
    from cdnaml.models.tree import engine
    from cdnaml.utils.synthetic import forest_digest
    df = _tree_df(spark, n=12000, d=13)
    calls = {"n": 0}
    orig = engine.K.node_compact

    def counted(*a, **k):
        calls["n"] += 1
        return orig(*a, **k)
    engine.K.node_compact = counted
    out = {}
    for tag, rs_min in (("ar", 1 << 62), ("rs", 0)):
        engine.RS_MIN_BYTES = rs_min
        engine.HIST_OVERLAP = 1
        for k, est in (("rf_reg", RandomForestRegressor(numTrees=3, maxDepth=11, maxBins=32, seed=5)),
                       ("rf_cls", RandomForestClassifier(numTrees=3, maxDepth=10, maxBins=32, seed=9,
                                                         labelCol="cls"))):
            m = est.fit(df)
            out[f"{tag}_{k}"] = forest_digest(m._forest)
            out[f"{tag}_{k}_nodes"] = int(sum(len(m._forest.tree_nodes(t)) for t in range(len(m._forest.roots))))
    assert calls["n"] > 0, "the node-id record levels did not run"
    return out


def scenario_ooc_uneven(spark):
    """Out-of-core (streamed) fits with the last rank's shard EMPTY: every rank must take the same
    streamed path (the choice is agreed over ranks) and the forests must equal the 1-rank streamed fit."""
    import torch
    from cdnaml.ml.regression import RandomForestRegressor
    from cdnaml.ml.xgboost import XgboostRegressor
    from cdnaml.models import util
    from cdnaml.sql import types as T
    from cdnaml.utils.synthetic import forest_digest
    comm = spark.comm
    W, r = comm.world_size, comm.rank
    n, d = 3001, 8
    rng = np.random.default_rng(5)
    X = rng.normal(size=(n, d)).astype(np.float32)
    y = (X[:, 0] * 2 - X[:, 1] + np.sin(2 * X[:, 2])).astype(np.float64)
    owners = max(W - 1, 1)  # the last rank of a multi-rank job holds no rows
    a, b = (n * r // owners, n * (r + 1) // owners) if r < owners else (n, n)

    def chunks():
        for r0 in range(a, b, 700):
            yield {"features": X[r0:min(b, r0 + 700)], "label": y[r0:min(b, r0 + 700)]}
    schema = T.StructType([T.StructField("features", T.VectorUDT(), True),
                           T.StructField("label", T.DoubleType(), True)])
    df = spark.createDataFrameFromChunks(chunks, max_rows=700, schema=schema)
    seen = {"streamed": 0}
    orig = util.streamed_columns

    def counted(*args, **kw):
        res = orig(*args, **kw)
        seen["streamed"] += res is not None
        return res
    import cdnaml.models.regression as R
    import cdnaml.models.xgboost as XG
    R.streamed_columns = XG.streamed_columns = counted
    out = {}
    for k, est in {"rf": RandomForestRegressor(numTrees=6, maxDepth=4, maxBins=32, seed=2),
                   "xgb": XgboostRegressor(n_estimators=3, max_depth=3, learning_rate=0.3, random_state=1,
                                           missing=0.0)}.items():
        out[k] = forest_digest(est.fit(df)._forest)
    out["streamed"] = int(comm.all_reduce_scalar(float(seen["streamed"]), "min"))
    return out


def scenario_cv(spark):
    from cdnaml.ml.evaluation import RegressionEvaluator
    from cdnaml.ml.regression import RandomForestRegressor
    from cdnaml.ml.tuning import CrossValidator, ParamGridBuilder
    df = _tree_df(spark, n=3000, d=6)
    rf = RandomForestRegressor(maxBins=32, seed=42)
    grid = ParamGridBuilder().addGrid(rf.maxDepth, [2, 4]).addGrid(rf.numTrees, [3, 6]).build()
    cv = CrossValidator(estimator=rf, estimatorParamMaps=grid, evaluator=RegressionEvaluator(), numFolds=3,
                        seed=42, parallelism=2)
    m = cv.fit(df)
    from cdnaml.utils.synthetic import forest_digest
    return {"avg": [round(float(v), 9) for v in m.avgMetrics], "best": forest_digest(m.bestModel._forest)}


def scenario_als(spark):
    from cdnaml.ml.recommendation import ALS
    rng = np.random.default_rng(5)
    nu, ni, r = 60, 40, 3
    U, V = rng.normal(size=(nu, r)), rng.normal(size=(ni, r))
    pairs = rng.choice(nu * ni, size=1500, replace=False)
    u, i = pairs // ni, pairs % ni
    pdf = pd.DataFrame({"userId": u, "movieId": i, "rating": (U[u] * V[i]).sum(1) + 3.0})
    df = spark.createDataFrame(pdf)
    comm = spark.comm
    a2a0 = comm.op_calls.get("all_to_all", 0)
    out = {}
    for name, kw in (("uf", {}), ("uf_implicit", {"implicitPrefs": True, "alpha": 2.0}),
                     ("uf_nonneg", {"nonnegative": True})):
        m = ALS(rank=3, maxIter=5, regParam=0.05, seed=42, userCol="userId", itemCol="movieId",
                ratingCol="rating", **kw).fit(df)
        out[name] = np.asarray(m._U, dtype=np.float64).reshape(-1).tolist()
        out[name.replace("uf", "vf")] = np.asarray(m._V, dtype=np.float64).reshape(-1).tolist()
    # block ALS (W > 1): factor blocks travel by all-to-all, no dense [n, r, r] all-reduce
    out["block"] = comm.world_size == 1 or comm.op_calls.get("all_to_all", 0) > a2a0
    return out


def scenario_hyperopt(spark):
    """GPUTrials in SPMD: trials spread over ranks (each a rank-local engine fit), results all-gathered; the
    search history must equal the one-process search."""
    from cdnaml.hyperopt import GPUTrials, fmin, hp, tpe
    from cdnaml.ml.evaluation import RegressionEvaluator
    from cdnaml.ml.feature import VectorAssembler
    from cdnaml.ml.regression import LinearRegression
    rng = np.random.default_rng(1)
    X = rng.normal(size=(400, 3))
    pdf = pd.DataFrame(X, columns=["a", "b", "c"])
    pdf["label"] = X @ np.array([1.0, -2.0, 0.5]) + 0.3 * rng.normal(size=400)

    def objective(p):
        df = spark.createDataFrame(pdf)                       # rank-local inside a trial: the full table
        va = VectorAssembler(inputCols=["a", "b", "c"], outputCol="features")
        m = LinearRegression(regParam=p["reg"], elasticNetParam=p["en"]).fit(va.transform(df))
        return round(RegressionEvaluator().evaluate(m.transform(va.transform(df))), 9)

    trials = GPUTrials(parallelism=2)
    best = fmin(objective, {"reg": hp.loguniform("reg", -6, 0), "en": hp.choice("en", [0.0, 0.5])},
                algo=tpe.suggest, max_evals=8, trials=trials, rstate=np.random.default_rng(7))
    return {"losses": [round(float(x), 9) for x in trials.losses()], "best_en": int(best["en"]),
            "best_reg": round(float(best["reg"]), 12), "n": len(trials.trials)}


def scenario_hyperopt_captured(spark):
    """the objective closes over DataFrames created BEFORE fmin (the course pattern, ML 08:91-104):
    each rank-local trial must still fit on the whole table, so the losses equal the one-process search."""
    from cdnaml.hyperopt import GPUTrials, fmin, hp, tpe
    from cdnaml.ml.evaluation import RegressionEvaluator
    from cdnaml.ml.feature import VectorAssembler
    from cdnaml.ml.regression import LinearRegression
    rng = np.random.default_rng(2)
    X = rng.normal(size=(500, 3))
    pdf = pd.DataFrame(X, columns=["a", "b", "c"])
    pdf["label"] = X @ np.array([0.5, 1.0, -1.5]) + 0.2 * rng.normal(size=500)
    train_df = spark.createDataFrame(pdf)                     # sharded: 1/W of the rows on each rank
    va = VectorAssembler(inputCols=["a", "b", "c"], outputCol="features")
    assembled = va.transform(train_df)                        # a vector column, captured too

    def objective(p):
        m = LinearRegression(regParam=p["reg"]).fit(assembled)
        n = train_df.count()
        return round(RegressionEvaluator().evaluate(m.transform(va.transform(train_df))), 9) + 1000.0 * (n != 500)

    trials = GPUTrials(parallelism=2)
    fmin(objective, {"reg": hp.loguniform("reg", -6, 0)}, algo=tpe.suggest, max_evals=6, trials=trials,
         rstate=np.random.default_rng(3))
    # after the search the captured frame is sharded again
    return {"losses": [round(float(x), 9) for x in trials.losses()], "n_after": train_df.count(),
            "restored": sum(b.n for b in train_df._local()) == 500 // spark.comm.world_size}


SCENARIOS = {"frame": scenario_frame, "ml": scenario_ml, "fault": scenario_fault, "trees": scenario_trees,
             "trees_uneven": scenario_trees_uneven, "trees_rs": scenario_trees_rs,
             "trees_rs_overlap": scenario_trees_rs_overlap, "trees_deep": scenario_trees_deep, "cv": scenario_cv, "als": scenario_als,
             "hyperopt": scenario_hyperopt,
             "ooc_uneven": scenario_ooc_uneven,
             "trees_rs_nccl": scenario_trees_rs_nccl,
             "hyperopt_captured": scenario_hyperopt_captured, "trace_rs_overlap": scenario_trace_rs_overlap}


def run(name):
    if name.endswith("_nccl") and int(os.environ.get("WORLD_SIZE", "1")) > 1:
        # the recording nccl-over-gloo proxy must be in place before the session builds its Comm
        sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
        import torch.distributed as dist
        import fake_nccl
        from cdnaml.parallel import comm as comm_mod
        comm_mod.init_from_env()
        assert dist.get_backend() == "gloo"
        fake_nccl.install(comm_mod)
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
    if sys.argv[1] != "fault":
        # orderly teardown (barrier, then destroy the group): left to interpreter exit, a gloo rank whose peer
        # already closed its sockets can abort ("terminate called without an active exception", SIGABRT)
        import cdnaml
        cdnaml.SparkSession.getActiveSession().comm.shutdown()
