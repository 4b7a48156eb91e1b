#!/usr/bin/env python
"""The other BASELINE.json configurations (the headline RF config is bench.py).

    python bench_configs.py lr        # 2: LinearRegression normal equations, bf16 MFMA Gram, 1e7 x 100
    python bench_configs.py cv        # 3: RandomForestRegressor + CrossValidator grid, 1e8 x 100
    python bench_configs.py clf       # L07 at scale: RandomForestClassifier + CrossValidator grid, 1e7 x 100
    python bench_configs.py gbdt      # 4: XGBoost-style GBDT, depth 8, 1e8 x 100 (rounds/s; --trees)
    python bench_configs.py infer     # 5: batch inference of a trained RF over 1e9 streamed rows (transform)
    python bench_configs.py airbnb    # 1: ML 02 LinearRegression on the Airbnb-SF schema (CPU plumbing)
    python bench_configs.py relational  # groupBy-count / groupBy-avg / join / dropDuplicates on 1e8 rows

Each prints one JSON line (same fields as bench.py).  Multi-GPU: launch under
``torch.distributed.run`` exactly like bench.py; rows are split across ranks.
Synthetic data is generated directly in HBM.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))


def _log(msg):
    if int(os.environ.get("RANK", "0")) == 0:
        print(f"[bench_configs] {msg}", file=sys.stderr, flush=True)


def _sync(dev):
    if dev.type == "cuda":
        torch.cuda.synchronize()


def _emit(spark, metric, value, unit, steps, warmup, ms, hib, scaling, dtype, model, rows, par,
          data="synthetic (generated in HBM)"):
    if spark.comm.rank == 0:
        print(json.dumps({"metric": metric, "value": value, "unit": unit, "n_gpus": spark.comm.world_size,
                          "steps": steps, "warmup": warmup, "ms_per_step": ms, "higher_is_better": hib,
                          "scaling": scaling, "vs_baseline": None, "dtype": dtype,
                          "data": data,
                          "config": {"model": model, "global_batch": rows, "seq_len": None, "parallelism": par}}),
              flush=True)


def _data(spark, n_total, d, seed=42, cls=False):
    comm = spark.comm
    W, rank = comm.world_size, comm.rank
    a, b = n_total * rank // W, n_total * (rank + 1) // W
    n = b - a
    dev = spark.device
    g = torch.Generator(device=dev).manual_seed(seed * 1000 + rank)
    X = torch.randn((n, d), generator=g, device=dev, dtype=torch.float32)
    wv = torch.randn(d, generator=torch.Generator(device=dev).manual_seed(seed), device=dev)
    y = (X @ wv).double() + 2.0 * torch.sin(X[:, 0].double() * 2.0) + 0.1 * torch.randn(
        n, generator=g, device=dev, dtype=torch.float64)
    if cls:
        y = (y > 0).double()
    return spark.createDataFrameFromLocalTensors({"features": X, "label": y}), n


TRACE = None


def _timed(spark, fn, steps, warmup):
    dev = spark.device
    if TRACE:
        from cdnaml.utils import tracing
        tracing.reset()
        tracing.enable()
        fn()
        _sync(dev)
        tracing.disable()
        _log("traced run (untimed):\n" + tracing.summary())
        tracing.export_chrome_trace(TRACE)
    for _ in range(warmup):
        fn()
    _sync(dev)
    spark.comm.barrier()
    _sync(dev)
    t0 = time.perf_counter()
    out = None
    for _ in range(steps):
        out = fn()
    _sync(dev)
    spark.comm.barrier()
    el = spark.comm.all_reduce_scalar(time.perf_counter() - t0, "max")
    return el / steps * 1000.0, out


def bench_lr(spark, args):
    from cdnaml.models.regression import LinearRegression
    n_total = int(args.rows or 1e7)
    df, n = _data(spark, n_total, 100)
    lr = LinearRegression(gramPrecision="bf16")
    # a ~1.3 ms fit: the default 3 timed fits right after one warmup read 1.6-1.7 ms on some boxes against 1.32 ms
    # steady state over 20 (scripts/lr_host_probe.py), so this config times 20 unless --steps says otherwise
    if args.steps_default:
        args.steps = 20
    ms, model = _timed(spark, lambda: lr.fit(df), args.steps, args.warmup)
    _log(f"LR fit {ms:.2f} ms, intercept {model.intercept:.4f}")
    _emit(spark, "rows/sec LinearRegression.fit (normal equations, bf16 MFMA Gram)", n_total / (ms / 1e3),
          "rows/s", args.steps, args.warmup, ms, True, "strong", "bf16", "LinearRegression(d=100)", n_total,
          f"dp{spark.comm.world_size}")


def bench_clf(spark, args):
    """S/Labs/ML 07L - Hyperparameter Tuning Lab.py:82,105-108,140-155 at scale: RandomForestClassifier (Gini,
    maxBins 40) over the lab's exact 3x3 grid maxDepth {2, 5, 10} x numTrees {10, 20, 100} with a 3-fold
    CrossValidator and BinaryClassificationEvaluator (areaUnderROC), 1e7 x 100 binary labels (--grid small: the
    round-3 2x2 grid {2, 5} x {5, 10}).  The fused tuner grows one forest per fold at the group's largest numTrees /
    maxDepth (100 trees, depth 10): binary labels ride the packed record path (class counts from (W, W1) sums,
    levels 0-7 on the row codes, node ids from level 8)."""
    from cdnaml.ml.classification import RandomForestClassifier
    from cdnaml.ml.evaluation import BinaryClassificationEvaluator
    from cdnaml.ml.tuning import CrossValidator, ParamGridBuilder
    n_total = int(args.rows or 1e7)
    df, n = _data(spark, n_total, 100, cls=True)
    rf = RandomForestClassifier(maxBins=40, seed=42)
    depths, trees = ([2, 5], [5, 10]) if args.grid == "small" else ([2, 5, 10], [10, 20, 100])
    grid = ParamGridBuilder().addGrid(rf.maxDepth, depths).addGrid(rf.numTrees, trees).build()
    cv = CrossValidator(estimator=rf, estimatorParamMaps=grid, evaluator=BinaryClassificationEvaluator(),
                        numFolds=3, seed=42)
    ms, model = _timed(spark, lambda: cv.fit(df), args.steps, args.warmup)
    _log(f"RF classifier CV {ms:.1f} ms for {len(grid) * 3 + 1} fits, best maxDepth={model.bestModel.getMaxDepth()} "
         f"numTrees={model.bestModel.getNumTrees}, AUC {max(model.avgMetrics):.4f}")
    gname = f"{len(depths)}x{len(trees)}"
    _emit(spark, f"rows/sec CrossValidator(RandomForestClassifier grid {gname}, 3 folds) fit", n_total / (ms / 1e3),
          "rows/s", args.steps, args.warmup, ms, True, "strong", "fp32",
          f"RandomForestClassifier(maxBins=40) CV maxDepth {depths} x numTrees {trees} x 3 folds", n_total,
          f"dp{spark.comm.world_size}")


def bench_cv(spark, args):
    from cdnaml.ml.evaluation import RegressionEvaluator
    from cdnaml.ml.tuning import CrossValidator, ParamGridBuilder
    from cdnaml.models.regression import RandomForestRegressor
    n_total = int(args.rows or 1e8)
    df, n = _data(spark, n_total, 100)
    rf = RandomForestRegressor(maxBins=40, seed=42)
    grid = ParamGridBuilder().addGrid(rf.maxDepth, [2, 5]).addGrid(rf.numTrees, [5, 10]).build()
    cv = CrossValidator(estimator=rf, estimatorParamMaps=grid, evaluator=RegressionEvaluator(), numFolds=3,
                        seed=42)
    ms, model = _timed(spark, lambda: cv.fit(df), args.steps, args.warmup)
    fits = len(grid) * 3 + 1
    _log(f"CV {ms:.1f} ms for {fits} fits, best maxDepth={model.bestModel.getMaxDepth()}")
    _emit(spark, "rows/sec CrossValidator(RandomForestRegressor grid 2x2, 3 folds) fit",
          n_total / (ms / 1e3), "rows/s", args.steps, args.warmup, ms, True, "strong", "fp32",
          "CrossValidator(RandomForestRegressor, maxDepth{2,5} x numTrees{5,10}, 3 folds, maxBins=40)",
          n_total, f"dp{spark.comm.world_size}")


def bench_gbdt(spark, args):
    from cdnaml.models.xgboost import XgboostRegressor
    n_total = int(args.rows or 1e8)
    df, n = _data(spark, n_total, 100)
    trees = args.trees or 500
    est = XgboostRegressor(n_estimators=trees, max_depth=8, learning_rate=0.1, max_bin=256, random_state=42)
    ms, model = _timed(spark, lambda: est.fit(df), args.steps, args.warmup)
    _log(f"GBDT {trees} trees depth 8: {ms:.1f} ms ({ms / trees:.2f} ms/tree)")
    _emit(spark, "boosting rounds/sec, XGBoost-style GBDT depth 8, 1e8x100", trees / (ms / 1e3), "trees/s",
          args.steps, args.warmup, ms, True, "strong", "fp32",
          f"XgboostRegressor(n_estimators={trees},max_depth=8,max_bin=256)", n_total,
          f"dp{spark.comm.world_size}")


def bench_infer(spark, args):
    """Config 5 through the product path: ``model.transform`` over a STREAMED DataFrame of 1e9 rows x 100
    fp32 features (400 GB: larger than HBM), consumed chunk by chunk with ``foreachBatch``.

    --mode host (default): chunks come from pinned host memory through ``createDataFrameFromChunks``
    (pinned double buffers, H2D on a copy stream overlapping the predict; the H2D of all 400 GB is in the
    timed region).  The host pool holds --pool distinct chunks, cycled (host RAM cannot hold 400 GB).
    --mode device: every chunk is generated on the device (``K.normal32_``: Philox normals keyed by global row
    id, one HBM write per element) into two staging buffers of ``device_chunks``: 1e9 distinct rows, with
    their generation inside the timed region.
    In both modes the forest is uploaded once and each staging buffer's predict is a replayed HIP graph."""
    from cdnaml.models.inference import device_chunks
    from cdnaml.models.regression import RandomForestRegressor
    dev = spark.device
    comm = spark.comm
    train, _ = _data(spark, int(2e6), 100)
    model = RandomForestRegressor(numTrees=20, maxDepth=5, maxBins=40, seed=42).fit(train)
    n_total = int(args.rows or 1e9)
    chunk = int(args.chunk)
    per_rank = n_total // comm.world_size
    n_chunks = max(1, per_rank // chunk)
    rows = n_chunks * chunk * comm.world_size
    g = torch.Generator(device=dev).manual_seed(7 + comm.rank)
    if args.mode == "host" and dev.type == "cuda":
        pool = []
        for _ in range(int(args.pool)):
            h = torch.empty((chunk, 100), dtype=torch.float32, pin_memory=True)
            h.copy_(torch.randn((chunk, 100), generator=g, dtype=torch.float32, device=dev).cpu())
            pool.append(h)

        def chunks():
            for i in range(n_chunks):
                yield {"features": pool[i % len(pool)]}
        df = spark.createDataFrameFromChunks(chunks, chunk)
    else:
        from cdnaml.ops import kernels as K
        row_base = comm.rank * n_chunks * chunk

        def make(r0, n, bufs):
            # every chunk is new data: rows keyed by global row id (Philox normals written straight into the
            # staging buffer on the compute stream), so the 1e9 rows are distinct and their generation is timed
            K.normal32_(bufs["features"][:n], 7, (row_base + r0) * 100, 0x10)
        df = device_chunks(spark, n_chunks * chunk, chunk, make, {"features": ((100,), torch.float32)})
    udf = None
    if args.api == "spark_udf":
        # the reference's route (ML 09 - AutoML.py:78-82, Labs/ML 12L:78-96): log the model with the tracking
        # flavour, load it as a Spark UDF from "runs:/<id>/model" and apply it column-wise to the streamed frame
        import tempfile
        from cdnaml import tracking as mlflow
        from cdnaml.models.pipeline import PipelineModel
        mlflow.set_tracking_uri(os.path.join(tempfile.mkdtemp(prefix="cfg_infer_"), "mlruns"))
        with mlflow.start_run() as run:
            mlflow.spark.log_model(PipelineModel([model]), "model")
        udf = mlflow.pyfunc.spark_udf(spark, f"runs:/{run.info.run_id}/model")
        pred = df.withColumn("prediction", udf("features"))
    else:
        pred = model.transform(df)
    acc = torch.zeros((), dtype=torch.float64, device=dev)

    def consume(b):
        acc.add_(b.columns["prediction"].values.sum())

    def step():
        acc.zero_()
        pred.foreachBatch(consume)
        return acc
    ms, tot = _timed(spark, step, args.steps, args.warmup)
    if args.mode == "device" and dev.type == "cuda":
        scratch = {"features": torch.empty((chunk, 100), dtype=torch.float32, device=dev)}
        gen_ms, _ = _timed(spark, lambda: [make(i * chunk, chunk, scratch) for i in range(n_chunks)], 2, 1)
        del scratch
        _log(f"generation alone: {gen_ms:.1f} ms ({n_chunks * chunk * 400 / gen_ms / 1e9:.2f} TB/s written)")
    from cdnaml.models.inference import predictor_for
    pr = predictor_for(udf.pm.stages[-1] if udf is not None else model, "value", [0.0])
    _log(f"inference {rows:.3e} rows in {ms:.1f} ms (mode={args.mode}, api={args.api}); graph captures="
         f"{pr.captures} replays={pr.replays}; mean prediction {float(tot) / (n_chunks * chunk):.6f}"
         + (f"; udf batches={udf.batches} plans built={udf.plans_built}" if udf is not None else ""))
    src = "pinned host chunks, H2D in the timed region" if args.mode == "host" else \
        "distinct rows generated on device per chunk, generation in the timed region"
    via = "mlflow.pyfunc.spark_udf (runs:/ URI) in withColumn" if args.api == "spark_udf" else "DataFrame transform"
    _emit(spark, f"rows/sec batch inference via {via}, RandomForest (20 trees, depth 5), 1e9 rows "
                 f"({src})", rows / (ms / 1e3), "rows/s", args.steps, args.warmup, ms, True,
          "weak" if comm.world_size > 1 else "strong", "fp32",
          f"RandomForestRegressionModel(numTrees=20,maxDepth=5) via {via}, streamed, hipGraph-replayed predict",
          rows, f"dp{comm.world_size}")


def bench_relational(spark, args):
    """groupBy-count, a fact x dimension join and dropDuplicates on 1e8 rows (K16 hash tables, K19 compaction;
    Labs/ML 00L - Dedup Lab.py:79-107, ML 01 - Data Cleansing.py:93,157-160, MLE 01:332-374)."""
    from cdnaml.sql import functions as F
    dev = spark.device
    comm = spark.comm
    n_total = int(args.rows or 1e8)
    a, b = n_total * comm.rank // comm.world_size, n_total * (comm.rank + 1) // comm.world_size
    n = b - a
    g = torch.Generator(device=dev).manual_seed(11 + comm.rank)
    k = torch.randint(0, 1_000_000, (n,), generator=g, device=dev)
    k2 = torch.randint(0, 50, (n,), generator=g, device=dev)
    v = torch.randn(n, generator=g, device=dev, dtype=torch.float64)
    fact = spark.createDataFrameFromLocalTensors({"k": k, "k2": k2, "v": v})
    dk = torch.arange(0, 1_000_000, 4, device=dev)
    dim = spark.createDataFrameFromLocalTensors({"k": dk, "w": dk.double() * 0.5}) if comm.rank == 0 else \
        spark.createDataFrameFromLocalTensors({"k": dk[:0], "w": dk[:0].double()})
    ops = {
        "groupBy(k).count": lambda: fact.groupBy("k").count().count(),
        "groupBy(k2).avg": lambda: fact.groupBy("k2").agg(F.avg("v")).count(),
        "join(dim on k)": lambda: fact.join(dim, on="k").count(),
        "dropDuplicates(k, k2)": lambda: fact.dropDuplicates(["k", "k2"]).count(),
    }
    total = 0.0
    for name, fn in ops.items():
        ms, cnt = _timed(spark, fn, args.steps, args.warmup)
        total += ms
        _log(f"{name}: {ms:.1f} ms -> {cnt} rows")
    _emit(spark, "rows/sec relational suite (groupBy-count, groupBy-avg, join, dropDuplicates) on 1e8 rows",
          4 * n_total / (total / 1e3), "rows/s", args.steps, args.warmup, total, True, "strong", "fp64",
          "groupBy/join/dropDuplicates on K16 device hash tables", n_total, f"dp{comm.world_size}")


def bench_expr(spark, args):
    """K18: feature-engineering expressions of the course (ML 01 price cast / filters, L03 log-price and exp back,
    MLE 03 when-label, ML 02 ratios) over 1e8 rows, one fused kernel each vs the operator-at-a-time path."""
    from cdnaml.sql import functions as F
    from cdnaml.sql import fused
    dev = spark.device
    comm = spark.comm
    n_total = int(args.rows or 1e8)
    n = n_total * (comm.rank + 1) // comm.world_size - n_total * comm.rank // comm.world_size
    g = torch.Generator(device=dev).manual_seed(5 + comm.rank)
    price = torch.exp(torch.randn(n, generator=g, device=dev, dtype=torch.float64) + 4.5)
    beds = torch.randint(0, 6, (n,), generator=g, device=dev, dtype=torch.int32)
    acc = torch.randint(1, 12, (n,), generator=g, device=dev, dtype=torch.int32)
    df = spark.createDataFrameFromLocalTensors({"price": price, "bedrooms": beds, "accommodates": acc})
    p, b, a = F.col("price"), F.col("bedrooms"), F.col("accommodates")
    exprs = {
        "log_price -> exp": F.exp(F.log(p) * 0.5 + 1.0) - 1.0,
        "price per bed": F.when(b > 0, p / b).otherwise(p),
        "priceClass label": F.when((p >= 150) & (a > 2), 1.0).otherwise(0.0),
        "ratio + round": F.round(p / (a * 1.0) * 100.0, 2) + F.sqrt(b * 1.0),
    }
    total = {True: 0.0, False: 0.0}
    for name, e in exprs.items():
        res = {}
        for on in (False, True):
            fused.FUSE = on
            ms, _ = _timed(spark, lambda: df.select(e.alias("r"))._plan.execute(), args.steps, args.warmup)
            res[on] = ms
            total[on] += ms
        _log(f"{name}: operator path {res[False]:.2f} ms, fused {res[True]:.2f} ms ({res[False] / res[True]:.1f}x)")
    fused.FUSE = True
    _log(f"total: operator path {total[False]:.2f} ms, fused {total[True]:.2f} ms")
    _emit(spark, "rows/sec fused column expressions (4 course feature expressions) on 1e8 rows",
          4 * n_total / (total[True] / 1e3), "rows/s", args.steps, args.warmup, total[True], True, "strong", "fp64",
          "K18 expr.hip fused elementwise", n_total, f"dp{comm.world_size}")


def bench_airbnb(spark, args):
    from cdnaml.ml.evaluation import RegressionEvaluator
    from cdnaml.ml.feature import VectorAssembler
    from cdnaml.ml.regression import LinearRegression
    from cdnaml.utils import datasets as D
    pdf = D.airbnb_clean()
    df = spark.createDataFrame(pdf)
    train, test = df.randomSplit([.8, .2], seed=42)
    va = VectorAssembler(inputCols=["bedrooms"], outputCol="features")

    def fit():
        m = LinearRegression(featuresCol="features", labelCol="price").fit(va.transform(train))
        return RegressionEvaluator(labelCol="price").evaluate(m.transform(va.transform(test)))
    ms, rmse = _timed(spark, fit, args.steps, args.warmup)
    _log(f"ML 02 LR on Airbnb schema: rmse {rmse:.2f}")
    _emit(spark, "ML 02 LinearRegression on Airbnb-SF schema (fit + evaluate latency)", ms, "ms", args.steps,
          args.warmup, ms, False, "strong", "fp64", "LinearRegression(bedrooms -> price)", len(pdf),
          f"dp{spark.comm.world_size}")


def bench_ooc(spark, args):
    """Out-of-core fits over a STREAMED frame too large for resident fp32 X: 5e8 x 100 rows
    (200 GB of fp32 features) generated chunk by chunk on the device (``device_chunks``; Philox normals keyed by
    global row id, label = a nonlinear function of the chunk's features), so every pass over the data -- the
    label pass, the quantile-sample pass, the binning pass (RF) or the Gram pass (LR) -- regenerates the rows and
    the generation is inside the timed region.  Resident: uint8 bins (+ seg10 rows), labels, codes.
    --model lr (default) | rf (RandomForestRegressor numTrees=--trees (4), maxDepth 5, maxBins 40)."""
    from cdnaml.models.inference import device_chunks
    from cdnaml.models.regression import LinearRegression, RandomForestRegressor
    from cdnaml.ops import kernels as K
    dev = spark.device
    comm = spark.comm
    n_total = int(args.rows or 5e8)
    chunk = int(args.chunk)
    per_rank = n_total // comm.world_size
    n_chunks = max(1, per_rank // chunk)
    rows = n_chunks * chunk * comm.world_size
    row_base = comm.rank * n_chunks * chunk
    wv = torch.randn(100, generator=torch.Generator(device=dev).manual_seed(3), device=dev)

    def make(r0, n, bufs):
        X = bufs["features"][:n]
        K.normal32_(X, 11, (row_base + r0) * 100, 0x10)
        torch.matmul(X, wv, out=bufs["label"][:n])
        bufs["label"][:n].add_(torch.sin(2.0 * X[:, 0]))
    if args.source == "host" and dev.type == "cuda":
        # pinned host chunks through createDataFrameFromChunks (pinned staging, H2D on the copy stream overlapping
        # the compute): every pass over the frame moves all rows over PCIe inside the timed region.  The host pool
        # holds --pool distinct chunks, cycled (host RAM cannot hold 320 GB of rows either).
        pool = []
        scratch = {"features": torch.empty((chunk, 100), dtype=torch.float32, device=dev),
                   "label": torch.empty((chunk,), dtype=torch.float32, device=dev)}
        for i in range(int(args.pool)):
            make(i * chunk, chunk, scratch)
            pool.append({k: v.cpu().pin_memory() for k, v in scratch.items()})
        del scratch

        def host_chunks():
            for i in range(n_chunks):
                yield pool[i % len(pool)]
        df = spark.createDataFrameFromChunks(host_chunks, chunk)
    else:
        df = device_chunks(spark, n_chunks * chunk, chunk, make,
                           {"features": ((100,), torch.float32), "label": ((), torch.float32)})
    if args.model == "rf":
        T = int(args.trees or 4)
        est = RandomForestRegressor(numTrees=T, maxDepth=5, maxBins=40, seed=42)
        name = f"RandomForestRegressor(numTrees={T},maxDepth=5,maxBins=40) streamed"
    else:
        est = LinearRegression()
        name = "LinearRegression(d=100) streamed"
    ms, model = _timed(spark, lambda: est.fit(df), args.steps, args.warmup)
    peak = torch.cuda.max_memory_allocated(dev) / 2 ** 30 if dev.type == "cuda" else 0.0
    _log(f"ooc {args.model}: {ms:.1f} ms per fit, {rows / ms * 1e3:.3e} rows/s, peak allocated {peak:.1f} GiB "
         f"(fp32 X would be {rows * 400 / 2 ** 30:.0f} GiB)")
    src = "pinned host chunks (cycled pool), H2D in the timed region" if args.source == "host" else \
        "chunks generated on device, generation in the timed region"
    _emit(spark, f"rows/sec out-of-core fit ({name}; {src})", rows / ms * 1e3, "rows/s", args.steps, args.warmup,
          ms, True, "strong", "fp32", name, rows, f"dp{comm.world_size}",
          data="synthetic (generated on the device, copied to pinned host chunks)" if args.source == "host"
          else "synthetic (generated in HBM)")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("config", choices=["lr", "cv", "clf", "gbdt", "infer", "airbnb", "relational", "expr", "ooc"])
    ap.add_argument("--model", choices=["lr", "rf"], default="lr", help="ooc: the streamed estimator")
    ap.add_argument("--grid", choices=["lab", "small"], default="lab", help="clf: the L07 3x3 grid or the 2x2 one")
    ap.add_argument("--rows", type=float, default=None)
    ap.add_argument("--steps", type=int, default=None, help="timed repetitions (default 3; lr: 20)")
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--trees", type=int, default=None)
    ap.add_argument("--chunk", type=float, default=1e7)
    ap.add_argument("--mode", choices=["host", "device"], default="host")
    ap.add_argument("--api", choices=["transform", "spark_udf"], default="transform",
                    help="infer: model.transform, or the tracking flavour loaded with pyfunc.spark_udf")
    ap.add_argument("--pool", type=int, default=6, help="distinct pinned host chunks (--mode host / --source host)")
    ap.add_argument("--source", choices=["host", "device"], default="device", help="ooc: where the chunks come from")
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--trace", default="", help="run one traced (untimed) step first; Chrome trace path")
    args = ap.parse_args()
    args.steps_default = args.steps is None
    if args.steps is None:
        args.steps = 3
    global TRACE
    TRACE = args.trace or None
    import cdnaml
    spark = cdnaml.SparkSession.builder.appName("bench_configs").getOrCreate()
    {"lr": bench_lr, "cv": bench_cv, "clf": bench_clf, "gbdt": bench_gbdt, "infer": bench_infer, "airbnb": bench_airbnb,
     "ooc": bench_ooc,
     "relational": bench_relational, "expr": bench_expr}[
        args.config](spark, args)
    spark.comm.shutdown()


if __name__ == "__main__":
    main()
