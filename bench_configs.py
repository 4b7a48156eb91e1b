#!/usr/bin/env python
"""The other BASELINE.json configurations (the headline RF config is bench.py).

    python bench_configs.py lr        # 2: LinearRegression normal equations, bf16 MFMA Gram, 1e7 x 100
    python bench_configs.py cv        # 3: RandomForestRegressor + CrossValidator grid, 1e8 x 100
    python bench_configs.py gbdt      # 4: XGBoost-style GBDT, depth 8, 1e8 x 100 (rounds/s; --trees)
    python bench_configs.py infer     # 5: batch inference of a trained RF over 1e9 rows (graph-captured)
    python bench_configs.py airbnb    # 1: ML 02 LinearRegression on the Airbnb-SF schema (CPU plumbing)

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


def _emit(spark, metric, value, unit, steps, warmup, ms, hib, scaling, dtype, model, rows, par):
    if spark.comm.rank == 0:
        print(json.dumps({"metric": metric, "value": value, "unit": unit, "n_gpus": spark.comm.world_size,
                          "steps": steps, "warmup": warmup, "ms_per_step": ms, "higher_is_better": hib,
                          "scaling": scaling, "vs_baseline": None, "dtype": dtype,
                          "data": "synthetic (generated in HBM)",
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
    ms, model = _timed(spark, lambda: lr.fit(df), args.steps, args.warmup)
    _log(f"LR fit {ms:.2f} ms, intercept {model.intercept:.4f}")
    _emit(spark, "rows/sec LinearRegression.fit (normal equations, bf16 MFMA Gram)", n_total / (ms / 1e3),
          "rows/s", args.steps, args.warmup, ms, True, "strong", "bf16", "LinearRegression(d=100)", n_total,
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
    """Stream synthetic chunks through a trained 20-tree RF; the per-chunk launch sequence is
    captured once in a HIP graph and replayed (1e9 rows do not fit in HBM as 100 float32 features)."""
    from cdnaml.models.regression import RandomForestRegressor
    dev = spark.device
    comm = spark.comm
    train, _ = _data(spark, int(2e6), 100)
    model = RandomForestRegressor(numTrees=20, maxDepth=5, maxBins=40, seed=42).fit(train)
    forest = model._forest
    n_total = int(args.rows or 1e9)
    chunk = int(args.chunk)
    per_rank = n_total // comm.world_size
    n_chunks = max(1, per_rank // chunk)
    tw = model._tree_w
    g = torch.Generator(device=dev).manual_seed(7 + comm.rank)
    # two resident chunk buffers scored alternately (each 20 GB at the default chunk, far
    # beyond L2/MALL, so every replay streams its features from HBM)
    bufs = [torch.randn((chunk, 100), generator=g, dtype=torch.float32, device=dev) for _ in range(2)]
    outs = [None, None]

    from cdnaml.ops import kernels as K
    nodes, roots, vals, masks = forest.device_arrays(dev, "value")
    tw_d = torch.tensor(np.asarray(tw, np.float32), device=dev)
    masks = masks.int().contiguous() if masks.numel() else torch.zeros(8, dtype=torch.int32, device=dev)

    heap = forest.heap_arrays(dev, "value") if dev.type == "cuda" else None

    def run_chunk(j):
        # device-resident forest arrays, no host->device traffic: capturable in a HIP graph
        out = K.tree_predict_heap(bufs[j], heap[0], heap[1], tw_d, heap[2]) if heap is not None else None
        outs[j] = out if out is not None else K.tree_predict(bufs[j], nodes, roots, tw_d, vals, masks, forest.K, None)
    graphs = None
    if dev.type == "cuda" and not args.no_graph:
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            run_chunk(0)
            run_chunk(1)
        torch.cuda.current_stream().wait_stream(s)
        graphs = []
        for j in range(2):
            gr = torch.cuda.CUDAGraph()
            with torch.cuda.graph(gr):
                run_chunk(j)
            graphs.append(gr)

    def step():
        for i in range(n_chunks):
            if graphs is not None:
                graphs[i & 1].replay()
            else:
                run_chunk(i & 1)
        return outs[(n_chunks - 1) & 1]
    ms, p = _timed(spark, step, args.steps, args.warmup)
    rows = n_chunks * chunk * comm.world_size
    _log(f"inference {rows:.3e} rows in {ms:.1f} ms; graph={graphs is not None}")
    _emit(spark, "rows/sec batch inference, trained RandomForest (20 trees, depth 5), 1e9 rows",
          rows / (ms / 1e3), "rows/s", args.steps, args.warmup, ms, True, "weak" if comm.world_size > 1 else "strong",
          "fp32", "RandomForestRegressionModel(numTrees=20,maxDepth=5) predict, hipGraph-captured", rows,
          f"dp{comm.world_size}")


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


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("config", choices=["lr", "cv", "gbdt", "infer", "airbnb"])
    ap.add_argument("--rows", type=float, default=None)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--trees", type=int, default=None)
    ap.add_argument("--chunk", type=float, default=2.5e7)
    ap.add_argument("--no-graph", action="store_true")
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--trace", default="", help="run one traced (untimed) step first; Chrome trace path")
    args = ap.parse_args()
    global TRACE
    TRACE = args.trace or None
    import cdnaml
    spark = cdnaml.SparkSession.builder.appName("bench_configs").getOrCreate()
    {"lr": bench_lr, "cv": bench_cv, "gbdt": bench_gbdt, "infer": bench_infer, "airbnb": bench_airbnb}[
        args.config](spark, args)


if __name__ == "__main__":
    main()
