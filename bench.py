#!/usr/bin/env python
"""Headline benchmark: rows/sec of RandomForestRegressor fit+transform on
1e8 x 100 synthetic rows (BASELINE.json), 1/2/4/8 MI355X GPUs.

    python bench.py --gpus N --steps K --warmup W
    python -m torch.distributed.run --nnodes=1 --nproc-per-node N \
        --master-addr 127.0.0.1 --master-port P bench.py --gpus N --steps K --warmup W

One process per GPU (RCCL over xGMI).  The 1e8-row dataset is fixed and split
across ranks (strong scaling); it is generated directly in HBM (synthetic,
random features, a nonlinear label).  A step = ``RandomForestRegressor.fit``
(global quantile binning, bootstrap, level-wise histogram build + RCCL
all-reduce, split search, row partition) + ``model.transform`` over all rows
(prediction column materialised on device).  Rank 0 prints one JSON line.
"""
from __future__ import annotations

import argparse
import json
import math
import os
import sys
import time

import torch


def log(msg):
    if int(os.environ.get("RANK", "0")) == 0:
        print(f"[bench] {msg}", file=sys.stderr, flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--rows", type=float, default=1e8, help="total rows (fixed across GPU counts)")
    ap.add_argument("--features", type=int, default=100)
    ap.add_argument("--trees", type=int, default=20)
    ap.add_argument("--depth", type=int, default=5)
    ap.add_argument("--bins", type=int, default=40)
    ap.add_argument("--seed", type=int, default=42)
    ap.add_argument("--trace", default="", help="after timing, run one traced step; write a Chrome trace here")
    args = ap.parse_args()

    sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
    import cdnaml
    from cdnaml.models.regression import RandomForestRegressor

    spark = cdnaml.SparkSession.builder.appName("bench").getOrCreate()
    comm = spark.comm
    W, rank = comm.world_size, comm.rank
    dev = spark.device
    n_total = int(args.rows)
    a, b = n_total * rank // W, n_total * (rank + 1) // W
    n = b - a
    d = args.features
    log(f"world={W} device={dev} rows/rank={n} features={d}")

    # ---- synthetic data, generated in HBM, keyed by GLOBAL row id (Philox): the 1e8-row table is the same
    # whatever the GPU count, so every N trains the identical forest (same nodes / digest)
    from cdnaml.utils.synthetic import forest_digest, regression_shard
    X, y, _ = regression_shard(n_total, d, args.seed, rank, W, dev)
    df = spark.createDataFrameFromLocalTensors({"features": X, "label": y})
    if dev.type == "cuda":
        torch.cuda.synchronize()
    log("data ready")

    rf = RandomForestRegressor(labelCol="label", featuresCol="features", numTrees=args.trees,
                               maxDepth=args.depth, maxBins=args.bins, seed=args.seed)

    from cdnaml.utils import tracing

    def step():
        with tracing.span("rf.fit"):
            model = rf.fit(df)
        with tracing.span("rf.transform"):
            parts = model.transform(df)._plan.execute()  # materialise predictions on device
        return model, parts

    for i in range(args.warmup):
        t0 = time.time()
        step()
        if dev.type == "cuda":
            torch.cuda.synchronize()
        log(f"warmup {i}: {time.time() - t0:.3f}s")

    comm.barrier()
    if dev.type == "cuda":
        torch.cuda.synchronize()
    t0 = time.perf_counter()
    marks = []
    for i in range(args.steps):
        model, parts = step()
        marks.append(time.perf_counter())
    if dev.type == "cuda":
        torch.cuda.synchronize()
    marks.append(time.perf_counter())
    comm.barrier()
    elapsed = time.perf_counter() - t0
    elapsed = comm.all_reduce_scalar(elapsed, "max")
    ms = elapsed / args.steps * 1000.0
    rows_per_s = n_total / (ms / 1000.0)
    # sanity: predictions are finite and correlate with the label
    p = parts[0].columns["prediction"].values
    ok = bool(torch.isfinite(p).all())
    corr = float(torch.corrcoef(torch.stack([p[:1000000], y[:1000000]]))[0, 1]) if n > 1 else float("nan")
    log(f"step {ms:.1f} ms, {rows_per_s:.3e} rows/s, pred finite={ok}, corr(pred,label)={corr:.3f}, "
        f"nodes={model.totalNumNodes} digest={forest_digest(model._forest)}")
    log("host step marks (ms): " + " ".join(f"{(b - a) * 1e3:.1f}" for a, b in zip([t0] + marks[:-1], marks)))
    if args.trace:
        tracing.reset()
        tracing.enable()
        step()
        if dev.type == "cuda":
            torch.cuda.synchronize()
        tracing.disable()
        log("traced step (untimed):\n" + tracing.summary())
        tracing.export_chrome_trace(args.trace if W == 1 else f"{args.trace}.rank{rank}")
    if rank == 0:
        print(json.dumps({
            "metric": "rows/sec fit+transform, RandomForestRegressor 1e8×100 synthetic, 1/2/4/8 GPU",
            "value": rows_per_s,
            "unit": "rows/s",
            "n_gpus": W,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": ms,
            "higher_is_better": True,
            "scaling": "strong",
            "vs_baseline": None,
            "dtype": "fp32",
            "data": "synthetic (Philox gaussian features keyed by global row id, generated in HBM; nonlinear label)",
            "config": {"model": f"RandomForestRegressor(numTrees={args.trees},maxDepth={args.depth},"
                                f"maxBins={args.bins})",
                       "global_batch": n_total, "seq_len": None, "num_features": d,
                       "parallelism": f"dp{W}"},
        }), flush=True)
    comm.shutdown()


if __name__ == "__main__":
    main()
