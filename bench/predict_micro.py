"""K8 tree_predict microbenchmark: X tile streaming vs tree walking.

python bench/predict_micro.py --rows 1e8 --trees 20 --depth 5
Times the predict kernel for T trees and for 1 tree (≈ the cost of streaming X through LDS).
"""
import argparse
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from cdnaml.ops import kernels as K  # noqa: E402


def complete_forest(T, depth, d, seed=0):
    rng = np.random.default_rng(seed)
    nodes, vals, roots = [], [], []
    for t in range(T):
        base = len(nodes)
        roots.append(base)
        n_int = 2 ** depth - 1
        for i in range(2 ** (depth + 1) - 1):
            if i < n_int:
                thr = np.float32(rng.normal())
                nodes.append([int(rng.integers(0, d)), int(thr.view(np.int32)), base + 2 * i + 1, base + 2 * i + 2])
            else:
                nodes.append([-1, len(vals), base + i, base + i])
                vals.append(float(rng.normal()))
    return (torch.tensor(nodes, dtype=torch.int32), torch.tensor(roots, dtype=torch.int32),
            torch.tensor(vals, dtype=torch.float32))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=float, default=1e8)
    ap.add_argument("--features", type=int, default=100)
    ap.add_argument("--trees", type=int, default=20)
    ap.add_argument("--depth", type=int, default=5)
    ap.add_argument("--reps", type=int, default=3)
    a = ap.parse_args()
    dev = torch.device("cuda")
    n, d = int(a.rows), a.features
    X = torch.randn((n, d), device=dev)
    for T in (1, a.trees):
        nodes, roots, vals = complete_forest(T, a.depth, d)
        nodes, roots, vals = nodes.to(dev), roots.to(dev), vals.to(dev)
        tw = torch.full((T,), 1.0 / T, device=dev)
        masks = torch.zeros(8, dtype=torch.int32, device=dev)
        K.tree_predict(X, nodes, roots, tw, vals, masks, 1, None)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(a.reps):
            K.tree_predict(X, nodes, roots, tw, vals, masks, 1, None)
        torch.cuda.synchronize()
        ms = (time.perf_counter() - t0) / a.reps * 1e3
        print(f"T={T:3d} depth={a.depth} int4 nodes: {ms:7.2f} ms  {n / ms / 1e6:.3f}e9 rows/s  "
              f"{n * d * 4 / ms / 1e9:.2f} TB/s of X", flush=True)
        # heap layout: the complete trees above are already in heap order per tree
        S = 2 ** (a.depth + 1) - 1
        nh = nodes.cpu().numpy().reshape(T, S, 4)
        heap = np.stack([nh[..., 0], nh[..., 1]], -1).astype(np.int32)
        leaf = nh[..., 0] < 0
        vh = vals.cpu().numpy()
        heap[..., 1][leaf] = vh[nh[..., 1][leaf]].astype(np.float32).view(np.int32)
        heap_t = torch.from_numpy(heap).to(dev)
        ref = K.tree_predict(X[:100000], nodes, roots, tw, vals, masks, 1, None)
        got = K.tree_predict_heap(X[:100000], heap_t, a.depth, tw, masks)
        assert torch.allclose(ref, got, atol=1e-5), "heap predict mismatch"
        K.tree_predict_heap(X, heap_t, a.depth, tw, masks)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(a.reps):
            K.tree_predict_heap(X, heap_t, a.depth, tw, masks)
        torch.cuda.synchronize()
        ms = (time.perf_counter() - t0) / a.reps * 1e3
        print(f"T={T:3d} depth={a.depth} heap:       {ms:7.2f} ms  {n / ms / 1e6:.3f}e9 rows/s  "
              f"{n * d * 4 / ms / 1e9:.2f} TB/s of X", flush=True)


if __name__ == "__main__":
    main()
