"""Histogram-kernel microbenchmark: one tree level of an RF, timed per variant.

    python bench/hist_micro.py --rows 1e7 [--variants all]

Builds binned synthetic data, a level state (node ids / bootstrap weights /
feature masks for T trees with L active nodes each) and times the histogram
kernel alone with HIP events, reporting ms and lane-updates/s.
"""
import argparse
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from cdnaml.ops import kernels as K  # noqa: E402


def make_state(n, d, T, L, B, masked, seed=0, dev="cuda", sub=False):
    g = torch.Generator(device=dev).manual_seed(seed)
    X = torch.randn((n, d), generator=g, device=dev)
    thr = torch.linspace(-2, 2, B - 1, device=dev)[None, :].expand(d, -1).contiguous()
    nthr = torch.full((d,), B - 1, dtype=torch.int32, device=dev)
    bins = K.binize(X, thr, nthr)
    del X
    # active ids: tree-major, L per tree; rows spread uniformly over a tree's nodes
    node = (torch.randint(0, L, (T, n), generator=g, device=dev, dtype=torch.int32) +
            (torch.arange(T, device=dev, dtype=torch.int32) * L)[:, None]).contiguous()
    A = T * L
    if sub and L > 1:
        # full+subtract: only one child of each sibling pair is built (even local ids here)
        loc = np.tile(np.arange(L), T)
        bs = np.where(loc % 2 == 0, np.cumsum(loc % 2 == 0) - 1, -1).astype(np.int32)
        build = torch.from_numpy(bs).to(dev)
        slot_tree = np.repeat(np.arange(T), L // 2).astype(np.int32)
        return _finish(n, d, T, L, B, masked, g, bins, node, build, slot_tree, np.repeat(np.arange(T), L), dev)
    build = torch.arange(A, dtype=torch.int32, device=dev)
    slot_tree = np.repeat(np.arange(T), L).astype(np.int32)
    id_tree = slot_tree.copy()
    w = K.poisson_weights(T, n, 1, 0, 1.0, device=dev)
    fm = None
    if masked:
        rng = np.random.default_rng(0)
        words = np.zeros((A, (d + 31) // 32), dtype=np.uint32)
        k = int(np.ceil(d / 3))
        for a in range(A):
            for f in rng.choice(d, k, replace=False):
                words[a, f >> 5] |= np.uint32(1) << np.uint32(f & 31)
        fm = torch.from_numpy(words.view(np.int32)).to(dev)
    y = torch.randn(n, generator=g, device=dev)
    return bins, node, w, y, build, slot_tree, id_tree, fm


def _finish(n, d, T, L, B, masked, g, bins, node, build, slot_tree, id_tree, dev):
    w = K.poisson_weights(T, n, 1, 0, 1.0, device=dev)
    S = len(slot_tree)
    fm = None
    if masked:
        rng = np.random.default_rng(0)
        words = np.zeros((S, (d + 31) // 32), dtype=np.uint32)
        k = int(np.ceil(d / 3))
        for a in range(S):
            for f in rng.choice(d, k, replace=False):
                words[a, f >> 5] |= np.uint32(1) << np.uint32(f & 31)
        fm = torch.from_numpy(words.view(np.int32)).to(dev)
    y = torch.randn(n, generator=g, device=dev)
    return bins, node, w, y, build, slot_tree, id_tree.astype(np.int32), fm


def timeit(fn, reps=3):
    fn()
    torch.cuda.synchronize()
    ts = []
    for _ in range(reps):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        fn()
        b.record()
        torch.cuda.synchronize()
        ts.append(a.elapsed_time(b))
    return min(ts)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=float, default=1e7)
    ap.add_argument("--d", type=int, default=100)
    ap.add_argument("--B", type=int, default=40)
    ap.add_argument("--variants", default="all")
    ap.add_argument("--reps", type=int, default=3)
    args = ap.parse_args()
    n, d, B = int(args.rows), args.d, args.B
    configs = [
        # (name, T, L, masked, weights, version, lane map, lds bytes)
        ("L0 T20 masked w v4", 20, 1, True, True, 4, 2, 65536),
        ("L0 T20 full   w v4 fast", 20, 1, False, True, 4, 5, 65536),
        ("L1 T20 full   w v4 fast", 20, 2, False, True, 4, 5, 65536),
        ("L4 T20 full   w v4 fast", 20, 16, False, True, 4, 5, 65536),
        ("L0 T20 masked w v4 fast", 20, 1, True, True, 4, 5, 65536),
        ("L4 T20 masked w v4 fast", 20, 16, True, True, 4, 5, 65536),
        ("L4 T20 full   w v4 fast 96K", 20, 16, False, True, 4, 5, 98304),
        ("L0 T20 full   w v5 packed", 20, 1, False, True, 5, 4, 65536),
        ("L4 T20 full   w v5 packed", 20, 16, False, True, 5, 4, 65536),
        ("L0 T20 masked w v5 packed", 20, 1, True, True, 5, 4, 65536),
        ("L4 T20 masked w v5 packed", 20, 16, True, True, 5, 4, 65536),
        ("L0 T20 masked w v4 rot", 20, 1, True, True, 4, 4, 65536),
        ("L0 T20 full   w v4 rot", 20, 1, False, True, 4, 4, 65536),
        ("L4 T20 masked w v4 rot", 20, 16, True, True, 4, 4, 65536),
        ("L4 T20 full   w v4 rot", 20, 16, False, True, 4, 4, 65536),
        ("L0 T20 masked w v4 m3", 20, 1, True, True, 4, 3, 65536),
        ("L0 T20 full   w v4", 20, 1, False, True, 4, 2, 65536),
        ("L0 T20 full   w v4 m3", 20, 1, False, True, 4, 3, 65536),
        ("L4 T20 masked w v4", 20, 16, True, True, 4, 2, 65536),
        ("L4 T20 masked w v4 m3", 20, 16, True, True, 4, 3, 65536),
        ("L4 T20 masked w v4 40K", 20, 16, True, True, 4, 2, 40960),
        ("L4 T20 masked w v4 128K", 20, 16, True, True, 4, 2, 131072),
        ("L4 T20 full   w v4", 20, 16, False, True, 4, 2, 65536),
        ("L0 T20 masked w v2", 20, 1, True, True, 2, 2, 65536),
        ("L4 T20 masked w v2", 20, 16, True, True, 2, 2, 65536),
    ]
    if args.variants != "all":
        configs = [c for c in configs if any(v in c[0] for v in args.variants.split(","))]
    sub_cfgs = []
    for lvl in range(5):
        for ver, tag in ((7, "pk8"), (8, "pkq")):
            sub_cfgs.append((f"L{lvl} T20 sub    codes {tag} 128K", 20, 1 << lvl, False, True, ver, 8, 131072))
    sub_cfgs.append(("L4 T20 sub msk codes pk8 128K", 20, 16, True, True, 7, 8, 131072))
    sub_cfgs.append(("L4 T20 sub msk codes pkq 128K", 20, 16, True, True, 8, 8, 131072))
    sub_cfgs.append(("L7 T1  sub    codes pk8 128K B256", 1, 128, False, True, 7, 8, 131072))
    sub_cfgs.append(("L7 T1  sub    codes pkq 128K B256", 1, 128, False, True, 8, 8, 131072))
    configs = sub_cfgs + [("L2 T20 full   codes pk8 128K", 20, 4, False, True, 7, 8, 131072),
               ("L3 T20 full   codes pk8 128K", 20, 8, False, True, 7, 8, 131072),
               ("L1 T20 full   codes pk8 128K", 20, 2, False, True, 7, 8, 131072),
               ("L4 T20 full   codes pk8 128K", 20, 16, False, True, 7, 8, 131072),
               ("L0 T20 full   codes pk8 128K", 20, 1, False, True, 7, 8, 131072),
               ("L4 T20 full   codes pk16 128K", 20, 16, False, True, 7, 16, 131072),
               ("L4 T20 masked codes pk8 128K", 20, 16, True, True, 7, 8, 131072),
               ("L0 T20 full   codes pk4", 20, 1, False, True, 7, 4, 65536),
               ("L4 T20 full   codes pk4", 20, 16, False, True, 7, 4, 65536),
               ("L0 T20 full   codes pk8 48K", 20, 1, False, True, 7, 8, 49152),
               ("L0 T20 full   codes pk8", 20, 1, False, True, 7, 8, 65536),
               ("L0 T20 full   codes pk16", 20, 1, False, True, 7, 16, 65536),
               ("L1 T20 full   codes pk8", 20, 2, False, True, 7, 8, 65536),
               ("L4 T20 full   codes pk8", 20, 16, False, True, 7, 8, 65536),
               ("L4 T20 masked codes pk8", 20, 16, True, True, 7, 8, 65536),
               ("L0 T20 full   codes", 20, 1, False, True, 6, 0, 65536),
               ("L1 T20 full   codes", 20, 2, False, True, 6, 0, 65536),
               ("L4 T20 full   codes", 20, 16, False, True, 6, 0, 65536),
               ("L0 T20 masked codes", 20, 1, True, True, 6, 0, 65536),
               ("L4 T20 masked codes", 20, 16, True, True, 6, 0, 65536)] + configs
    if args.variants != "all":
        configs = [c for c in configs if any(v in c[0] for v in args.variants.split(","))]
    for name, T, L, masked, wts, ver, lmap, lds in configs:
        if ver in (6, 7, 8):
            K.HIST5_PACKED = ver >= 7
            K.HIST5_COMPACT = 2 if ver == 8 else 0
            K.HIST5_PACKED_MAXT = lmap if ver >= 7 else 8
            Bc = 256 if "B256" in name else B
            sub = " sub " in name
            bins, node, w, y, build, st, it, fm = make_state(n, d, T, L, Bc, masked, sub=sub)
            codes = K.codes_init(w, T, n, "cuda")
            loc = node - (torch.arange(T, device="cuda", dtype=torch.int32) * L)[:, None]
            c = codes.to(torch.int32) & 0xFFFF
            loc = torch.where((c & 0xFF) == 0xFF, torch.full_like(loc, 0xFF), loc)
            codes = ((c & 0xFF00) | loc).to(torch.int16).contiguous()
            tfirst = torch.arange(T, dtype=torch.int32) * L
            del node
            wmax = int(w.max().item())
            fn = lambda: K.hist_codes(0, bins, d, codes, tfirst, None, y, None, 0, build, st, it, fm, Bc,  # noqa: E731
                                      lds_budget=lds, wmax=wmax)
            ms = timeit(fn, args.reps)
            frac_w = float((w > 0).float().mean())
            feats = int(np.ceil(d / 3)) if masked else d
            upd = n * T * frac_w * feats * (0.5 if (sub and L > 1) else 1.0)
            print(f"{name:28s} {ms:9.2f} ms  {upd / ms * 1e3:9.3e} upd/s  ({upd:.2e} row-tree-feature updates)",
                  flush=True)
            del bins, codes, w, y
            torch.cuda.empty_cache()
            continue
        bins, node, w, y, build, st, it, fm = make_state(n, d, T, L, B, masked)
        K.HIST_MAP = lmap
        fn = lambda: K.hist_moments(bins, d, node, w if wts else None, None, y, build, st, fm, B,  # noqa: E731
                                    lds_budget=lds, id_tree=it)
        ms = timeit(fn, args.reps)
        frac_w = float((w > 0).float().mean()) if wts else 1.0
        feats = int(np.ceil(d / 3)) if masked else d
        upd = n * T * frac_w * feats
        print(f"{name:28s} {ms:9.2f} ms  {upd / ms * 1e3:9.3e} upd/s  ({upd:.2e} row-tree-feature updates)",
              flush=True)
        del bins, node, w, y
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
