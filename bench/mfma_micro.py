"""A/B of the level-histogram paths on the headline shape (GPU):

  atomic: codes_compact (item records of the built rows) + seg_hist_flat (LDS atomics)
  mfma:   hist_mfma (int8 one-hot GEMM over all rows; planar bins converted once per fit)

for levels with nb built nodes per tree (nb = 1: levels 0-1 of a forest, 2: level 2, ...).
    python bench/mfma_micro.py --rows 1e8 --trees 20 --nb 1 2 4
"""
import argparse
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from cdnaml.ops import kernels as K  # noqa: E402


def timed(fn, reps):
    fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        out = fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / reps * 1e3, out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=float, default=1e8)
    ap.add_argument("--d", type=int, default=100)
    ap.add_argument("--B", type=int, default=40)
    ap.add_argument("--trees", type=int, default=20)
    ap.add_argument("--nb", type=int, nargs="+", default=[1, 2, 4])
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--only", default="", help="atomic | mfma: time one path only (profiling)")
    args = ap.parse_args()
    dev = torch.device("cuda")
    n, d, B, T = int(args.rows), args.d, args.B, args.trees
    g = torch.Generator(device=dev).manual_seed(0)
    X = torch.randn(n, d, generator=g, device=dev)
    q = torch.linspace(0, 1, B + 1, device=dev)[1:-1]
    thr = torch.quantile(X[:100000].float(), q, dim=0).t().contiguous()
    nthr = torch.full((d,), B - 1, dtype=torch.int32, device=dev)
    bins, rm = K.binize(X, thr, nthr, want_rm=True)
    del X
    v1 = torch.randn(n, generator=g, device=dev)
    t_pl, (bp, ldp) = timed(lambda: K.planar_bins(bins), args.reps)
    print(f"planar_bins: {t_pl:.2f} ms")
    sc = K.seg_scales(None, v1, 12, n)
    for nb in args.nb:
        nloc = 2 * nb
        gg = torch.Generator(device=dev).manual_seed(nb)
        w = torch.poisson(torch.ones((T, n), device=dev), generator=gg).clamp(0, 12).to(torch.int32)
        loc = torch.randint(0, nloc, (T, n), generator=gg, device=dev, dtype=torch.int32)
        loc = torch.where(w == 0, torch.full_like(loc, 0xFF), loc)
        codes = ((w << 8) | loc).to(torch.int16)
        del w, loc
        tfirst = np.arange(T, dtype=np.int32) * nloc
        slot_of = np.full(T * nloc, -1, dtype=np.int32)
        built = [t * nloc + k for t in range(T) for k in range(0, nloc, 2)]   # one of each sibling pair
        slot_of[built] = np.arange(len(built))
        S = len(built)

        def atomic():
            rec, _, _, _, sg = K.codes_compact(codes, torch.from_numpy(tfirst), slot_of, S, None, v1,
                                               rec_scale=sc[1])
            sb = np.concatenate([sg, np.arange(S)[:, None]], 1)
            return K.seg_hist(bins, d, B, rec, None, None, None, sb, S, 12, sc, bins_rm=rm, interleave=True,
                              rec=True, raw=True)

        def mfma():
            return K.hist_mfma(bp, ldp, n, d, B, codes, tfirst, slot_of, S, v1, sc[1])

        if args.only:
            t, _ = timed(atomic if args.only == "atomic" else mfma, args.reps)
            print(f"nb={nb} slots={S}: {args.only} {t:.2f} ms", flush=True)
            continue
        ta, ha = timed(atomic, args.reps)
        tm, hm = timed(mfma, args.reps)
        same = bool(torch.equal(ha, hm))
        print(f"nb={nb} slots={S}: atomic {ta:.2f} ms, mfma {tm:.2f} ms, identical={same}", flush=True)
        del codes


if __name__ == "__main__":
    main()
