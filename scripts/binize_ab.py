"""A/B of the K4 binize variants at the headline shape (1e8 x 100 fp32, 40 bins, row-major copy).

Each variant runs in its own process (the kernel selectors read their environment once):
    python scripts/binize_ab.py            # parent: runs every variant, prints one line each
"""
import os
import subprocess
import sys

VARIANTS = {
    "v2": {"CDNAML_BINIZE_V5": "0"},
    "v5": {},
    "v5_seg10": {"AB_S10": "1"},
}
# round 3 A/B (1x MI355X, 1e8 x 100 fp32, 40 bins): v5 16.02 ms, v5 + seg10 rows 16.72 ms; a third register set
# (two tiles of loads in flight) 16.33 / 17.04 ms; non-temporal X loads 31.2 ms (2x slower) -- both dropped,
    "v5_3sets": {"CDNAML_BINIZE_VAR": "1"},
    "v5_nt": {"CDNAML_BINIZE_VAR": "2"},
    "v5_3sets_nt": {"CDNAML_BINIZE_VAR": "3"},
    "v5_seg10": {"AB_S10": "1"},
    "v5_seg10_3sets": {"AB_S10": "1", "CDNAML_BINIZE_VAR": "1"},
    "v5_seg10_nt": {"AB_S10": "1", "CDNAML_BINIZE_VAR": "2"},
}


def child() -> None:
    import torch
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    from cdnaml.ops import kernels as K
    dev = torch.device("cuda:0")
    n, d, nb = 100_000_000, 100, 40
    g = torch.Generator(device=dev).manual_seed(0)
    X = torch.randn((n, d), generator=g, device=dev)
    q = torch.linspace(0, 1, nb + 1, device=dev)[1:-1]
    thr = torch.quantile(X[:1_000_000].T.contiguous(), q, dim=1).T.contiguous()  # [d, nb - 1]
    nthr = torch.full((d,), nb - 1, dtype=torch.int32, device=dev)
    ref = None
    for _ in range(2):
        b, rm = K.binize(X, thr, nthr, want_rm=True, rm_layout="s10" if os.environ.get("AB_S10") else "std")
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(5):
        b, rm = K.binize(X, thr, nthr, want_rm=True, rm_layout="s10" if os.environ.get("AB_S10") else "std")
    e.record()
    torch.cuda.synchronize()
    ms = s.elapsed_time(e) / 5
    ref = K.binize(X[:200_000].cpu(), thr.cpu(), nthr.cpu())
    ok = torch.equal(b[:, :200_000].cpu(), ref) and rm is not None
    print(f"{os.environ.get('AB_NAME')}: {ms:.2f} ms  ({(n * d * 4 + n * 128 + n * 104) / ms / 1e9:.2f} TB/s)  "
          f"exact={ok}", flush=True)


if __name__ == "__main__":
    if os.environ.get("AB_NAME"):
        child()
    else:
        rc = 0
        for name, env in VARIANTS.items():
            r = subprocess.run([sys.executable, os.path.abspath(__file__)], env={**os.environ, **env, "AB_NAME": name},
                               timeout=300)
            rc = rc or r.returncode
        sys.exit(rc)
