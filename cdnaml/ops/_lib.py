"""Loader for the in-tree native HIP kernel library (``cdnaml/_native``).

The kernels in ``csrc/kernels/*.hip`` are compiled with ``hipcc
--offload-arch=gfx950`` into ``libcdnaml_hip.so`` and bound through ctypes:
entry points are plain C functions taking raw device pointers plus the
caller's HIP stream, so there is no dependency on the torch C++ ABI and no
hipify step.  The library is built in-tree (it ships to GPU boxes with the
repository snapshot); if it is missing or older than its sources it is
rebuilt on first use.

On a machine with a visible GPU, a failure to build or load the library is
an error — GPU code paths never silently fall back to eager PyTorch.
"""
from __future__ import annotations

import ctypes
import glob
import os
import subprocess
import threading
from ctypes import c_double, c_float, c_int, c_int64, c_uint32, c_uint64, c_void_p

_ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
_SRC_DIR = os.path.join(_ROOT, "csrc", "kernels")
_OUT_DIR = os.path.join(_ROOT, "cdnaml", "_native")
# CDNAML_HIP_DEBUG=1: the checked build (-O1 -g -DCDNA_DEBUG: device bounds checks in the record histogram,
# partition and predict kernels, read back after every call) in its own file next to the release library
DEBUG = os.environ.get("CDNAML_HIP_DEBUG", "0") not in ("", "0")
LIB_PATH = os.path.join(_OUT_DIR, "libcdnaml_hip_debug.so" if DEBUG else "libcdnaml_hip.so")
ARCH = os.environ.get("CDNAML_OFFLOAD_ARCH", "gfx950")
_DEBUG_UNITS = ("seg", "hist5", "trees", "hashagg", "relational")

_lock = threading.Lock()
_lib = None
_load_error = None


def _sources():
    return sorted(glob.glob(os.path.join(_SRC_DIR, "*.hip")) + glob.glob(os.path.join(_SRC_DIR, "*.h")))


def _path(debug: bool) -> str:
    return os.path.join(_OUT_DIR, "libcdnaml_hip_debug.so" if debug else "libcdnaml_hip.so")


def _stale(path: str = LIB_PATH) -> bool:
    if not os.path.exists(path):
        return True
    t = os.path.getmtime(path)
    return any(os.path.getmtime(s) > t for s in _sources())


def build(force: bool = False, verbose: bool = False, debug: bool = DEBUG) -> str:
    """Compile the HIP kernel library for gfx950 (in-tree); ``debug``: the checked build."""
    LIB_PATH = _path(debug)
    if not force and not _stale(LIB_PATH):
        return LIB_PATH
    os.makedirs(_OUT_DIR, exist_ok=True)
    hipcc = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
    srcs = sorted(glob.glob(os.path.join(_SRC_DIR, "*.hip")))
    tmp = LIB_PATH + f".tmp{os.getpid()}"
    objdir = os.path.join(_OUT_DIR, f".obj{os.getpid()}{'d' if debug else ''}")
    os.makedirs(objdir, exist_ok=True)
    flags = [f"--offload-arch={ARCH}", "-O1" if debug else "-O3", "-std=c++17", "-fPIC"] + \
        (["-g", "-DCDNA_DEBUG"] if debug else [])

    def compile_one(src):
        obj = os.path.join(objdir, os.path.basename(src) + ".o")
        cmd = [hipcc] + flags + ["-c", src, "-o", obj]
        if verbose:
            print(" ".join(cmd), flush=True)
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f"hipcc failed on {src}:\n{r.stderr[-4000:]}")
        return obj

    # one translation unit per kernel file, compiled in parallel, then one link
    from concurrent.futures import ThreadPoolExecutor
    jobs = max(1, min(len(srcs), int(os.environ.get("MAX_JOBS", os.cpu_count() or 4)), 16))
    try:
        with ThreadPoolExecutor(jobs) as ex:
            objs = list(ex.map(compile_one, srcs))
        cmd = [hipcc] + flags + ["-shared", "-o", tmp] + objs
        if verbose:
            print(" ".join(cmd), flush=True)
        res = subprocess.run(cmd, capture_output=True, text=True)
        if res.returncode != 0:
            raise RuntimeError(f"hipcc link failed building {LIB_PATH}:\n{res.stderr[-4000:]}")
    finally:
        for f in glob.glob(os.path.join(objdir, "*")):
            os.remove(f)
        os.rmdir(objdir)
    os.replace(tmp, LIB_PATH)
    return LIB_PATH


_SIGS = {
    # name: (argtypes, restype)
    "cdna_gram_workspace": ([c_int64, c_int, c_int], c_int64),
    "cdna_quantile_thresholds": ([c_void_p, c_int, c_int, c_int, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p,
                                  c_void_p],
                                 c_int),
    "cdna_gram": ([c_void_p, c_int64, c_int, c_int64, c_void_p, c_void_p, c_float, c_void_p, c_void_p, c_int,
                   c_void_p], c_int),
    "cdna_binize": ([c_void_p, c_int64, c_int, c_int64, c_void_p, c_void_p, c_int, c_int, c_float, c_void_p, c_void_p,
                     c_int, c_int64, c_int, c_int, c_void_p],
                    c_int),
    "cdna_hist4": ([c_int, c_void_p, c_int64, c_int, c_int, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_int,
                    c_void_p, c_void_p, c_int, c_int, c_int, c_int, c_void_p, c_int, c_int, c_int, c_float, c_float,
                    c_void_p, c_void_p], c_int),
    "cdna_hist4_bytes_per_bin": ([c_int, c_int], c_int),
    "cdna_hist5": ([c_int, c_void_p, c_int64, c_int, c_int, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_int,
                    c_void_p, c_void_p, c_int, c_int, c_int, c_int, c_void_p, c_int, c_int, c_int, c_float, c_float,
                    c_int, c_void_p, c_void_p], c_int),
    "cdna_hist5_max_trees": ([], c_int),
    "cdna_seg_hist": ([c_int, c_void_p, c_int64, c_int, c_int, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p,
                       c_int, c_float, c_float, c_void_p, c_int, c_void_p], c_int),
    "cdna_seg_hist_root_wide": ([c_void_p, c_int64, c_int, c_int, c_int, c_void_p, c_void_p, c_float, c_void_p, c_int,
                                 c_void_p, c_int, c_void_p, c_int, c_void_p], c_int),
    "cdna_seg_hist_root": ([c_void_p, c_int64, c_int, c_int, c_void_p, c_void_p, c_float, c_void_p, c_int, c_void_p,
                            c_int, c_void_p, c_int, c_uint64, c_uint64, c_double, c_int, c_void_p], c_int),
    "cdna_poisson_max_draw": ([c_double], c_int),
    "cdna_seg_partition": ([c_int, c_void_p, c_int64, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_int,
                            c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p,
                            c_void_p, c_void_p, c_int64, c_void_p, c_void_p], c_int),
    "cdna_codes_compact": ([c_int, c_void_p, c_int64, c_int, c_int, c_void_p, c_void_p, c_void_p, c_void_p,
                            c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_float, c_void_p], c_int),
    "cdna_bins_row_major": ([c_void_p, c_int64, c_int, c_int, c_void_p, c_void_p], c_int),
    "cdna_expr_eval": ([c_void_p, c_int, c_void_p, c_int, c_void_p, c_void_p, c_void_p, c_int64, c_void_p, c_int,
                        c_void_p, c_void_p], c_int),
    "cdna_partition7": ([c_void_p, c_int64, c_int, c_int, c_int, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p,
                         c_void_p, c_void_p, c_void_p, c_void_p], c_int),
    "cdna_split_decode": ([c_void_p, c_int, c_void_p, c_int, c_void_p, c_int, c_int, c_double, c_double, c_int, c_int,
                           c_int, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p,
                           c_int, c_double, c_void_p, c_void_p, c_void_p], c_int),
    "cdna_split_scan_ex": ([c_void_p, c_void_p, c_void_p, c_int, c_int, c_int, c_int, c_int, c_int, c_double, c_void_p,
                            c_void_p, c_void_p, c_void_p], c_int),
    "cdna_split_scan": ([c_void_p, c_void_p, c_void_p, c_int, c_int, c_int, c_int, c_int, c_int, c_double, c_double,
                         c_double, c_double, c_void_p, c_void_p, c_void_p], c_int),
    "cdna_compact_mask": ([c_int, c_void_p, c_int64, c_int64, c_void_p, c_void_p, c_void_p, c_void_p], c_int),
    "cdna_col_moments": ([c_int, c_void_p, c_int64, c_int, c_int64, c_void_p, c_int64, c_int64, c_void_p, c_void_p],
                         c_int),
    "cdna_partition_dest": ([c_int, c_void_p, c_int64, c_int, c_int64, c_void_p, c_void_p, c_void_p, c_void_p],
                            c_int),
    "cdna_codes_compact_w": ([c_int, c_int, c_void_p, c_int64, c_int, c_int, c_void_p, c_void_p, c_void_p, c_void_p,
                              c_int64, c_int, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p,
                              c_float, c_void_p, c_int, c_void_p], c_int),
    "cdna_wave_scan": ([c_void_p, c_int, c_int, c_int, c_void_p, c_void_p], c_int),
    "cdna_hash_insert": ([c_void_p, c_int64, c_void_p, c_int64, c_void_p, c_int, c_void_p, c_void_p], c_int),
    "cdna_hash_lookup": ([c_void_p, c_int64, c_void_p, c_int64, c_int, c_void_p, c_void_p], c_int),
    "cdna_dict_encode": ([c_void_p, c_void_p, c_void_p, c_int64, c_void_p, c_int64, c_void_p, c_int, c_void_p,
                          c_void_p], c_int),
    "cdna_pack_keys": ([c_int, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_int64, c_void_p, c_void_p], c_int),
    "cdna_hp_hist": ([c_void_p, c_int64, c_int, c_int64, c_void_p, c_void_p], c_int),
    "cdna_hp_part": ([c_int, c_int64, c_int, c_int, c_int64, c_int, c_int, c_int, c_int, c_void_p, c_void_p, c_void_p,
                      c_int, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p,
                      c_void_p], c_int),
    "cdna_hp_agg_lds_bytes": ([c_int, c_int], c_int),
    "cdna_hp_agg_lds_budget": ([], c_int),
    "cdna_hp_agg": ([c_void_p, c_void_p, c_void_p, c_int64, c_void_p, c_int, c_int, c_int, c_int, c_int, c_void_p,
                     c_void_p, c_int, c_int, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p,
                     c_void_p], c_int),
    "cdna_la_groups": ([c_void_p, c_int64, c_int64, c_int, c_int, c_int, c_void_p, c_void_p, c_int, c_void_p, c_void_p,
                        c_void_p, c_int, c_int, c_void_p, c_void_p, c_void_p, c_void_p, c_int64, c_void_p, c_void_p,
                        c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p], c_int),
    "cdna_bucket_compact": ([c_int, c_void_p, c_int64, c_int, c_int64, c_void_p, c_void_p, c_void_p, c_void_p], c_int),
    "cdna_gather": ([c_void_p, c_int64, c_int64, c_int, c_void_p, c_void_p, c_void_p, c_void_p], c_int),
    "cdna_join_build_dense": ([c_void_p, c_void_p, c_int64, c_int64, c_int64, c_void_p, c_void_p, c_void_p, c_void_p],
                              c_int),
    "cdna_join_probe_dense": ([c_void_p, c_void_p, c_int64, c_int64, c_int64, c_void_p, c_void_p, c_void_p, c_void_p,
                              c_void_p, c_void_p, c_void_p], c_int),
    "cdna_join_build": ([c_void_p, c_void_p, c_int64, c_void_p, c_int64, c_void_p, c_void_p, c_void_p, c_void_p],
                        c_int),
    "cdna_join_probe": ([c_void_p, c_void_p, c_int64, c_void_p, c_int64, c_void_p, c_void_p, c_void_p, c_void_p,
                         c_void_p, c_void_p], c_int),
    "cdna_grouped_reduce": ([c_int, c_void_p, c_void_p, c_int64, c_int, c_int64, c_void_p, c_void_p], c_int),
    "cdna_als_max_rank": ([], c_int),
    "cdna_als_accumulate": ([c_int, c_void_p, c_void_p, c_void_p, c_void_p, c_int, c_int, c_double, c_void_p,
                             c_void_p, c_void_p, c_void_p], c_int),
    "cdna_als_solve": ([c_int, c_int, c_void_p, c_void_p, c_void_p, c_void_p, c_int, c_int, c_void_p, c_void_p,
                        c_void_p], c_int),
    "cdna_codes_init": ([c_void_p, c_int64, c_void_p, c_void_p, c_void_p], c_int),
    "cdna_partition5": ([c_void_p, c_int64, c_int, c_int, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p,
                         c_void_p, c_void_p, c_void_p, c_int, c_void_p, c_float, c_void_p, c_void_p], c_int),
    "cdna_partition": ([c_void_p, c_int64, c_int, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p,
                        c_void_p], c_int),
    "cdna_tree_predict": ([c_void_p, c_int64, c_int, c_int64, c_void_p, c_int64, c_void_p, c_void_p, c_int, c_void_p,
                           c_void_p, c_int, c_void_p, c_void_p, c_int64, c_void_p], c_int),
    "cdna_heap_last_level": ([c_void_p, c_int, c_int, c_void_p, c_void_p, c_void_p, c_void_p, c_int, c_int, c_double,
                              c_double, c_void_p, c_int, c_int, c_void_p], c_int),
    "cdna_tree_predict_heap": ([c_void_p, c_int64, c_int, c_int64, c_void_p, c_int, c_void_p, c_int, c_void_p,
                                c_double, c_void_p, c_void_p, c_int, c_void_p], c_int),
    "cdna_sample_gather": ([c_void_p, c_int64, c_int64, c_int, c_uint64, c_uint64, c_uint32, c_double, c_void_p,
                            c_void_p, c_int64, c_void_p, c_void_p], c_int),
    "cdna_fill_chunk": ([c_void_p, c_int, c_int64, c_int, c_int, c_int64], c_int64),
    "cdna_seg_work": ([c_void_p, c_int, c_int64, c_int, c_void_p, c_int64], c_int64),
    "cdna_tree_predict_heap_binned": ([c_void_p, c_int64, c_int, c_int, c_void_p, c_int, c_void_p, c_int, c_void_p,
                                       c_int, c_double, c_void_p, c_void_p, c_void_p, c_void_p], c_int),
    "cdna_predict_binned_add": ([c_void_p, c_int64, c_void_p, c_int, c_void_p, c_void_p, c_float, c_void_p,
                                 c_void_p], c_int),
    "cdna_node_compact": ([c_int, c_void_p, c_void_p, c_int64, c_int, c_int, c_void_p, c_void_p, c_void_p, c_void_p,
                           c_void_p, c_float, c_int, c_void_p], c_int),
    "cdna_feature_masks": ([c_void_p, c_int, c_int, c_int, c_void_p, c_void_p], c_int),
    "cdna_codes_to_nodes": ([c_void_p, c_int64, c_int, c_void_p, c_void_p, c_void_p, c_void_p], c_int),
    "cdna_uniform": ([c_void_p, c_int64, c_uint64, c_uint64, c_uint32, c_void_p], c_int),
    "cdna_sample_rows": ([c_int64, c_uint64, c_uint64, c_uint32, c_double, c_void_p, c_int64, c_void_p, c_void_p],
                         c_int),
    "cdna_cast_absmax": ([c_void_p, c_int64, c_void_p, c_void_p, c_void_p, c_void_p], c_int),
    "cdna_normal_f32": ([c_void_p, c_int64, c_uint64, c_uint64, c_uint32, c_void_p], c_int),
    "cdna_poisson": ([c_void_p, c_int, c_int64, c_uint64, c_uint64, c_double, c_void_p, c_void_p, c_int, c_void_p],
                     c_int),
    "cdna_reg_metrics": ([c_void_p, c_void_p, c_void_p, c_int64, c_void_p, c_void_p, c_void_p], c_int),
    "cdna_score_hist": ([c_void_p, c_void_p, c_int64, c_double, c_double, c_int, c_void_p, c_void_p], c_int),
    "cdna_kmeans_step": ([c_void_p, c_int64, c_int, c_int64, c_void_p, c_int, c_void_p, c_void_p, c_void_p,
                          c_void_p, c_int, c_void_p], c_int),
    "cdna_hist_assemble": ([c_void_p, c_int, c_double, c_double, c_void_p, c_void_p, c_int, c_int64, c_int,
                            c_void_p, c_void_p], c_int),
    "cdna_grad_hess": ([c_void_p, c_void_p, c_void_p, c_int64, c_int, c_int, c_void_p, c_void_p, c_void_p,
                        c_void_p], c_int),
    "cdna_logistic_grad": ([c_void_p, c_int64, c_int, c_int64, c_void_p, c_void_p, c_void_p, c_double, c_void_p,
                            c_void_p, c_int, c_void_p], c_int),
}


def lib():
    """Return the loaded ctypes library (building it if needed)."""
    global _lib, _load_error
    if _lib is not None:
        return _lib
    with _lock:
        if _lib is not None:
            return _lib
        try:
            build()
            L = ctypes.CDLL(LIB_PATH)
            for name, (args, res) in _SIGS.items():
                fn = getattr(L, name)
                fn.argtypes = args
                fn.restype = res
            for u in _DEBUG_UNITS:
                getattr(L, f"cdna_debug_status_{u}").restype = c_uint32
            _lib = L
        except Exception as e:  # pragma: no cover - exercised on GPU boxes
            _load_error = e
            raise
    return _lib


def available() -> bool:
    try:
        lib()
        return True
    except Exception:
        return False


def check(code: int, name: str):
    if code != 0:
        raise RuntimeError(f"native kernel {name} failed with hipError {code}")
    if DEBUG:
        import torch
        if torch.cuda.is_available() and torch.cuda.is_current_stream_capturing():
            return  # the status read synchronises the device: not allowed inside a HIP graph capture
        for u in _DEBUG_UNITS:
            v = int(getattr(_lib, f"cdna_debug_status_{u}")())
            if v:
                raise RuntimeError(f"checked build: device bounds check 0x{v:04X} failed in {u}.hip "
                                   f"(after {name})")
