"""Tracing / profiling: scoped timers on HIP events, per-op stats and
Chrome-trace export, plus collective byte counters.

    from cdnaml.utils import tracing
    tracing.enable()                      # or CDNAML_TRACE=1
    ... fit ...
    print(tracing.summary())              # table: op, calls, total ms, mean ms
    tracing.export_chrome_trace("trace.json")   # chrome://tracing / Perfetto

Spans are recorded with ``torch.cuda.Event`` pairs on the current HIP stream
(no device sync inside the span; timings resolve lazily at summary/export),
or ``perf_counter`` on CPU.  Each rank writes its own ``pid`` so multi-GPU
traces can be merged.  When disabled, ``span`` costs one attribute lookup.
"""
from __future__ import annotations

import contextlib
import json
import os
import threading
import time
from collections import defaultdict
from typing import Dict, List, Optional

import torch

_state = {"enabled": os.environ.get("CDNAML_TRACE", "0") not in ("0", "", "false"), "events": [],
          "lock": threading.Lock(), "t0": time.perf_counter()}

# roctx ranges: every span is also pushed as a ROCTx range, so `rocprofv3 --marker-trace` lines
# the engine's phases (tree.hist, tree.allreduce, ...) up with the kernels.  CDNAML_ROCTX=1 turns ranges on
# even when span timing is off; libroctx64 is loaded lazily (absent library: ranges are a no-op).
_roctx = {"lib": None, "tried": False, "on": os.environ.get("CDNAML_ROCTX", "0") not in ("0", "", "false")}


def _roctx_lib():
    if not _roctx["tried"]:
        _roctx["tried"] = True
        import ctypes
        for path in ("libroctx64.so", "/opt/rocm/lib/libroctx64.so"):
            try:
                lib = ctypes.CDLL(path)
                lib.roctxRangePushA.argtypes = [ctypes.c_char_p]
                lib.roctxRangePushA.restype = ctypes.c_int
                lib.roctxRangePop.restype = ctypes.c_int
                _roctx["lib"] = lib
                break
            except OSError:
                continue
    return _roctx["lib"]


def enable_roctx(on: bool = True) -> bool:
    """Emit ROCTx ranges for spans; returns whether libroctx64 is available."""
    _roctx["on"] = on
    return _roctx_lib() is not None


def enable(on: bool = True):
    _state["enabled"] = on


def disable():
    _state["enabled"] = False


def is_enabled() -> bool:
    return _state["enabled"]


def reset():
    with _state["lock"]:
        _state["events"] = []
        _state["t0"] = time.perf_counter()


def _rank() -> int:
    try:
        from ..session import SparkSession
        s = SparkSession.getActiveSession()
        return s.comm.rank if s is not None else 0
    except Exception:  # noqa: BLE001
        return 0


class _Span:
    __slots__ = ("name", "cat", "args", "t_host0", "t_host1", "ev0", "ev1", "tid", "rank")

    def duration_ms(self) -> float:
        if self.ev0 is not None:
            self.ev1.synchronize()
            return float(self.ev0.elapsed_time(self.ev1))
        return (self.t_host1 - self.t_host0) * 1e3


@contextlib.contextmanager
def span(name: str, cat: str = "op", device: Optional[torch.device] = None, **args):
    """Time a region.  On a GPU the region is bracketed by HIP events on the current stream."""
    rx = _roctx_lib() if _roctx["on"] else None
    if rx is not None:
        rx.roctxRangePushA(name.encode())
    if not _state["enabled"]:
        try:
            yield
        finally:
            if rx is not None:
                rx.roctxRangePop()
        return
    s = _Span()
    s.name, s.cat, s.args = name, cat, args
    s.tid = threading.get_ident() & 0xFFFF
    s.rank = _rank()
    use_cuda = torch.cuda.is_available() and (device is None or getattr(device, "type", "cuda") == "cuda")
    s.ev0 = s.ev1 = None
    if use_cuda:
        s.ev0 = torch.cuda.Event(enable_timing=True)
        s.ev1 = torch.cuda.Event(enable_timing=True)
        s.ev0.record()
    s.t_host0 = time.perf_counter()
    try:
        yield
    finally:
        if use_cuda:
            s.ev1.record()
        s.t_host1 = time.perf_counter()
        if rx is not None:
            rx.roctxRangePop()
        with _state["lock"]:
            _state["events"].append(s)


def begin(name: str, cat: str = "op", **args) -> Optional[_Span]:
    """Open a span that :func:`end` closes later -- an interval that does not nest in one ``with`` block (an async
    collective from issue to wait, while other spans run).  None when tracing is off."""
    if not _state["enabled"]:
        return None
    s = _Span()
    s.name, s.cat, s.args = name, cat, args
    s.tid = (threading.get_ident() & 0xFFFF) + 1   # its own track: it overlaps the spans of this thread
    s.rank = _rank()
    s.ev0 = s.ev1 = None
    if torch.cuda.is_available():
        s.ev0 = torch.cuda.Event(enable_timing=True)
        s.ev1 = torch.cuda.Event(enable_timing=True)
        s.ev0.record()
    s.t_host0 = time.perf_counter()
    return s


def end(s: Optional[_Span]) -> None:
    if s is None:
        return
    if s.ev1 is not None:
        s.ev1.record()
    s.t_host1 = time.perf_counter()
    with _state["lock"]:
        _state["events"].append(s)


def traced(name: Optional[str] = None, cat: str = "op"):
    """Decorator form of :func:`span`."""
    def deco(fn):
        label = name or fn.__qualname__

        def wrapper(*a, **k):
            with span(label, cat):
                return fn(*a, **k)
        wrapper.__wrapped__ = fn
        wrapper.__name__ = fn.__name__
        wrapper.__doc__ = fn.__doc__
        return wrapper
    return deco


def stats() -> Dict[str, Dict[str, float]]:
    out: Dict[str, Dict[str, float]] = defaultdict(lambda: {"calls": 0, "total_ms": 0.0, "max_ms": 0.0,
                                                             "bytes": 0.0})
    for s in list(_state["events"]):
        d = s.duration_ms()
        o = out[s.name]
        o["calls"] += 1
        o["total_ms"] += d
        o["max_ms"] = max(o["max_ms"], d)
        if s.cat == "comm" and "bytes" in s.args:
            o["bytes"] += float(s.args["bytes"])
    for o in out.values():
        o["mean_ms"] = o["total_ms"] / max(o["calls"], 1)
        # collectives: achieved bus-agnostic rate (payload bytes / span time)
        o["GB_s"] = o["bytes"] / (o["total_ms"] * 1e6) if o["bytes"] and o["total_ms"] > 0 else 0.0
    return dict(out)


def summary(sort: str = "total_ms") -> str:
    st = stats()
    rows = sorted(st.items(), key=lambda kv: -kv[1][sort])
    lines = [f"{'op':40s} {'calls':>7s} {'total ms':>11s} {'mean ms':>10s} {'max ms':>10s} {'GB/s':>8s}"]
    for k, v in rows:
        gbs = f"{v['GB_s']:8.1f}" if v.get("GB_s") else f"{'':8s}"
        lines.append(f"{k[:40]:40s} {v['calls']:7d} {v['total_ms']:11.2f} {v['mean_ms']:10.3f} {v['max_ms']:10.3f} "
                     f"{gbs}")
    try:
        from ..session import SparkSession
        s = SparkSession.getActiveSession()
        if s is not None and s.comm.distributed:
            lines.append(f"collectives: {s.comm.calls} calls, {s.comm.bytes_reduced / 1e6:.1f} MB")
    except Exception:  # noqa: BLE001
        pass
    return "\n".join(lines)


def export_chrome_trace(path: str) -> str:
    """Write a Chrome trace-event JSON (one ``X`` event per span)."""
    evs: List[dict] = []
    t0 = _state["t0"]
    for s in list(_state["events"]):
        dur = s.duration_ms() * 1e3
        evs.append({"name": s.name, "cat": s.cat, "ph": "X", "pid": s.rank, "tid": s.tid,
                    "ts": (s.t_host0 - t0) * 1e6, "dur": dur, "args": {k: str(v) for k, v in s.args.items()}})
    with open(path, "w") as f:
        json.dump({"traceEvents": evs, "displayTimeUnit": "ms"}, f)
    return path
