"""Batch inference engine (ML 12 - Inference with Pandas UDFs.py:73-143,
Labs/ML 12L - Pandas UDF Lab.py:78-96, ML 09 - AutoML.py:78-82).

Three pieces, used by ``Model.transform``, ``tracking.pyfunc.spark_udf`` and the spark-flavour pyfunc:

``ForestPredictor``
    A fitted forest uploaded to the device once per process and device: heap-layout trees, tree weights,
    categorical masks.  The model is "broadcast" once, not per batch.  A predict call on a device buffer
    that recurs (the staging buffers of a chunked source, a UDF's fixed-size batch) is captured once in a
    HIP graph and replayed afterwards.  One-off buffers launch the kernel directly, since capturing them
    would cost more than it saves.

``SparkSession.createDataFrameFromChunks``
    A streamed DataFrame over host chunks, for inputs larger than HBM (1e9 x 100 fp32 is 400 GB).  Chunks go
    through two pinned staging buffers and a side copy stream into two device buffers.  The H2D copy of
    chunk i + 1 overlaps the compute on chunk i.  A device buffer is refilled only after the compute stream
    has passed the work enqueued on its previous chunk (HIP events).  Narrow plans (``transform``, ``select``)
    run chunk by chunk through ``Plan.iter_execute``; ``foreachBatch`` / ``count`` consume them.

``device_chunks``
    The same streaming contract for chunks generated on the device (synthetic benchmark data keyed by global
    row id: distinct rows, nothing resident beyond the two buffers).
"""
from __future__ import annotations

import os
import threading
from collections import OrderedDict
from typing import Callable, Dict, Iterable, Iterator, Optional

import numpy as np
import torch

GRAPH_PREDICT = os.environ.get("CDNAML_GRAPH_PREDICT", "1") != "0"
GRAPH_MIN_ROWS = 1024


class ForestPredictor:
    """Device-resident forest with graph-captured predict per recurring input buffer (see module doc)."""

    def __init__(self, forest, tree_w, base=None, values_kind: str = "value", device=None):
        self.forest = forest
        self.kind = values_kind
        self.device = torch.device(device) if device is not None else None
        self.tw_host = np.asarray(tree_w, np.float64)
        self.base = base
        self._dev: Dict[str, tuple] = {}
        self._graphs: "OrderedDict[tuple, tuple]" = OrderedDict()
        self._lock = threading.Lock()
        self._seen: Dict[tuple, int] = {}
        self.replays = 0
        self.captures = 0
        self.binned = 0   # calls served from the training tensor's bins (forest.FitBins)

    def _arrays(self, dev):
        key = str(dev)
        if key not in self._dev:
            from ..ops import kernels as K
            f = self.forest
            base_np = np.asarray(0.0 if self.base is None else self.base, np.float64).reshape(-1)
            pre = getattr(f, "_heap_np", None)
            hkey = ("heap", str(dev), self.kind)
            if (dev.type == "cuda" and f.K == 1 and self.kind == "value" and pre is not None and hkey not in f._dev
                    and pre[0].shape[0] == len(f.roots)):
                # the trainer-built heap table rides the same pinned staging block and copy as the tree weights
                tw, bb, h_t, m_t = K.upload(dev, self.tw_host.reshape(-1), base_np, K.pack_heap(*pre),
                                            np.zeros(8, np.int32))
                f._dev[hkey] = (h_t, pre[2], m_t)
            else:
                # async pinned uploads: a pageable torch.tensor(..., device=) copy waits for the queue to drain
                tw, bb = K.upload(dev, self.tw_host.reshape(-1), base_np)
            heap = f.heap_arrays(dev, self.kind) if (dev.type == "cuda" and f.K == 1) else None
            b = None if self.base is None else bb
            self._dev[key] = (tw, heap, b)
        return self._dev[key]

    def _launch(self, X: torch.Tensor, dtype=torch.float64) -> torch.Tensor:
        from ..ops import kernels as K
        tw, heap, b = self._arrays(X.device)
        if heap is not None:
            b0 = 0.0 if self.base is None else float(np.asarray(self.base, np.float64).reshape(-1)[0])
            out = K.tree_predict_heap(X, heap[0], heap[1], tw, heap[2], b0, dtype=dtype)
            if out is not None:
                self.forest.settle()  # the trainer's deferred node lists, while the GPU predicts
                return out
        nodes, roots, vals, masks = self.forest.device_arrays(X.device, self.kind)
        return K.tree_predict(X, nodes, roots, tw, vals, masks, self.forest.K, b).to(dtype)

    def _launch_binned(self, X: torch.Tensor, dtype) -> Optional[torch.Tensor]:
        """The forest's training tensor itself (forest.FitBins): predict from the fit's uint8 bins -- the same
        branches and fp64 sums as the fp32 path (K.tree_predict_heap_binned), a quarter of the bytes."""
        fb = getattr(self.forest, "_fit_bins", None)
        if fb is None or self.kind != "value" or not X.is_cuda or not fb.matches(X):
            return None
        from ..ops import kernels as K
        tw, heap, _ = self._arrays(X.device)
        if heap is None:
            return None
        got = fb.take(X)  # one transform per fit: the bins' memory goes back to the next fit
        if got is None:
            return None
        bins, thr_up = got
        b0 = 0.0 if self.base is None else float(np.asarray(self.base, np.float64).reshape(-1)[0])
        out = K.tree_predict_heap_binned(bins, thr_up, fb.d, heap[0], heap[1], tw, b0, dtype=dtype)
        if out is not None:
            self.binned += 1
            self.forest.settle()  # the trainer's deferred node lists, while the GPU predicts
        return out

    def __call__(self, X: torch.Tensor, dtype=torch.float64) -> torch.Tensor:
        """[n, d] features -> [n, K] predictions (a fresh tensor the caller owns): fp64 leaf values, weights and
        sums in one fixed tree order (K.ordered_tree_sum), stored as ``dtype``."""
        out = self._launch_binned(X, dtype)  # one launch: never graph-captured (a replay cannot re-check X)
        if out is not None:
            return out
        if not (GRAPH_PREDICT and X.is_cuda and X.shape[0] >= GRAPH_MIN_ROWS and X.is_contiguous()):
            return self._launch(X, dtype)
        if threading.current_thread() is not threading.main_thread():
            # worker threads (applyInPandas pools, GPUTrials, GroupedModel) may allocate or synchronise while
            # another thread captures: graphs are captured and replayed from the main thread only
            return self._launch(X, dtype)
        key = (X.data_ptr(), tuple(X.shape), X.dtype, X.device.index, dtype)
        with self._lock:
            return self._graph_call(X, key, dtype)

    def _graph_call(self, X: torch.Tensor, key, dtype=torch.float64) -> torch.Tensor:
        g = self._graphs.get(key)
        if g is None:
            # capture on the second sighting of a buffer: staging buffers recur, one-off tensors do not
            self._seen[key] = self._seen.get(key, 0) + 1
            if self._seen[key] < 2:
                return self._launch(X, dtype)
            self._arrays(X.device)
            s = torch.cuda.Stream(device=X.device)
            s.wait_stream(torch.cuda.current_stream(X.device))
            with torch.cuda.stream(s):
                self._launch(X, dtype)  # warm-up outside capture (allocator, LDS attributes)
            torch.cuda.current_stream(X.device).wait_stream(s)
            graph = torch.cuda.CUDAGraph()
            with torch.cuda.graph(graph, capture_error_mode="thread_local"):
                out = self._launch(X, dtype)
            g = (graph, out)
            self._graphs[key] = g
            self.captures += 1
            while len(self._graphs) > 8:
                self._graphs.popitem(last=False)
        graph, out = g
        graph.replay()
        self.replays += 1
        return out.clone()  # the graph's output buffer is rewritten by its next replay


def predictor_for(model, values_kind: str = "value", base=None) -> ForestPredictor:
    """The model's cached ForestPredictor (created on first use; dropped when the forest changes)."""
    p = getattr(model, "_predictor_cache", None)
    if p is None or p.forest is not model._forest or p.kind != values_kind:
        p = ForestPredictor(model._forest, model._tree_w, base, values_kind)
        model._predictor_cache = p
    return p


# --------------------------------------------------------------------------- chunked sources
def _schema_of(arrays: dict):
    from ..sql import types as T
    fields = []
    for k, a in arrays.items():
        a = torch.as_tensor(a) if not isinstance(a, torch.Tensor) else a
        dt = T.VectorUDT() if a.dim() == 2 else T.from_torch(a.dtype)
        fields.append(T.StructField(k, dt, True))
    return T.StructType(fields)


class HostChunkStream:
    """Host chunks -> device batches through pinned double buffers and a copy stream (see module doc).

    ``chunks``: a callable returning an iterator of ``{column: numpy array | cpu tensor}`` (chunks of at
    most ``max_rows`` rows, columns [n] or [n, d]); called again for every pass over the DataFrame."""

    def __init__(self, session, chunks: Callable[[], Iterable[dict]], max_rows: int, buffers: int = 2):
        self.session = session
        self.chunks = chunks
        self.max_rows = int(max_rows)
        self.nbuf = max(2, int(buffers))
        self.dev = session.device
        self._dbuf = None   # per slot: {col: device tensor [max_rows, ...]}
        self._hbuf = None   # per slot: {col: pinned host tensor}
        self._copy_stream = None

    def _alloc(self, first: dict):
        pin = self.dev.type == "cuda"
        self._dbuf, self._hbuf = [], []
        for _ in range(self.nbuf):
            d, h = {}, {}
            for k, a in first.items():
                t = torch.as_tensor(a)
                shape = (self.max_rows,) + tuple(t.shape[1:])
                dt = torch.float32 if t.dim() == 2 else t.dtype
                d[k] = torch.empty(shape, dtype=dt, device=self.dev)
                h[k] = torch.empty(shape, dtype=dt, pin_memory=pin) if pin else None
            self._dbuf.append(d)
            self._hbuf.append(h)
        if self.dev.type == "cuda":
            self._copy_stream = torch.cuda.Stream(device=self.dev)

    def __iter__(self) -> Iterator:
        return self.iter_columns(None)

    def iter_columns(self, columns=None) -> Iterator:
        """A pass that copies only ``columns`` (None: all) to the device: a pass over the labels of a frame whose
        features are hundreds of GB moves only the label bytes over PCIe."""
        from ..sql import types as T
        from ..sql.batch import Batch, ColumnData
        cuda = self.dev.type == "cuda"
        want = None if columns is None else set(columns)
        freed = [None] * self.nbuf     # event: compute work on the slot's previous chunk is enqueued before it
        ready = [None] * self.nbuf     # event: the slot's H2D copy finished
        it = iter(self.chunks())
        pending = []                   # (slot, n) filled, not yet yielded

        keep = [None] * self.nbuf      # pinned source chunks referenced until their H2D is done

        def fill(slot):
            try:
                ch = next(it)
            except StopIteration:
                return False
            if self._dbuf is None:
                self._alloc(ch)
            n = len(next(iter(ch.values())))
            if n > self.max_rows:
                raise ValueError(f"chunk of {n} rows exceeds max_rows={self.max_rows}")
            if cuda:
                if ready[slot] is not None:
                    ready[slot].synchronize()   # the slot's previous H2D has drained its pinned buffer
                with torch.cuda.stream(self._copy_stream):
                    if freed[slot] is not None:
                        self._copy_stream.wait_event(freed[slot])
                    srcs = []
                    for k, a in ch.items():
                        if want is not None and k not in want:
                            continue
                        src = torch.as_tensor(a)
                        d = self._dbuf[slot][k]
                        if src.is_pinned() and src.dtype == d.dtype and src.is_contiguous():
                            d[:n].copy_(src, non_blocking=True)       # already pinned: DMA straight from it
                            srcs.append(src)
                        else:
                            h = self._hbuf[slot][k]
                            h[:n].copy_(src.to(h.dtype) if src.dtype != h.dtype else src)
                            d[:n].copy_(h[:n], non_blocking=True)
                    keep[slot] = srcs
                    ev = torch.cuda.Event()
                    ev.record(self._copy_stream)
                    ready[slot] = ev
            else:
                for k, a in ch.items():
                    if want is None or k in want:
                        self._dbuf[slot][k][:n].copy_(torch.as_tensor(a))
            pending.append((slot, n))
            return True

        slot = 0
        fill(slot)
        slot = 1 % self.nbuf
        while pending:
            s, n = pending.pop(0)
            if cuda:
                torch.cuda.current_stream(self.dev).wait_event(ready[s])
            cols = {}
            for k, t in self._dbuf[s].items():
                if want is not None and k not in want:
                    continue
                v = t[:n]
                cols[k] = ColumnData(v, T.VectorUDT() if v.dim() == 2 else T.from_torch(v.dtype))
            yield Batch(cols, n, self.dev)
            if cuda:  # the consumer has enqueued its work on slot s: the slot may be refilled after it
                ev = torch.cuda.Event()
                ev.record(torch.cuda.current_stream(self.dev))
                freed[s] = ev
            # the next chunk's host staging + H2D overlap the GPU work just enqueued on this one
            if fill(slot):
                slot = (slot + 1) % self.nbuf


def chunked_dataframe(session, chunks: Callable[[], Iterable[dict]], max_rows: int, schema=None):
    """DataFrame streamed from host chunks (``SparkSession.createDataFrameFromChunks``)."""
    from ..sql.dataframe import DataFrame, SourcePlan
    stream = HostChunkStream(session, chunks, max_rows)
    if schema is None:
        first = next(iter(chunks()))
        schema = _schema_of(first)
    plan = SourcePlan(session, "HostChunkScan", None, schema, iter_fn=lambda: iter(stream))
    # column-projected passes and the host chunks themselves, for out-of-core fits (models.util.streamed_columns):
    # a label pass copies only the labels, the quantile sample gathers its rows on the host
    plan.iter_cols_fn = stream.iter_columns
    plan.host_chunks_fn = chunks
    return DataFrame(plan, session)


def device_chunks(session, n_rows: int, chunk_rows: int, make: Callable[[int, int, dict], None], columns: dict,
                  schema=None):
    """DataFrame streamed from chunks generated on the device into reused buffers.

    ``columns``: {name: (trailing shape tuple, torch dtype)}; ``make(row0, n, bufs)`` fills ``bufs[name][:n]``
    for the rank-local rows [row0, row0 + n).  Two buffer slots; a slot is rewritten only after the compute
    stream has passed the previous consumer (same ordering contract as HostChunkStream)."""
    from ..sql import types as T
    from ..sql.batch import Batch, ColumnData
    from ..sql.dataframe import DataFrame, SourcePlan
    dev = session.device
    bufs = [{k: torch.empty((chunk_rows,) + tuple(shp), dtype=dt, device=dev) for k, (shp, dt) in columns.items()}
            for _ in range(2)]

    def gen():
        for i, r0 in enumerate(range(0, n_rows, chunk_rows)):
            n = min(chunk_rows, n_rows - r0)
            b = bufs[i & 1]
            make(r0, n, b)   # enqueued on the compute stream after the slot's previous consumer: in order
            cols = {k: ColumnData(t[:n], T.VectorUDT() if t.dim() == 2 else T.from_torch(t.dtype))
                    for k, t in b.items()}
            yield Batch(cols, n, dev)
    if schema is None:
        schema = T.StructType([T.StructField(k, T.VectorUDT() if len(shp) else T.from_torch(dt), True)
                               for k, (shp, dt) in columns.items()])
    return DataFrame(SourcePlan(session, "DeviceChunkScan", None, schema, iter_fn=gen), session)
