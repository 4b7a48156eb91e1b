"""Collective communication over RCCL/xGMI.

SPMD process model: one process per GPU, ``torch.distributed`` with the
``nccl`` backend (= RCCL on ROCm) when GPUs are present, ``gloo`` on CPU.
A single-process run uses the trivial communicator (every collective is the
identity), so the same engine code runs in CPU CI, on one GPU and on an
8-GPU xGMI node.

Collectives used by the engine:
  * all_reduce (sum/min/max) — sufficient statistics (Gram, histograms,
    metrics); several tensors are fused into ONE flat bucket per call so a
    tree level or an optimiser iteration costs one RCCL launch;
  * all_gather (fixed / variable length) — quantile sketches, dictionaries;
  * all_to_all_v — hash shuffles (groupBy / join / dropDuplicates / repartition);
  * broadcast — model parameters, tuning trial configs.

Failure handling:
  * every collective runs inside ``_guard``: a failure surfaces as
    :class:`CommError` naming the rank, the collective and its call number;
  * watchdog: the process group is created with ``CDNAML_COMM_TIMEOUT``
    seconds (default 1800), so a peer that died or hangs turns a blocked
    collective into an error instead of a silent hang;
  * fault injection: ``CDNAML_FAULT=rank:op:n`` makes ``rank`` fail its n-th
    ``op`` call (op = all_reduce, all_gather, broadcast, all_to_all, barrier
    or ``*``) before anything is sent; the failing rank tears its process
    group down so peers error out promptly.
"""
from __future__ import annotations

import datetime
import os
import pickle
from typing import Any, List, Optional, Sequence

import torch
import torch.distributed as dist


class CommError(RuntimeError):
    """A collective failed on this rank (injected, a peer died, or the watchdog timed out)."""

    def __init__(self, rank: int, op: str, call: int, cause: str):
        super().__init__(f"[rank {rank}] collective {op} (call #{call}) failed: {cause}")
        self.rank, self.op, self.call = rank, op, call


def _parse_fault(spec: Optional[str]):
    if not spec:
        return None
    try:
        r, op, n = spec.split(":")
        return int(r), op, int(n)
    except ValueError:
        raise ValueError(f"CDNAML_FAULT must be rank:op:n, got {spec!r}") from None


class _Guard:
    def __init__(self, comm: "Comm", op: str):
        self.comm, self.op = comm, op

    def __enter__(self):
        c = self.comm
        c.op_calls[self.op] = c.op_calls.get(self.op, 0) + 1
        self.n = c.op_calls[self.op]
        f = c.fault
        if f is not None and f[0] == c.rank and f[1] in (self.op, "*"):
            k = self.n if f[1] == self.op else sum(c.op_calls.values())
            if k == f[2]:
                c.fault = None
                err = CommError(c.rank, self.op, self.n, "injected fault (CDNAML_FAULT)")
                c.abort()
                raise err
        return self

    def __exit__(self, et, ev, tb):
        if ev is not None and not isinstance(ev, CommError) and isinstance(ev, (RuntimeError, ConnectionError,
                                                                                  OSError)):
            raise CommError(self.comm.rank, self.op, self.n, f"{type(ev).__name__}: {ev}") from ev
        return False


class _Pending:
    """An in-flight all-reduce (Comm.all_reduce_async)."""

    def __init__(self, work, w: torch.Tensor, t: torch.Tensor, comm: Optional["Comm"] = None):
        self.work, self.w, self.t, self.comm = work, w, t, comm

    def wait(self) -> torch.Tensor:
        if self.work is not None:
            with self.comm._guard("all_reduce_wait"):
                self.work.wait()
            self.work = None
            if self.w.data_ptr() != self.t.data_ptr():
                self.t.copy_(self.w)
        return self.t


class _PendingRS:
    """An in-flight reduce-scatter (Comm.reduce_scatter_async); ``wait()`` -> this rank's slice."""

    def __init__(self, work, w, out, device, comm):
        self.work, self.w, self.out, self.device, self.comm = work, w, out, device, comm

    def wait(self) -> torch.Tensor:
        if self.work is not None:
            with self.comm._guard("reduce_scatter_wait"):
                self.work.wait()
            self.work = None
            if self.out is None:  # gloo: the all-reduced host copy, sliced
                self.out = self.w[self.comm.rank]
            self.out = self.out.to(self.device)
        return self.out


class Comm:
    """Communicator bound to this process's device."""

    def __init__(self, device: torch.device):
        self.device = device
        self.initialized = dist.is_available() and dist.is_initialized()
        self.rank = dist.get_rank() if self.initialized else 0
        self.world_size = dist.get_world_size() if self.initialized else 1
        self.backend = dist.get_backend() if self.initialized else "local"
        self.bytes_reduced = 0
        self.calls = 0
        self.op_calls = {}
        self.fault = _parse_fault(os.environ.get("CDNAML_FAULT"))

    def _guard(self, op: str) -> _Guard:
        return _Guard(self, op)

    def abort(self) -> None:
        """Tear this rank's process group down (peers' pending collectives then fail)."""
        if self.initialized and dist.is_initialized():
            try:
                dist.destroy_process_group()
            except Exception:  # noqa: BLE001 - best effort during failure handling
                pass
            self.initialized = False

    def shutdown(self) -> None:
        """Orderly end of a distributed job: every rank reaches a barrier, then tears its process group down.

        Left to interpreter exit, the group's destructors run in whatever order the ranks happen to exit; a
        gloo rank whose peers already closed their sockets can then abort (SIGABRT) after the job's work is
        done, which turns a finished run into a failed launch."""
        if self.initialized and dist.is_initialized():
            if self.world_size > 1:
                self.barrier()
            dist.destroy_process_group()
            self.initialized = False

    # ----------------------------------------------------------------- info
    @property
    def distributed(self) -> bool:
        return self.world_size > 1

    def _dev_tensor(self, t: torch.Tensor):
        """nccl needs device tensors, gloo needs host tensors."""
        if self.backend == "nccl":
            return t if t.is_cuda else t.to(self.device)
        return t if not t.is_cuda else t.cpu()

    # ------------------------------------------------------------ all_reduce
    def all_reduce(self, t: torch.Tensor, op: str = "sum") -> torch.Tensor:
        """In-place all-reduce; returns t."""
        if not self.distributed:
            return t
        self.calls += 1
        self.bytes_reduced += t.numel() * t.element_size()
        rop = {"sum": dist.ReduceOp.SUM, "max": dist.ReduceOp.MAX, "min": dist.ReduceOp.MIN}[op]
        w = self._dev_tensor(t)
        if not w.is_contiguous():
            w = w.contiguous()
        with self._guard("all_reduce"):
            dist.all_reduce(w, op=rop)
        if w.data_ptr() != t.data_ptr():
            t.copy_(w)
        return t

    def all_reduce_async(self, t: torch.Tensor, op: str = "sum") -> "_Pending":
        """Start an in-place all-reduce and return a handle whose ``wait()`` completes it.

        RCCL: the collective is enqueued on the process group's stream after the work already queued on the
        current stream, so kernels launched after this call overlap with it; ``wait()`` makes the current
        stream wait for it.  gloo: the host copy is reduced on gloo's thread and copied back on ``wait()``."""
        if not self.distributed:
            return _Pending(None, t, t)
        self.calls += 1
        self.bytes_reduced += t.numel() * t.element_size()
        rop = {"sum": dist.ReduceOp.SUM, "max": dist.ReduceOp.MAX, "min": dist.ReduceOp.MIN}[op]
        w = self._dev_tensor(t)
        if not w.is_contiguous():
            w = w.contiguous()
        with self._guard("all_reduce"):
            work = dist.all_reduce(w, op=rop, async_op=True)
        return _Pending(work, w, t, self)

    def all_reduce_many(self, tensors: Sequence[torch.Tensor], op: str = "sum") -> List[torch.Tensor]:
        """Fuse several same-dtype tensors into one bucket -> one collective."""
        if not self.distributed or not tensors:
            return list(tensors)
        dt = tensors[0].dtype
        flat = torch.cat([t.reshape(-1).to(dt) for t in tensors])
        self.all_reduce(flat, op)
        out, o = [], 0
        for t in tensors:
            k = t.numel()
            t.copy_(flat[o:o + k].view_as(t))
            o += k
            out.append(t)
        return out

    def all_reduce_scalar(self, x: float, op: str = "sum") -> float:
        if not self.distributed:
            return x
        t = torch.tensor([x], dtype=torch.float64, device=self.device)
        return float(self.all_reduce(t, op)[0])

    # ------------------------------------------------------------ gathers
    def all_gather_object(self, obj: Any) -> List[Any]:
        if not self.distributed:
            return [obj]
        out = [None] * self.world_size
        with self._guard("all_gather"):
            dist.all_gather_object(out, obj)
        return out

    def broadcast_object(self, obj: Any, src: int = 0) -> Any:
        if not self.distributed:
            return obj
        box = [obj]
        with self._guard("broadcast"):
            dist.broadcast_object_list(box, src=src)
        return box[0]

    def all_gather_varlen(self, t: torch.Tensor) -> List[torch.Tensor]:
        """Gather tensors whose first dimension differs per rank."""
        if not self.distributed:
            return [t]
        n = torch.tensor([t.shape[0]], dtype=torch.int64, device=self.device)
        sizes = [torch.zeros_like(n) for _ in range(self.world_size)]
        n_w = self._dev_tensor(n)
        sizes_w = [self._dev_tensor(s) for s in sizes]
        with self._guard("all_gather"):
            dist.all_gather(sizes_w, n_w)
        sizes = [int(s.item()) for s in sizes_w]
        mx = max(sizes)
        pad = torch.zeros((mx,) + tuple(t.shape[1:]), dtype=t.dtype, device=t.device)
        pad[: t.shape[0]] = t
        pad_w = self._dev_tensor(pad)
        bufs = [torch.empty_like(pad_w) for _ in range(self.world_size)]
        with self._guard("all_gather"):
            dist.all_gather(bufs, pad_w)
        return [b[:s].to(t.device) for b, s in zip(bufs, sizes)]

    def reduce_scatter(self, t: torch.Tensor) -> torch.Tensor:
        """t [W, ...] (the same shape on every rank) -> this rank's slice of the element-wise sum, t.sum over
        ranks [rank].  RCCL: one reduce_scatter (each rank receives 1/W of the bytes an all-reduce moves);
        gloo has no reduce-scatter, so it all-reduces and slices (the same integer sums)."""
        if not self.distributed:
            return t[0]
        W = self.world_size
        assert t.shape[0] == W
        self.calls += 1
        self.bytes_reduced += t.numel() * t.element_size() // W
        if self.backend == "nccl":
            w = self._dev_tensor(t).contiguous()
            out = torch.empty(w.shape[1:], dtype=w.dtype, device=w.device)
            with self._guard("reduce_scatter"):
                dist.reduce_scatter_tensor(out, w)
            return out.to(t.device)
        w = self._dev_tensor(t).contiguous().clone()
        with self._guard("reduce_scatter"):
            dist.all_reduce(w)
        return w[self.rank].to(t.device)

    def reduce_scatter_async(self, t: torch.Tensor) -> "_PendingRS":
        """``reduce_scatter`` started on the collective stream; ``wait()`` returns this rank's slice.

        RCCL: ``reduce_scatter_tensor(async_op=True)`` is enqueued behind the work already on the current stream, so
        kernels launched afterwards (the next slot chunk's histogram) overlap it.  gloo: an async all-reduce of a
        host copy, sliced on ``wait()`` (the same integer sums)."""
        if not self.distributed:
            return _PendingRS(None, None, t[0], None, self)
        W = self.world_size
        assert t.shape[0] == W
        self.calls += 1
        self.bytes_reduced += t.numel() * t.element_size() // W
        if self.backend == "nccl":
            w = self._dev_tensor(t).contiguous()
            out = torch.empty(w.shape[1:], dtype=w.dtype, device=w.device)
            with self._guard("reduce_scatter"):
                work = dist.reduce_scatter_tensor(out, w, async_op=True)
            return _PendingRS(work, w, out, t.device, self)
        w = self._dev_tensor(t).contiguous().clone()
        with self._guard("reduce_scatter"):
            work = dist.all_reduce(w, async_op=True)
        return _PendingRS(work, w, None, t.device, self)

    def all_gather_tensor(self, t: torch.Tensor) -> torch.Tensor:
        """Same-shape tensors of every rank stacked: [W, *t.shape]."""
        if not self.distributed:
            return t[None]
        w = self._dev_tensor(t).contiguous()
        self.calls += 1
        if self.backend == "nccl":
            out = torch.empty((self.world_size,) + tuple(w.shape), dtype=w.dtype, device=w.device)
            with self._guard("all_gather"):
                dist.all_gather_into_tensor(out, w)
        else:
            bufs = [torch.empty_like(w) for _ in range(self.world_size)]
            with self._guard("all_gather"):
                dist.all_gather(bufs, w)
            out = torch.stack(bufs)
        return out.to(t.device)

    def broadcast(self, t: torch.Tensor, src: int = 0) -> torch.Tensor:
        if not self.distributed:
            return t
        w = self._dev_tensor(t)
        with self._guard("broadcast"):
            dist.broadcast(w, src=src)
        if w.data_ptr() != t.data_ptr():
            t.copy_(w)
        return t

    # ------------------------------------------------------------ all-to-all
    def all_to_all_counts(self, send_counts: Sequence[int]) -> List[int]:
        """Rows each rank will send here, given the rows this rank sends to each (one tiny all-to-all; the only
        host round trip of a shuffle -- pass its result to every all_to_all_v with the same routing)."""
        if not self.distributed:
            return [int(send_counts[0])]
        W = self.world_size
        send_n = torch.tensor([int(c) for c in send_counts], dtype=torch.int64)
        recv_n = torch.empty(W, dtype=torch.int64)
        s_w, r_w = self._dev_tensor(send_n), self._dev_tensor(recv_n)
        with self._guard("all_to_all"):
            dist.all_to_all_single(r_w, s_w)
        self.calls += 1
        return [int(x) for x in r_w.cpu().tolist()]

    def all_to_all_v(self, chunks: List[torch.Tensor], recv_counts: Optional[Sequence[int]] = None
                     ) -> List[torch.Tensor]:
        """chunks[j] goes to rank j; returns the list received from every rank.

        Without ``recv_counts`` the counts are exchanged first (one tiny all-to-all and a host read), then the
        payload in a single all_to_all_single over xGMI (every link carries its own pair).  Exchanges whose
        routing is known (the block-ALS factor replies of every iteration, the columns of one shuffle) pass the
        counts and skip that round trip.
        """
        if not self.distributed:
            return [chunks[0]]
        W = self.world_size
        assert len(chunks) == W
        ref = chunks[0]
        tail = tuple(ref.shape[1:])
        inner = 1
        for s in tail:
            inner *= s
        if recv_counts is None:
            recv_counts = self.all_to_all_counts([c.shape[0] for c in chunks])
            self.calls -= 1
        recv_counts = [int(x) for x in recv_counts]
        flat = torch.cat([c.reshape(-1) for c in chunks]) if any(c.numel() for c in chunks) else \
            torch.empty(0, dtype=ref.dtype, device=ref.device)
        dtype = flat.dtype
        is_bool = dtype == torch.bool
        if is_bool:
            flat = flat.to(torch.uint8)
        fw = self._dev_tensor(flat)
        out = torch.empty(sum(recv_counts) * inner, dtype=fw.dtype, device=fw.device)
        with self._guard("all_to_all"):
            dist.all_to_all_single(out, fw, output_split_sizes=[r * inner for r in recv_counts],
                                   input_split_sizes=[int(c.shape[0]) * inner for c in chunks])
        self.calls += 2
        self.bytes_reduced += flat.numel() * flat.element_size()
        out = out.to(ref.device)
        if is_bool:
            out = out.bool()
        res, o = [], 0
        for r in recv_counts:
            res.append(out[o:o + r * inner].view((r,) + tail))
            o += r * inner
        return res

    def barrier(self):
        if self.distributed:
            with self._guard("barrier"):
                if self.backend == "nccl":
                    dist.barrier(device_ids=[self.device.index])
                else:
                    dist.barrier()


def rank_device_index(backend: Optional[str] = None) -> int:
    """This process's GPU: LOCAL_RANK.  Several ranks may share a GPU only under the host-staged gloo backend
    (LOCAL_RANK % device_count, the 1-GPU rehearsal); RCCL does not support two ranks on one device, so under
    nccl a LOCAL_RANK beyond the visible GPUs is an error here rather than an obscure failure later."""
    lr = int(os.environ.get("LOCAL_RANK", "0"))
    ndev = max(1, torch.cuda.device_count())
    if backend is None:
        ws = int(os.environ.get("WORLD_SIZE", "1"))
        backend = os.environ.get("CDNAML_COMM_BACKEND") or ("nccl" if ws > 1 else "gloo")
    if backend == "nccl" and lr >= ndev:
        raise RuntimeError(f"LOCAL_RANK {lr} but only {ndev} GPU(s) visible: one RCCL rank per GPU "
                           f"(set CDNAML_COMM_BACKEND=gloo to share a GPU between ranks)")
    return lr % ndev


def init_from_env(device_type: Optional[str] = None, timeout_s: Optional[float] = None) -> None:
    """Initialise torch.distributed from torchrun-style env vars (idempotent).

    MASTER_ADDR should be 127.0.0.1 for single-node runs.  The collective
    watchdog timeout is ``timeout_s`` or ``CDNAML_COMM_TIMEOUT`` (seconds).
    """
    if timeout_s is None:
        timeout_s = float(os.environ.get("CDNAML_COMM_TIMEOUT", "1800"))
    if not dist.is_available() or dist.is_initialized():
        return
    ws = int(os.environ.get("WORLD_SIZE", "1"))
    if ws <= 1:
        return
    if device_type is None:
        device_type = "cuda" if torch.cuda.is_available() else "cpu"
    # CDNAML_COMM_BACKEND=gloo on GPUs: host-staged collectives, so several ranks can share one GPU (a 1-GPU box
    # rehearses the multi-rank GPU code path: ranks map to cuda:(LOCAL_RANK % device_count))
    backend = os.environ.get("CDNAML_COMM_BACKEND") or ("nccl" if device_type == "cuda" else "gloo")
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    kwargs = dict(backend=backend, timeout=datetime.timedelta(seconds=timeout_s))
    if backend == "nccl":
        lr = rank_device_index(backend)
        torch.cuda.set_device(lr)
        kwargs["device_id"] = torch.device("cuda", lr)
    dist.init_process_group(**kwargs)
