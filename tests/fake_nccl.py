"""A recording stand-in for ``torch.distributed`` under ``backend == "nccl"``.

CPU CI runs the multi-rank paths over gloo, where ``Comm`` takes its gloo branches (reduce-scatter as all-reduce
and slice, all-gather as a list gather).  The RCCL branches -- ``dist.reduce_scatter_tensor``,
``dist.all_gather_into_tensor``, ``barrier(device_ids=...)``, the device-tensor staging of ``_dev_tensor`` -- would
otherwise first run on an 8-GPU node.  ``install(comm_module)`` swaps the ``dist`` that ``cdnaml.parallel.comm``
uses for a proxy that:

* reports ``get_backend() == "nccl"``, so every ``Comm`` built afterwards takes the RCCL branches;
* implements the nccl-only collectives with gloo primitives (same results: integer sums are exact);
* checks what RCCL requires of every call and records each violation instead of failing inside gloo:
  contiguous buffers, matching dtypes, ``out.numel() * W == in.numel()`` (reduce-scatter) and
  ``out.numel() == W * in.numel()`` (all-gather), all-to-all split sizes that add up to the buffers;
* counts every collective by name.

``RECORD`` holds the counters and ``VIOLATIONS`` the failed checks (``"op: message"``)."""
from __future__ import annotations

import collections

import torch
import torch.distributed as _real

RECORD = collections.Counter()
VIOLATIONS = []


def _check(cond, op, msg):
    if not cond:
        VIOLATIONS.append(f"{op}: {msg}")


def _tensor_ok(op, *ts):
    for t in ts:
        _check(isinstance(t, torch.Tensor), op, f"not a tensor: {type(t).__name__}")
        if isinstance(t, torch.Tensor):
            _check(t.is_contiguous(), op, f"non-contiguous buffer {tuple(t.shape)} stride {t.stride()}")


class _Done:
    """A completed work handle (the proxy runs the gloo emulation of an async collective synchronously)."""

    def wait(self):
        return True

    def is_completed(self):
        return True


class NcclOverGloo:
    """Proxy module: attribute access falls through to torch.distributed except for the overrides below."""

    ReduceOp = _real.ReduceOp

    def __getattr__(self, name):
        return getattr(_real, name)

    # --------------------------------------------------------------- identity
    def get_backend(self, group=None):
        return "nccl"

    # ----------------------------------------------------------- collectives
    def all_reduce(self, t, op=_real.ReduceOp.SUM, group=None, async_op=False):
        RECORD["all_reduce_async" if async_op else "all_reduce"] += 1
        _tensor_ok("all_reduce", t)
        return _real.all_reduce(t, op=op, group=group, async_op=async_op)

    def reduce_scatter_tensor(self, out, inp, op=_real.ReduceOp.SUM, group=None, async_op=False):
        RECORD["reduce_scatter_tensor_async" if async_op else "reduce_scatter_tensor"] += 1
        W = _real.get_world_size()
        _tensor_ok("reduce_scatter_tensor", out, inp)
        _check(out.dtype == inp.dtype, "reduce_scatter_tensor", f"dtype {out.dtype} vs {inp.dtype}")
        _check(out.device == inp.device, "reduce_scatter_tensor", f"device {out.device} vs {inp.device}")
        _check(out.numel() * W == inp.numel(), "reduce_scatter_tensor",
               f"out {tuple(out.shape)} x W={W} != in {tuple(inp.shape)}")
        buf = inp.clone()
        _real.all_reduce(buf, op=op, group=group)
        r = _real.get_rank()
        out.copy_(buf.reshape(W, -1)[r].reshape(out.shape))
        return _Done() if async_op else None

    def all_gather_into_tensor(self, out, inp, group=None, async_op=False):
        RECORD["all_gather_into_tensor"] += 1
        W = _real.get_world_size()
        _tensor_ok("all_gather_into_tensor", out, inp)
        _check(out.dtype == inp.dtype, "all_gather_into_tensor", f"dtype {out.dtype} vs {inp.dtype}")
        _check(out.numel() == W * inp.numel(), "all_gather_into_tensor",
               f"out {tuple(out.shape)} != W={W} x in {tuple(inp.shape)}")
        bufs = [torch.empty_like(inp) for _ in range(W)]
        _real.all_gather(bufs, inp, group=group)
        out.copy_(torch.stack(bufs).reshape(out.shape))
        return None

    def all_gather(self, bufs, t, group=None, async_op=False):
        RECORD["all_gather"] += 1
        _tensor_ok("all_gather", t, *bufs)
        for b in bufs:
            _check(b.shape == t.shape and b.dtype == t.dtype, "all_gather", "buffer shape / dtype mismatch")
        return _real.all_gather(bufs, t, group=group, async_op=async_op)

    def all_to_all_single(self, out, inp, output_split_sizes=None, input_split_sizes=None, group=None,
                          async_op=False):
        RECORD["all_to_all_single"] += 1
        _tensor_ok("all_to_all_single", out, inp)
        _check(out.dtype == inp.dtype, "all_to_all_single", f"dtype {out.dtype} vs {inp.dtype}")
        if input_split_sizes is not None:
            _check(sum(input_split_sizes) == inp.numel(), "all_to_all_single",
                   f"input splits {sum(input_split_sizes)} != {inp.numel()}")
        if output_split_sizes is not None:
            _check(sum(output_split_sizes) == out.numel(), "all_to_all_single",
                   f"output splits {sum(output_split_sizes)} != {out.numel()}")
        return _real.all_to_all_single(out, inp, output_split_sizes=output_split_sizes,
                                       input_split_sizes=input_split_sizes, group=group, async_op=async_op)

    def broadcast(self, t, src=0, group=None, async_op=False):
        RECORD["broadcast"] += 1
        _tensor_ok("broadcast", t)
        return _real.broadcast(t, src=src, group=group, async_op=async_op)

    def barrier(self, group=None, async_op=False, device_ids=None):
        RECORD["barrier"] += 1
        # RCCL's barrier takes this rank's device (Comm passes [device.index]); gloo takes none
        _check(device_ids is not None, "barrier", "nccl barrier without device_ids")
        return _real.barrier(group=group, async_op=async_op)


def install(comm_module):
    """Route ``comm_module.dist`` through the proxy; returns a callable that restores it."""
    prev = comm_module.dist
    comm_module.dist = NcclOverGloo()
    RECORD.clear()
    VIOLATIONS.clear()

    def restore():
        comm_module.dist = prev
    return restore
