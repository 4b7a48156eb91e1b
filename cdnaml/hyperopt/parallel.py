"""Concurrent trials: ``SparkTrials(parallelism=2)`` (Labs/ML 08L:89-112) and
``GPUTrials``.

Placement follows the engine's one-process-per-GPU design:

* one process: worker threads share this process's GPU (the session's device), each with its own HIP
  stream, so independent single-node fits -- sklearn on the host or this engine's kernels -- overlap.
  Proposals are made on the driver thread from the trials completed so far, exactly like hyperopt's
  asynchronous SparkTrials loop.
* SPMD (torchrun, W ranks): trials are spread over the ranks -- every rank draws the same batch of W x
  parallelism proposals (same history, same ``rstate``), evaluates the ones assigned to it on ITS GPU with a
  rank-local communicator (a trial is a single-node fit, like a SparkTrials task on one worker), and the
  results are all-gathered so every rank's ``Trials`` and TPE state stay identical.

Failed trials are recorded (status ``fail``) instead of aborting the search.  Trials are auto-logged as nested
tracking runs under the active run (Databricks SparkTrials behaviour, L08:89), by rank 0 only.
"""
from __future__ import annotations

import contextlib

import concurrent.futures as cf
import threading
import time
from typing import List, Optional

import torch

from .base import Trials


def _captured_frames(fn) -> list:
    """DataFrames an objective reaches without creating them: closure cells, default arguments, the module
    globals its code names, ``functools.partial`` arguments -- one level deep plus nested helper functions
    (in a fixed order, so every rank replicates the same frames in the same collective order)."""
    import functools
    import types

    from ..sql.dataframe import DataFrame
    out, seen_fn, seen_df = [], set(), set()

    def visit_value(v, depth):
        if isinstance(v, DataFrame):
            if id(v) not in seen_df:
                seen_df.add(id(v))
                out.append(v)
        elif isinstance(v, (list, tuple)):
            for x in v:
                visit_value(x, depth)
        elif isinstance(v, dict):
            for x in v.values():
                visit_value(x, depth)
        elif isinstance(v, functools.partial):
            visit_value(v.func, depth)
            visit_value(v.args, depth)
            visit_value(v.keywords, depth)
        elif isinstance(v, (types.FunctionType, types.MethodType)) and depth < 3:
            visit_fn(v, depth + 1)

    def visit_fn(f, depth):
        f = getattr(f, "__func__", f)
        if id(f) in seen_fn or not hasattr(f, "__code__"):
            return
        seen_fn.add(id(f))
        for cell in f.__closure__ or ():
            try:
                visit_value(cell.cell_contents, depth)
            except ValueError:  # empty cell
                pass
        visit_value(f.__defaults__ or (), depth)
        g = getattr(f, "__globals__", {})
        for name in f.__code__.co_names:
            if name in g:
                visit_value(g[name], depth)
    visit_value(fn, 0)
    return out


def _replicate_captured_frames(fn, session, rank_local) -> list:
    """Swap the plan of every captured (rank-sharded) DataFrame for a replicated copy of the whole table;
    returns [(frame, original plan)] to restore after the search."""
    frames = _captured_frames(fn)
    restore = []
    for df in frames:
        pdf = df.toPandas()                     # collective: every rank gets every row, in global order
        schema = df.schema
        with rank_local(session):
            rep = session.createDataFrame(pdf, schema)
        restore.append((df, df._plan))
        df._plan = rep._plan
    return restore


class GPUTrials(Trials):
    def __init__(self, parallelism: Optional[int] = None, timeout: Optional[float] = None,
                 devices: Optional[List[int]] = None, spark_session=None, autolog: bool = True):
        super().__init__()
        self.spark = spark_session
        if devices is not None:
            self.devices = list(devices)
        else:
            dev = self._session_device()
            # this process's GPU only: the other visible GPUs belong to the other ranks of an SPMD job
            self.devices = [dev.index if dev.index is not None else torch.cuda.current_device()] \
                if dev is not None and dev.type == "cuda" else []
        self.parallelism = int(parallelism) if parallelism else 4
        self.timeout = timeout
        self._autolog = autolog
        self._local = threading.local()

    def _session(self):
        if self.spark is not None:
            return self.spark
        try:
            from ..session import SparkSession
            return SparkSession.getActiveSession()
        except Exception:  # noqa: BLE001
            return None

    def _session_device(self):
        s = self._session()
        if s is not None:
            return s.device
        return torch.device("cuda", torch.cuda.current_device()) if torch.cuda.is_available() else None

    @contextlib.contextmanager
    def _rank_local(self, session):
        """Run a trial on this rank alone: engine fits inside use a one-rank communicator."""
        if session is None or not session.comm.distributed:
            yield
            return
        from ..parallel.comm import Comm
        saved = session.comm
        local = Comm(saved.device)
        local.initialized, local.rank, local.world_size, local.backend = False, 0, 1, "local"
        session.comm = local
        try:
            yield
        finally:
            session.comm = saved

    def _run_spmd(self, comm, session, fn, space, next_assignment, should_stop, max_evals):
        # DataFrames the objective closes over were sharded under the GLOBAL communicator (1/W of the rows
        # on each rank); a rank-local trial must see the whole table, as a SparkTrials task does, so they
        # are replicated on every rank for the duration of the search
        restore = _replicate_captured_frames(fn, session, self._rank_local)
        try:
            return self._run_spmd_loop(comm, session, fn, space, next_assignment, should_stop, max_evals)
        finally:
            for df, plan in restore:
                df._plan = plan

    def _run_spmd_loop(self, comm, session, fn, space, next_assignment, should_stop, max_evals):
        from .fmin import _TrialLogger, evaluate_trial
        log = _TrialLogger(self) if comm.rank == 0 else None
        W, me = comm.world_size, comm.rank
        t0 = time.time()
        per = max(1, self.parallelism)
        while True:
            timed_out = comm.broadcast_object(self.timeout is not None and time.time() - t0 >= self.timeout)
            k = min(W * per, max_evals - len(self))
            if timed_out or should_stop() or k <= 0:
                break
            assigns = [next_assignment() for _ in range(k)]        # identical on every rank
            trials = [self.new_trial(a, space) for a in assigns]
            mine = [i for i in range(k) if i % W == me]

            def run(i):
                evaluate_trial(fn, space, trials[i], True)
                return i
            # one rank-local communicator for the whole local batch (swapped once: the worker threads share it)
            with self._rank_local(session):
                if len(mine) > 1:
                    with cf.ThreadPoolExecutor(max_workers=per, thread_name_prefix="cdnaml-trial") as ex:
                        list(ex.map(run, mine))
                else:
                    for i in mine:
                        run(i)
            keys = ("state", "result", "book_time", "refresh_time")
            done = comm.all_gather_object({i: {kk: trials[i][kk] for kk in keys} for i in mine})
            for part in done:
                for i, fields in part.items():
                    trials[i].update(fields)
            if log is not None:
                for tr, a in zip(trials, assigns):
                    log.log(tr, a)
        if log is not None:
            log.close()

    def _worker_ctx(self, slot: int):
        if not self.devices:
            return None, None
        dev = self.devices[slot % len(self.devices)]
        return dev, torch.cuda.Stream(device=dev)

    def _run_parallel(self, fn, space, next_assignment, should_stop, max_evals, catch):
        from .fmin import _TrialLogger, evaluate_trial
        session = self._session()
        if session is not None and session.comm.distributed:
            return self._run_spmd(session.comm, session, fn, space, next_assignment, should_stop, max_evals)
        log = _TrialLogger(self)
        t0 = time.time()
        slots = list(range(self.parallelism))
        ctx = {s: self._worker_ctx(s) for s in slots}

        def run(slot, tr):
            dev, stream = ctx[slot]
            if stream is not None:
                with torch.cuda.device(dev), torch.cuda.stream(stream):
                    res = evaluate_trial(fn, space, tr, True)
                    stream.synchronize()
                return res
            return evaluate_trial(fn, space, tr, True)

        running = {}
        free = list(slots)
        with cf.ThreadPoolExecutor(max_workers=self.parallelism, thread_name_prefix="cdnaml-trial") as ex:
            while True:
                timed_out = self.timeout is not None and time.time() - t0 >= self.timeout
                while free and not timed_out and not should_stop() and \
                        len(self) < max_evals:
                    a = next_assignment()
                    tr = self.new_trial(a, space)
                    slot = free.pop()
                    running[ex.submit(run, slot, tr)] = (slot, tr, a)
                if not running:
                    break
                done, _ = cf.wait(list(running), return_when=cf.FIRST_COMPLETED)
                for f in done:
                    slot, tr, a = running.pop(f)
                    free.append(slot)
                    f.result()
                    log.log(tr, a)
        log.close()


class SparkTrials(GPUTrials):
    """``SparkTrials(parallelism, timeout, spark_session)``: one trial per worker slot."""

    def __init__(self, parallelism: Optional[int] = None, timeout: Optional[float] = None, spark_session=None):
        super().__init__(parallelism=parallelism or 4, timeout=timeout, spark_session=spark_session)
