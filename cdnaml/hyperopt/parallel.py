"""Concurrent trials: ``SparkTrials(parallelism=2)`` (Labs/ML 08L:89-112) and
``GPUTrials``.

Each worker thread owns a HIP stream (and a device, round-robin over the
visible GPUs when ``devices`` is not given), so independent single-node fits —
sklearn on the host or this engine's kernels on the GPU — overlap.  Proposals
are made on the driver thread from the trials completed so far, exactly like
hyperopt's asynchronous SparkTrials loop.  Failed trials are recorded (status
``fail``) instead of aborting the search.  Trials are auto-logged as nested
tracking runs under the active run (Databricks SparkTrials behaviour, L08:89).
"""
from __future__ import annotations

import concurrent.futures as cf
import threading
import time
from typing import List, Optional

import torch

from .base import Trials


class GPUTrials(Trials):
    def __init__(self, parallelism: Optional[int] = None, timeout: Optional[float] = None,
                 devices: Optional[List[int]] = None, spark_session=None, autolog: bool = True):
        super().__init__()
        ngpu = torch.cuda.device_count() if torch.cuda.is_available() else 0
        self.devices = list(devices) if devices is not None else list(range(ngpu))
        default_par = max(1, len(self.devices)) if self.devices else 4
        self.parallelism = int(parallelism) if parallelism else default_par
        self.timeout = timeout
        self._autolog = autolog
        self._local = threading.local()

    def _worker_ctx(self, slot: int):
        if not self.devices:
            return None, None
        dev = self.devices[slot % len(self.devices)]
        return dev, torch.cuda.Stream(device=dev)

    def _run_parallel(self, fn, space, next_assignment, should_stop, max_evals, catch):
        from .fmin import _TrialLogger, evaluate_trial
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
