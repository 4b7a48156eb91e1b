"""Multi-rank GPU code path rehearsed on one GPU.

The driver's 8-GPU scaling runs take the RCCL path of the tree engine: level histograms built in slot chunks
whose all-reduces overlap the next chunk (``ForestTrainer._hist_overlapped``), the record-free level-0/1
kernel on each rank's shard, device-side split decode, per-rank row shards.  A 1-GPU box cannot start RCCL with
two ranks on one device, so here 2 and 3 ranks share cuda:0 over ``gloo`` (CDNAML_COMM_BACKEND=gloo: host-staged collectives,
the same int64 sums) and must grow the forest the single-rank run grows: bench.py's digest is a function of the
global table only (rows keyed by global row id), whatever the GPU count.
"""
import os
import re
import socket
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _digest(cmd, env):
    r = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=280, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-3000:]
    m = re.findall(r"digest=([0-9a-f]+)", r.stderr)
    assert m, r.stderr[-3000:]
    return m[-1]


@pytest.mark.gpu
@pytest.mark.timeout(600)
def test_ranks_sharing_one_gpu_grow_the_single_rank_forest():
    env = {**os.environ, "CDNAML_COMM_BACKEND": "gloo", "OMP_NUM_THREADS": "2"}
    args = ["bench.py", "--rows", "300001", "--steps", "1", "--warmup", "0"]
    ref = _digest([sys.executable] + args, env)
    for nproc in (2, 3):
        cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={nproc}",
               "--master-addr", "127.0.0.1", "--master-port", str(_port())] + args + ["--gpus", str(nproc)]
        assert _digest(cmd, env) == ref, f"{nproc} ranks on one GPU grew a different forest"
