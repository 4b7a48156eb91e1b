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


def _worker(scenario, tmp_path, nproc, device):
    import json
    out = tmp_path / f"{scenario}_{device}_{nproc}.json"
    env = {**os.environ, "CDNAML_COMM_BACKEND": "gloo", "OMP_NUM_THREADS": "2", "PYTHONPATH": ROOT,
           "CDNAML_DEVICE": device, "CDNAML_CONF_CDNAML__WAREHOUSE__DIR": str(tmp_path / f"wh_{device}{nproc}")}
    for k in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        env.pop(k, None)
    w = os.path.join(ROOT, "tests", "dist_worker.py")
    cmd = [sys.executable, w, scenario, str(out)] if nproc == 1 else \
        [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={nproc}",
         "--master-addr", "127.0.0.1", "--master-port", str(_port()), w, scenario, str(out)]
    r = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=280, cwd=str(tmp_path))
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-3000:]
    return json.loads(out.read_text())


@pytest.mark.gpu
@pytest.mark.timeout(600)
def test_deep_forests_gpu_ranks_match_cpu(tmp_path):
    """Forests deeper than 8 levels on the GPU path (device split decode + node-id partition, GPU-drawn feature
    subsets, node_compact record histograms), with and without reduce-scatter: 1 and 2 ranks on cuda:0 grow the
    forests the CPU emulation grows, bit for bit."""
    cpu = _worker("trees_deep", tmp_path, 1, "cpu")
    for nproc in (1, 2):
        assert _worker("trees_deep", tmp_path, nproc, "cuda") == cpu, nproc
