"""Multi-process SPMD correctness on CPU (gloo, world_size 2): the distributed
engine must give the single-process answers."""
import json
import os
import socket
import subprocess
import sys

import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _run(scenario, tmp_path, nproc):
    out = tmp_path / f"{scenario}_{nproc}.json"
    env = dict(os.environ, CDNAML_DEVICE="cpu", OMP_NUM_THREADS="2", PYTHONPATH=ROOT)
    for k in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        env.pop(k, None)
    env["CDNAML_CONF_CDNAML__WAREHOUSE__DIR"] = str(tmp_path / f"wh{nproc}")
    if nproc == 1:
        cmd = [sys.executable, os.path.join(HERE, "dist_worker.py"), scenario, str(out)]
    else:
        cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={nproc}",
               "--master-addr", "127.0.0.1", "--master-port", str(_free_port()),
               os.path.join(HERE, "dist_worker.py"), scenario, str(out)]
    r = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=600, cwd=str(tmp_path))
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    return json.loads(out.read_text())


@pytest.mark.parametrize("scenario", ["frame", "ml"])
def test_two_ranks_match_one(scenario, tmp_path):
    one = _run(scenario, tmp_path, 1)
    two = _run(scenario, tmp_path, 2)
    for k in one:
        if isinstance(one[k], list) and one[k] and isinstance(one[k][0], float):
            assert two[k] == pytest.approx(one[k], rel=1e-6, abs=1e-6), k
        elif isinstance(one[k], float):
            assert two[k] == pytest.approx(one[k], rel=1e-5, abs=1e-6), k
        else:
            assert two[k] == one[k], k
