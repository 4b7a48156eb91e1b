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


def test_fault_injection_surfaces_rank_and_op(tmp_path):
    """an injected failure on rank 1 becomes a CommError on BOTH ranks (rank 1:
    the injected fault; rank 0: its blocked collective errors out via the torn-down group or the
    watchdog) within the watchdog timeout, instead of a hang."""
    out = tmp_path / "fault.json"
    env = dict(os.environ, CDNAML_DEVICE="cpu", OMP_NUM_THREADS="2", PYTHONPATH=ROOT,
               CDNAML_FAULT="1:all_reduce:2", CDNAML_COMM_TIMEOUT="30")
    for k in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        env.pop(k, None)
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()),
           os.path.join(HERE, "dist_worker.py"), "fault", str(out)]
    r = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=300, cwd=str(tmp_path))
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    r1 = json.loads((tmp_path / "fault.json.rank1").read_text())
    r0 = json.loads((tmp_path / "fault.json.rank0").read_text())
    assert r1["error"] and "injected fault" in r1["error"] and r1["op"] == "all_reduce" and r1["err_rank"] == 1
    assert r0["error"] and r0["err_rank"] == 0 and r0["seconds"] < 60


def test_fault_spec_parsing():
    from cdnaml.parallel.comm import _parse_fault
    assert _parse_fault("3:barrier:1") == (3, "barrier", 1)
    assert _parse_fault(None) is None
    with pytest.raises(ValueError):
        _parse_fault("3-barrier")
