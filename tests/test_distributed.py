"""Multi-process SPMD correctness on CPU (gloo, world_size 2): the distributed
engine must give the single-process answers."""
import json
import os
import socket
import subprocess
import sys

import pytest

# every test here launches torchrun process groups (about 4 of the CPU suite's 5 minutes): the tight iteration loop
# is `pytest tests -m "not gpu and not slow"`
pytestmark = pytest.mark.slow

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _port_clash(err: str) -> bool:
    """The free port picked by _free_port was taken before torchrun bound it (a launch race, not a test
    failure): retried once on a fresh port."""
    return any(k in err for k in ("Address already in use", "EADDRINUSE", "address already in use"))


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
    if r.returncode != 0 and nproc > 1 and _port_clash(r.stderr):
        cmd[cmd.index("--master-port") + 1] = str(_free_port())
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


def _bench(tmp_path, nproc, rows="3e4", extra=(), env_extra=None):
    env = dict(os.environ, CDNAML_DEVICE="cpu", OMP_NUM_THREADS="1", PYTHONPATH=ROOT, **(env_extra or {}))
    for k in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        env.pop(k, None)
    args = [os.path.join(ROOT, "bench.py"), "--gpus", str(nproc), "--rows", rows, "--steps", "1", "--warmup", "0",
            *extra]
    if nproc == 1:
        cmd = [sys.executable] + args
    else:
        cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={nproc}",
               "--master-addr", "127.0.0.1", "--master-port", str(_free_port())] + args
    r = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=600, cwd=str(tmp_path))
    if r.returncode != 0 and nproc > 1 and _port_clash(r.stderr):
        cmd[cmd.index("--master-port") + 1] = str(_free_port())
        r = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=600, cwd=str(tmp_path))
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    line = [ln for ln in r.stdout.splitlines() if ln.startswith("{")][-1]
    res = json.loads(line)
    assert res["n_gpus"] == nproc and res["steps"] == 1 and res["config"]["parallelism"] == f"dp{nproc}"
    tail = [ln for ln in r.stderr.splitlines() if "digest=" in ln][-1]
    return res, tail.split("nodes=")[1]


def test_bench_trains_identical_forest_on_1_2_4_8_ranks(tmp_path):
    """The headline bench itself under torch.distributed.run (gloo) at W = 1, 2, 4, 8: the data is keyed by
    global row id and the level histograms are int64 fixed-point sums all-reduced exactly (the same integer
    path RCCL ranks take: item records, raw segment histograms, one global quantisation scale), so every
    world size must print the same node count and forest digest."""
    ref = None
    for w in (1, 2, 4, 8):
        # W = 2 and 8 build every level in slot chunks whose all-reduces overlap the next chunk
        # (_hist_overlapped; by default only for level histograms of >= 64 MiB)
        ov = {"CDNAML_TUNE": "HIST_OVERLAP_MIN_BYTES=0"} if w in (2, 8) else None
        res, tag = _bench(tmp_path, w, env_extra=ov)
        if ref is None:
            ref = tag
        assert tag == ref, (w, tag, ref)


@pytest.mark.parametrize("scenario,worlds", [("trees", (2, 4)), ("trees_uneven", (2, 4)), ("trees_deep", (2, 3)),
                                             ("cv", (2,)),
                                             ("als", (2, 4)), ("hyperopt", (2,)),
                                             ("hyperopt_captured", (2,))])
def test_models_identical_across_world_sizes(scenario, worlds, tmp_path):
    """RF (T=20), DecisionTree, GBT, XGBoost regressor (packed unit-hessian path) and classifier (hessian
    path), RF classifier, CrossValidator and ALS at W ranks equal the 1-rank fit (tree models bit-identical;
    block ALS factors (explicit, implicit, nonnegative) to 1e-6), including shards that are empty or imbalanced."""
    one = _run(scenario, tmp_path, 1)
    for w in worlds:
        got = _run(scenario, tmp_path, w)
        if scenario == "als":
            assert got["block"]
            for key in ("uf", "vf", "uf_implicit", "vf_implicit", "uf_nonneg", "vf_nonneg"):
                # fp32 model factors of fp64 solves that differ only in summation order
                assert got[key] == pytest.approx(one[key], abs=1e-6), (w, key)
        else:
            assert got == one, (w, got, one)


def test_reduce_scatter_by_feature_forests_identical(tmp_path):
    """Verdict r2 item 9: level histograms reduce-scattered by feature (K6 on each rank's slice, winners
    all-gathered) give the 1-rank forests bit for bit at W = 2, 4 and 8."""
    one = _run("trees_rs", tmp_path, 1)
    assert one.pop("rs_levels") == 0
    for w in (2, 4, 8):
        got = _run("trees_rs", tmp_path, w)
        assert got.pop("rs_levels") > 0, w
        assert got == one, w


def test_reduce_scatter_with_overlap_enabled(tmp_path):
    """the chunked overlap composes with reduce-scatter by feature (each slot chunk's
    histogram reduce-scattered asynchronously while the next builds, the parents cut to the rank's feature slice);
    forests equal the 1-rank fits at W = 2, 4 and 8, with the RF headline shape scaled down and a depth-8 / 256-bin
    GBDT overlapped + reduce-scattered at every level."""
    one = _run("trees_rs_overlap", tmp_path, 1)
    for tag in ("a", "b", "c"):
        assert one.pop(f"{tag}_levels") == {"rs": 0, "ov": 0, "ov_rs": 0}
    for w in (2, 4, 8):
        got = _run("trees_rs_overlap", tmp_path, w)
        la, lb, lc = got.pop("a_levels"), got.pop("b_levels"), got.pop("c_levels")
        assert la["ov"] > la["ov_rs"] > 0, (w, la)          # overlapped all-reduce at the shallow levels, RS below
        assert lb["rs"] > 0 and lb["ov_rs"] > 0, (w, lb)    # RS from level 0, deeper levels overlapped RS
        assert lc["ov"] == lc["ov_rs"] > 0, (w, lc)         # every multi-slot level overlapped + RS
        assert got == one, w


def test_overlapped_reduce_scatter_trace(tmp_path):
    """The Chrome trace of a 2-rank gloo fit shows each chunk's tree.reduce_scatter in flight while a later
    tree.hist_chunk runs (the overlap is real, not serialised)."""
    got = _run("trace_rs_overlap", tmp_path, 2)
    assert got["rs_spans"] > 0 and got["chunk_spans"] > 0
    assert got["overlapping"] > 0, got


def test_ooc_fit_with_an_empty_shard(tmp_path):
    """the streamed / materialised choice is agreed over ranks, and a rank without chunks streams an
    empty shard -- no rank falls back alone (different collectives would hang the fit)."""
    one = _run("ooc_uneven", tmp_path, 1)
    assert one["streamed"] == 2
    for w in (2, 3):
        got = _run("ooc_uneven", tmp_path, w)
        assert got == one, (w, got, one)


def test_rccl_branches_through_recording_fake(tmp_path):
    """the RCCL branches of Comm (never run by gloo CI) through tests/fake_nccl.py -- a
    recording nccl-over-gloo torch.distributed proxy that checks contiguity, dtypes, in/out sizes and split
    sums of every call.  Direct collective checks, then the reduce-scatter-by-feature forests at W = 2 and 4,
    which must equal the 1-rank (gloo) fits bit for bit."""
    one = _run("trees_rs", tmp_path, 1)
    assert one.pop("rs_levels") == 0
    for w in (2, 4):
        got = _run("trees_rs_nccl", tmp_path, w)
        assert got.pop("backend") == "nccl"
        assert got.pop("violations") == [], w
        for k in ("rs_ok", "rs_noncontig_ok", "ag_ok", "ar_async_ok", "a2a_ok", "rs_async_ok", "overlap_same"):
            assert got.pop(k) is True, (w, k)
        rec = got.pop("record_min")
        assert rec.get("reduce_scatter_tensor", 0) > 0 and rec.get("all_gather_into_tensor", 0) > 0, (w, rec)
        assert rec.get("reduce_scatter_tensor_async", 0) > 0, (w, rec)
        assert rec.get("barrier", 0) > 0, (w, rec)
        assert got.pop("rs_levels") > 0, w
        assert got == one, w
