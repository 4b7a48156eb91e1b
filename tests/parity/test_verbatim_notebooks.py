"""Verbatim notebook runs: every code cell of every reference notebook in the
Solutions tree -- lectures, labs and electives -- is executed UNCHANGED through ``cdnaml.compat`` and the
notebook runtime (``cdnaml.utils.notebook``: the Databricks globals, ``%run ./Includes/Classroom-Setup``,
``%sql`` cells, the ``dbfs:/`` / ``/dbfs/`` namespace) on the synthetic course datasets at 5 % scale.

The notebooks are read from the on-disk reference (``CDNAML_REFERENCE_DIR`` or
``/root/reference/Scalable-Machine-Learning-with-Apache-Spark``); nothing is vendored and the tests skip when it
is absent.  Cells allowed to fail are listed in ``ALLOW`` with the reason; every other cell must pass.

CPU: the notebooks run in 4 worker processes (each one DBFS root / tracking store / warehouse per notebook).
GPU (``-m gpu``): all notebooks run in THIS process on ``cuda`` so the HIP library is the one that executes.
"""
import json
import os
import subprocess
import sys

import pytest

from tests.conftest import ROOT, session_device

REF = os.environ.get("CDNAML_REFERENCE_DIR", "/root/reference/Scalable-Machine-Learning-with-Apache-Spark")
SOL = os.path.join(REF, "Solutions")
SCALE = 0.05

# (notebook, first line of the failing cell) -> reason.  Only environment limits belong here.
ALLOW = {
    ("ML 08L - Hyperopt Lab.py", 95): "sklearn 1.7 rejects RandomForestRegressor(max_features='auto') "
                                      "(removed in sklearn 1.3); the lab targets sklearn 0.24",
}
# Not run at all: MLE 04 needs fbprophet/statsmodels (out of scope); MLE 05 has no code cells.
SKIP = {"MLE 04 - Time Series Forecasting.py", "MLE 05 - Databricks Best Practices.py"}


def _notebooks():
    if not os.path.isdir(SOL):
        return []
    out = []
    for sub in ("", "Labs", "ML Electives"):
        d = os.path.join(SOL, sub)
        for f in sorted(os.listdir(d)):
            if f.endswith(".py") and (f.startswith("ML ") or f.startswith("MLE ")) and f not in SKIP:
                out.append(os.path.join(sub, f) if sub else f)
    return out


NOTEBOOKS = _notebooks()
pytestmark = pytest.mark.skipif(not NOTEBOOKS, reason=f"reference notebooks not found under {SOL}")


def _check(res):
    name = os.path.basename(res["path"])
    assert not res["setup_error"], res["setup_error"]
    bad = [c for c in res["cells"] if not c["ok"] and (name, c["line"]) not in ALLOW]
    msg = "\n".join(f"cell {c['index']} (L{c['line']}) {c['first_line']!r}: {c['error'][:600]}" for c in bad)
    assert not bad, f"{name}: {len(bad)} failing cell(s)\n{msg}"
    assert res["n_ok"] > 0 or name.startswith("ML 00a"), f"{name}: no code cell ran"


@pytest.fixture(scope="module")
def cpu_results(tmp_path_factory):
    """Run every notebook on the host in 4 worker processes; {relative notebook path: result}."""
    if not NOTEBOOKS:
        return {}
    work = tmp_path_factory.mktemp("verbatim_cpu")
    groups = [NOTEBOOKS[i::4] for i in range(4)]
    env = dict(os.environ, CDNAML_DEVICE="cpu", PYTHONPATH=ROOT + os.pathsep + os.environ.get("PYTHONPATH", ""),
               OMP_NUM_THREADS="2", MKL_NUM_THREADS="2", MPLBACKEND="Agg")
    procs = []
    for gi, g in enumerate(groups):
        out = str(work / f"g{gi}.json")
        cmd = [sys.executable, "-m", "cdnaml.utils.notebook", "--scale", str(SCALE), "--workdir",
               str(work / f"g{gi}"), "--json", out] + [os.path.join(SOL, p) for p in g]
        log = open(str(work / f"g{gi}.log"), "w")
        procs.append((subprocess.Popen(cmd, env=env, stdout=log, stderr=subprocess.STDOUT, cwd=str(work)), out,
                      log, g))
    results = {}
    for p, out, log, g in procs:
        try:
            p.wait(timeout=1500)
        except subprocess.TimeoutExpired:
            p.kill()
            p.wait()
        log.close()
        if os.path.exists(out):
            with open(out) as f:
                for r in json.load(f):
                    results[os.path.relpath(r["path"], SOL)] = r
        for nb in g:
            results.setdefault(nb, {"path": nb, "cells": [], "n_ok": 0,
                                    "setup_error": f"worker exited {p.returncode}; log {log.name}"})
    return results


@pytest.mark.parametrize("notebook", NOTEBOOKS)
def test_notebook_verbatim_cpu(notebook, cpu_results):
    _check(cpu_results[notebook])


@pytest.mark.gpu
def test_notebooks_verbatim_cuda(tmp_path):
    """Every notebook on the MI355X in this process (the HIP library loaded here does the work)."""
    import cdnaml.compat as compat
    from cdnaml.ops import _lib
    from cdnaml.utils import notebook as N

    with session_device("cuda"):
        _lib.lib()
        env0 = {k: os.environ.get(k) for k in ("CDNAML_DBFS_ROOT", "CDNAML_TRACKING_URI", "MPLBACKEND")}
        os.environ["MPLBACKEND"] = "Agg"
        compat.install()
        try:
            res = N.run_many([os.path.join(SOL, p) for p in NOTEBOOKS], str(tmp_path), SCALE, verbose=True)
        finally:
            compat.uninstall()
            for k, v in env0.items():
                if v is None:
                    os.environ.pop(k, None)
                else:
                    os.environ[k] = v
    errors = []
    for r in res:
        try:
            _check(r.to_json())
        except AssertionError as e:
            errors.append(str(e))
    assert not errors, "\n\n".join(errors)
