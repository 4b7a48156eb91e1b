"""K7e: the partition writes the next level's item records itself (hist5.hip partition7 EMIT + split.hip emit_plan)
instead of a codes_count_w + codes_scatter_w pass.  The level histograms are exact int64 sums whatever the record
order, so forests grown on emitted records must equal the compaction path's forests bit for bit; the checked build
also compares the device capacity plan with the host's and the emitted records per slot with the compaction's."""
import os
import subprocess
import sys

import numpy as np
import pytest
import torch

from cdnaml.ops import _lib, kernels as K

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope="module")
def spark():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    _lib.lib()
    import cdnaml
    return cdnaml.SparkSession.builder.getOrCreate()


def _fit(spark, n, d, T, depth, seed, emit, **kw):
    from cdnaml.models.regression import RandomForestRegressor
    from cdnaml.utils.synthetic import forest_digest
    g = torch.Generator(device="cuda").manual_seed(seed)
    X = torch.randn((n, d), generator=g, device="cuda")
    y = (X[:, 0] * 2 - X[:, 1] + torch.sin(3 * X[:, 2]) + 0.3 * X[:, 3] * X[:, 4]).double()
    df = spark.createDataFrameFromLocalTensors({"features": X, "label": y})
    calls = {"plan": 0}
    orig = K.RecordEmit.plan

    def plan(self, so, child):
        calls["plan"] += 1
        return orig(self, so, child)
    old = K.EMIT_RECORDS
    K.EMIT_RECORDS = emit
    K.RecordEmit.plan = plan
    try:
        m = RandomForestRegressor(numTrees=T, maxDepth=depth, maxBins=40, seed=seed, **kw).fit(df)
    finally:
        K.EMIT_RECORDS = old
        K.RecordEmit.plan = orig
    return forest_digest(m._forest), calls["plan"]


@pytest.mark.parametrize("n,d,T,depth", [(300_000, 100, 20, 6), (120_003, 96, 17, 5), (200_000, 100, 24, 8)])
def test_emitted_records_grow_the_compaction_forest(spark, n, d, T, depth):
    ref, c0 = _fit(spark, n, d, T, depth, 7, False)
    got, c1 = _fit(spark, n, d, T, depth, 7, True)
    assert c0 == 0 and c1 >= 2, (c0, c1)  # the partitions of levels 1 .. depth-2 emit (<= 256 active nodes)
    assert got == ref


def test_emit_plan_matches_host_plan(spark):
    """emit_plan_kernel against emit_plan_host on random decisions (ties, lone children, leaves)."""
    rng = np.random.default_rng(3)
    A = 200
    so = np.zeros((A, 8))
    so[:, 3] = rng.integers(1, 50, A)
    so[:, 5] = np.where(rng.random(A) < 0.2, so[:, 3], rng.integers(1, 50, A))
    act = rng.random(2 * A) < 0.8
    child = np.full(2 * A, -1, np.int32)
    child[act] = np.arange(int(act.sum()))
    em = K.RecordEmit(torch.device("cuda"), 1000, A, torch.empty(1, dtype=torch.int64, device="cuda"),
                      torch.zeros(1000, device="cuda"), 1.0, 16, 7)
    em.plan(torch.from_numpy(so).cuda(), torch.from_numpy(child).cuda())
    cs, st, cap = K.emit_plan_host(so[:, 3], so[:, 5], child, 16, em.padb)
    S = len(st)
    assert int(em.nslots.item()) == S
    np.testing.assert_array_equal(em.cslot.cpu().numpy(), cs)
    np.testing.assert_array_equal(em.seg_start[:S].cpu().numpy(), st)
    np.testing.assert_array_equal(em.seg_lim[:S].cpu().numpy(), st + cap)
    np.testing.assert_array_equal(em.cursor.view(-1, em.cs)[:S, 0].cpu().numpy(), st)


SCRIPT = r"""
import numpy as np, torch
import cdnaml
from cdnaml.ops import _lib, kernels as K
from cdnaml.models.tree import engine
assert _lib.DEBUG
spark = cdnaml.SparkSession.builder.getOrCreate()
from cdnaml.models.regression import RandomForestRegressor
g = torch.Generator(device="cuda").manual_seed(1)
X = torch.randn((150_000, 100), generator=g, device="cuda")
y = (X[:, 0] * 2 - X[:, 1] + (X[:, 2] > 0).float()).double()
df = spark.createDataFrameFromLocalTensors({"features": X, "label": y})
calls = {"n": 0}
orig = engine.ForestTrainer._check_emitted
def counted(*a):
    calls["n"] += 1
    return orig(*a)
engine.ForestTrainer._check_emitted = staticmethod(counted)
m = RandomForestRegressor(numTrees=20, maxDepth=5, maxBins=40, seed=3).fit(df)
assert calls["n"] == 3, calls["n"]
print("emit checked ok")
"""


def test_emit_checked_build(tmp_path):
    """Checked build (engine._check_emitted at every emitting level): the device plan equals the host plan, the
    segments stay inside their capacities, and each slot's records minus the zero-weight padding are exactly the
    compaction's records of the same codes."""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    env = dict(os.environ, CDNAML_HIP_DEBUG="1", CDNAML_P7_EMIT="1")
    r = subprocess.run([sys.executable, "-c", SCRIPT], env=env, cwd=ROOT, capture_output=True, text=True,
                       timeout=600)
    assert r.returncode == 0 and "emit checked ok" in r.stdout, r.stdout[-2000:] + r.stderr[-3000:]
