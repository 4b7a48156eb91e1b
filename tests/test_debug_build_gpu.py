"""The checked HIP build (CDNAML_HIP_DEBUG=1 -> cdnaml/_native/libcdnaml_hip_debug.so, -O1 -g -DCDNA_DEBUG,
SURVEY §5.2): a clean forest fit + transform passes its device bounds checks, and a corrupted forest (a split
feature outside the row) is reported as a bounds-check failure instead of an out-of-range access."""
import os
import subprocess
import sys

import pytest
import torch

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

SCRIPT = r"""
import numpy as np, torch
import cdnaml
from cdnaml.ops import _lib, kernels as K
assert _lib.DEBUG and _lib.LIB_PATH.endswith("libcdnaml_hip_debug.so")
spark = cdnaml.SparkSession.builder.getOrCreate()
from cdnaml.models.regression import RandomForestRegressor
g = torch.Generator(device="cuda").manual_seed(0)
X = torch.randn((200_000, 24), generator=g, device="cuda")
y = (X[:, 0] * 2 - X[:, 1] + (X[:, 2] > 0).float()).double()
df = spark.createDataFrameFromLocalTensors({"features": X, "label": y})
m = RandomForestRegressor(numTrees=20, maxDepth=5, maxBins=40, seed=1).fit(df)   # record / partition7 paths
p = m.transform(df)._plan.execute()[0].columns["prediction"].values
torch.cuda.synchronize()
assert torch.isfinite(p).all()
heap, D, masks = m._forest.heap_arrays(X.device)
bad = heap.clone()
bad[0, 0] = 24 + 5                                      # root split on feature 29 of a 24-feature row
tw = torch.full((heap.shape[0],), 1.0 / heap.shape[0], device="cuda", dtype=torch.float64)
try:
    K.tree_predict_heap(X, bad, D, tw, masks, 0.0)
    torch.cuda.synchronize()
    K.reg_metrics(y, y)       # any later checked call reports it too
    raise SystemExit("no bounds-check failure reported")
except RuntimeError as e:
    assert "bounds check 0x7E02" in str(e), e
print("debug build ok")
"""


def test_checked_build_fit_and_bounds_report(tmp_path):
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    env = dict(os.environ, CDNAML_HIP_DEBUG="1")
    r = subprocess.run([sys.executable, "-c", SCRIPT], env=env, cwd=ROOT, capture_output=True, text=True,
                       timeout=600)
    assert r.returncode == 0 and "debug build ok" in r.stdout, r.stdout[-2000:] + r.stderr[-3000:]
