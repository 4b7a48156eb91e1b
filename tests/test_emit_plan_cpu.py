"""The host record-emission plan (K.emit_plan_host, twin of split.hip emit_plan_kernel) builds exactly the nodes the
engine's subtraction rule builds (engine._built_nodes), numbered in active order, with CH-aligned capacities."""
import numpy as np

from cdnaml.models.tree.engine import _built_nodes
from cdnaml.ops import kernels as K


def test_emit_plan_host_matches_engine_rule():
    rng = np.random.default_rng(0)
    for trial in range(50):
        A = int(rng.integers(1, 300))
        wl = rng.integers(1, 40, A).astype(float)
        wr = np.where(rng.random(A) < 0.25, wl, rng.integers(1, 40, A)).astype(float)
        act = rng.random(2 * A) < 0.7
        child = np.full(2 * A, -1, np.int64)
        child[act] = np.arange(int(act.sum()))
        ch, padb = 16, 16 * 5
        cslot, start, cap = K.emit_plan_host(wl, wr, child, ch, padb)
        # the engine's view of the next level: active children in (node, side) order with sibling links
        w_all = np.stack([wl, wr], 1).reshape(-1)[act]
        pos = np.full(2 * A, -1)
        pos[act] = np.arange(int(act.sum()))
        lp, rp = pos[0::2], pos[1::2]
        both = (lp >= 0) & (rp >= 0)
        sib = np.full(int(act.sum()), -1)
        sib[lp[both]] = rp[both]
        sib[rp[both]] = lp[both]
        parent = np.where(sib >= 0, 0, -1)
        build = _built_nodes(w_all, sib, parent)
        ids = np.nonzero(build)[0]
        exp = np.full(2 * A, -1)
        exp[np.nonzero(act)[0][ids]] = np.arange(len(ids))
        np.testing.assert_array_equal(cslot, exp)
        assert np.all(cap % ch == 0) and np.all(start % ch == 0)
        np.testing.assert_array_equal(cap, np.ceil(w_all[ids] / ch).astype(np.int64) * ch + padb)
        assert np.all(cap >= w_all[ids] + padb)


def test_emit_chunk_bounds():
    assert K.emit_chunk(0, 4096, 100) == 8
    assert K.emit_chunk(1e12, 4096, 1) == 128
    per = 5.7e8 / (4096 * 160)
    ch = K.emit_chunk(5.7e8, 4096, 160)
    assert ch * 16 <= per < ch * 32 or ch == 128
