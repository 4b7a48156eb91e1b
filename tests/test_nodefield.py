"""Forest node storage (cdnaml/models/tree/forest.py NodeField): the list-like face over growable numpy arrays that
the trainer, the tuner's cuts, the predictors and the model summaries share."""
import pickle

import numpy as np
import pytest

from cdnaml.models.tree.forest import Forest, NodeField, freeze_cut


def test_scalar_field_is_list_like():
    f = NodeField(np.int64)
    f.append(3)
    f.extend([4, 5])
    f.extend(np.arange(6, 40))  # grows past the initial capacity
    assert len(f) == 37 and f[0] == 3 and f[-1] == 39 and type(f[1]) is int
    assert f[np.int64(2)] == 5
    assert f[1:4] == [4, 5, 6]
    f[0] = 9
    f[1:3] = [7, 7]
    assert list(f)[:4] == [9, 7, 7, 6]
    assert f == [9, 7, 7] + list(range(6, 40))
    assert f.pop() == 39 and len(f) == 36
    with pytest.raises(IndexError):
        f[36]
    a = np.asarray(f)
    a[0] = -1  # __array__ hands out a copy
    assert f[0] == 9
    assert f.array().base is not None and f.array()[0] == 9  # array(): a view of the live nodes


def test_row_field_rows_are_read_only_views():
    v = NodeField(np.float64, 3)
    v.append([1.0, 2.0, 3.0])
    v.extend(np.ones((2, 3)))
    r = v[0]
    assert r.tolist() == [1.0, 2.0, 3.0]
    with pytest.raises(ValueError):
        r[0] = 5.0
    v[1] = np.array([4.0, 5.0, 6.0])
    assert v[1].tolist() == [4.0, 5.0, 6.0] and v.array().shape == (3, 3)
    assert [x.tolist() for x in v[1:]] == [[4.0, 5.0, 6.0], [1.0, 1.0, 1.0]]


def test_frozen_field_and_pickle():
    f = NodeField(np.float64, data=[0.5, 1.5])
    f.frozen = True
    for op in (lambda: f.append(1.0), lambda: f.extend([1.0]), lambda: f.__setitem__(0, 2.0), lambda: f.pop()):
        with pytest.raises(TypeError):
            op()
    g = pickle.loads(pickle.dumps(f))
    assert g == f and g.frozen and type(g[0]) is float


def test_forest_fields_round_trip_and_cut_freeze():
    fo = Forest(2)
    ids = fo.add_many(np.array([[0.1, 0.9], [0.7, 0.3], [0.5, 0.5]]), np.array([3.0, 2.0, 1.0]), 0,
                      np.zeros(3))
    fo.roots = [0]
    fo.set_splits([0], [4], [0.25], [7], [1.5], [True], [1], [2])
    assert ids.tolist() == [0, 1, 2]
    assert fo.feat == [4, -1, -1] and fo.thr[0] == 1.5 and fo.bin[0] == 7 and fo.left[0] == 1
    assert fo.value[2].tolist() == [0.5, 0.5] and fo.catmask[1].shape == (8,)
    back = Forest.from_state(fo.state())
    assert back.feat == fo.feat and back.value == fo.value and back.roots == [0]
    freeze_cut(fo)
    with pytest.raises(TypeError):
        fo.thr[0] = 2.0
    fo.thr = [t + 0.0 for t in fo.thr]  # reassigning a field still works (a fresh, unfrozen field)
    fo.thr[0] = 2.0
    assert fo.thr[0] == 2.0


def test_forest_pickled_with_list_fields_still_loads():
    """A forest pickled when the node fields were plain lists (before NodeField) unpickles into NodeFields."""
    fo = Forest(1)
    fo.add_many(np.array([[0.5], [1.5]]), np.array([2.0, 1.0]), 0, np.zeros(2))
    fo.roots = [0]
    st = fo.__getstate__()
    old = dict(st)
    for n in ("feat", "thr", "bin", "left", "right", "is_cat", "weight", "gain", "impurity", "depth"):
        old["_" + n] = list(st["_" + n])
    old["_value"] = [np.array([0.5]), np.array([1.5])]
    old["_catmask"] = [np.zeros(8, np.uint32)] * 2
    old["_heap_np"] = (np.zeros((1, 6), np.int32), 1)        # the pre-r5 (table, D) heap
    old["_settling"] = False                                  # the pre-r6 bool flag, no lock
    f2 = Forest.__new__(Forest)
    f2.__setstate__(old)
    assert isinstance(f2.value, NodeField) and f2.value[1].tolist() == [1.5] and f2.feat == [-1, -1]
    assert f2.catmask.array().shape == (2, 8)
    assert f2._heap_np is None and f2._settling is None
    f2.settle()
    import copy
    f3 = copy.deepcopy(f2)
    assert f3.feat == [-1, -1] and f3._settle_lock is not f2._settle_lock


def test_forest_settle_blocks_other_threads():
    """A reader on another thread waits for the settling thread instead of reading a half-built forest
    (settle() was guarded by a flag, not a lock)."""
    import threading
    import time

    fo = Forest(1)
    fo.roots = [0]
    started = threading.Event()

    def slow_level():
        started.set()
        time.sleep(0.2)
        fo.add(np.array([0.5]), 1.0, 0)
    fo._pending.append(slow_level)
    t = threading.Thread(target=fo.settle)
    t.start()
    started.wait()
    n = len(fo.lists()["feat"])   # blocks until the settling thread finished
    t.join()
    assert n == 1
