"""Forest storage: the struct-of-arrays node store of an ensemble on the host, the device
tables the predictors read (node arrays, the packed predict heap), the pending bookkeeping a trainer leaves to run
while the GPU predicts (``Forest.settle``) and the frozen node lists of a tuner-cut forest."""
from __future__ import annotations

import operator
import threading
import weakref
from typing import List, Optional

import numpy as np
import torch

from ...ops import kernels as K

# single-output forests of depth <= 8 predict from a heap layout (8-byte nodes, fixed-step walks)
HEAP_PREDICT = True
# a regression forest keeps its training matrix's uint8 bins while that feature tensor lives: a transform of the
# same, unmodified tensor reads 1 byte per feature instead of 4 (FitBins; bit-identical predictions)
REUSE_FIT_BINS = True


def _tensor_key(X: torch.Tensor):
    try:
        ver = X._version
    except RuntimeError:  # inference-mode tensors carry no version counter: never matched
        return None
    return (X.data_ptr(), tuple(X.shape), tuple(X.stride()), X.dtype, str(X.device), ver)


class FitBins:
    """The bins a forest was fit on, kept for a transform of the SAME feature tensor (models/inference.py).

    A transform of the training frame (fit + transform of one DataFrame, a training-set evaluation) would
    otherwise re-read the fp32 rows the fit has just cut into uint8 bins.  The trees split on thresholds of that
    binning, and for such a threshold v:  x <= v  <=>  t_bin(x) <= v  (K.tree_predict_heap_binned), so the heap
    walk over the bins takes the same branches as over X: the predictions are bit-identical.

    ``matches(X)``: X is the fit's source tensor -- same storage pointer, shape, strides, dtype and device, the
    source still alive (a weak reference: freed memory reused by another tensor never matches) and its version
    counter unchanged since the fit (an in-place write drops the match; DataFrames are immutable, and a write through
    an alias that bypasses the version counter -- ``.data``, a DLPack / numpy view -- is not seen).

    The bins serve ONE transform (a fit is typically followed by one pass over its own frame) and are released after
    it, or as soon as the source tensor dies, so a kept model does not pin a second copy of the matrix: the next fit
    reuses their memory (holding them across fits made the allocator map a fresh 10 GB segment at 1e8 x 100, a
    240 ms stall).  Forests with categorical features or missing-value bins are never given one."""

    def __init__(self, src: torch.Tensor, bins: torch.Tensor, thresholds: np.ndarray, nthr: np.ndarray, d: int,
                 B: int):
        self._ref = weakref.ref(src)
        self._key = _tensor_key(src)
        self.bins = bins
        self.d = int(d)
        self.thr_up, = K.upload(bins.device, K.bin_upper_edges(thresholds, nthr, int(B)))
        self._lock = threading.Lock()
        self._fin = weakref.finalize(src, FitBins._release, weakref.ref(self))
        self.hits = 0

    @staticmethod
    def _release(ref) -> None:
        fb = ref()
        if fb is not None:
            fb.release()

    def release(self) -> None:
        """Drop the bins (stream-ordered: work already queued on them is unaffected)."""
        self.bins = self.thr_up = None
        self._fin.detach()

    def matches(self, X: torch.Tensor) -> bool:
        src = self._ref()
        return (src is not None and self.bins is not None and self._key is not None
                and _tensor_key(X) == self._key and _tensor_key(src) == self._key)

    def take(self, X: torch.Tensor):
        """(bins, thr_up) for a transform of X when X is the fit's tensor, released from this object at once (one
        transform per fit; of two threads transforming the frame together exactly one gets them), else None."""
        with self._lock:
            if not self.matches(X):
                return None
            out = (self.bins, self.thr_up)
            self.hits += 1
            self.release()
            return out

    def __getstate__(self):
        raise TypeError("FitBins holds device tensors of one process")


# ============================================================ forest storage
class NodeField:
    """One node field of a :class:`Forest`: list-like -- ``f[i]`` is a Python scalar (a read-only numpy row for the
    [N, k] fields ``value`` / ``catmask``), slices are lists, ``append`` / ``extend`` / item and slice assignment,
    iteration, ``==`` -- over a growable numpy array (``array()``: a view of the live nodes).  The trainer appends
    whole levels and the predictors / tuners read the arrays: no list <-> array round trips (the L07 classifier
    grid spent ~0.5 s per CrossValidator fit converting 100-tree depth-10 forests between the two)."""

    def __init__(self, dtype, width: int = 0, data=None):
        self._w = int(width)
        self._a = np.zeros((16,) if self._w == 0 else (16, self._w), dtype=dtype)
        self._ro = self._read_only()
        self._n = 0
        self.frozen = False
        if data is not None:
            self.extend(data)

    def __len__(self) -> int:
        return self._n

    def array(self) -> np.ndarray:
        """The live nodes' values (a view: read-only use)."""
        return self._a[:self._n]

    def __array__(self, dtype=None, copy=None):
        a = self._a[:self._n]
        return a.astype(dtype) if dtype is not None and a.dtype != dtype else a.copy()

    def _check(self):
        if self.frozen:
            raise TypeError("the node lists of a cut forest are immutable; build a new Forest instead")

    def _read_only(self) -> np.ndarray:
        ro = self._a.view()
        ro.flags.writeable = False  # rows handed out by [i] are read-only views
        return ro

    def _reserve(self, m: int) -> None:
        if m > len(self._a):
            b = np.zeros((max(m, 2 * len(self._a)),) + self._a.shape[1:], dtype=self._a.dtype)
            b[:self._n] = self._a[:self._n]
            self._a = b
            self._ro = self._read_only()

    def append(self, v) -> None:
        self._check()
        self._reserve(self._n + 1)
        self._a[self._n] = v
        self._n += 1

    def extend(self, vals) -> None:
        self._check()
        if isinstance(vals, NodeField):
            vals = vals.array()
        arr = np.asarray(vals, dtype=self._a.dtype)
        if self._w:
            arr = arr.reshape(-1, self._w)
        m = arr.shape[0] if arr.ndim else 0
        self._reserve(self._n + m)
        self._a[self._n:self._n + m] = arr
        self._n += m

    def _index(self, i) -> int:
        i = operator.index(i)
        if i < 0:
            i += self._n
        if not 0 <= i < self._n:
            raise IndexError("node index out of range")
        return i

    def __getitem__(self, i):
        if i.__class__ is int and 0 <= i < self._n:  # the per-node loops' case: no index normalisation
            return self._a.item(i) if self._w == 0 else self._ro[i]
        if isinstance(i, slice):
            sub = self._a[:self._n][i]
            return sub.tolist() if self._w == 0 else [r.copy() for r in sub]
        i = self._index(i)
        return self._a.item(i) if self._w == 0 else self._ro[i]

    def pop(self):
        self._check()
        v = self[self._n - 1]
        self._n -= 1
        return v

    def __setitem__(self, i, v) -> None:
        self._check()
        if isinstance(i, slice):
            self._a[:self._n][i] = np.asarray(v, dtype=self._a.dtype)
        else:
            self._a[self._index(i)] = v

    def __iter__(self):
        a = self._a[:self._n]
        return iter(a.tolist()) if self._w == 0 else iter([r.copy() for r in a])

    def __eq__(self, other) -> bool:
        o = other.array() if isinstance(other, NodeField) else np.asarray(other)
        a = self._a[:self._n]
        return a.shape == o.shape and bool(np.array_equal(a, o))

    __hash__ = None

    def __repr__(self) -> str:
        return f"NodeField({self._a[:self._n]!r})"

    def __reduce__(self):
        return (_node_field, (self._a.dtype.str, self._w, self._a[:self._n].copy(), self.frozen))


def _node_field(dtype, width, data, frozen=False):
    f = NodeField(np.dtype(dtype), width, data)
    f.frozen = frozen
    return f


def _fields(K_: int) -> dict:
    return {"feat": NodeField(np.int64), "thr": NodeField(np.float64), "bin": NodeField(np.int64),
            "left": NodeField(np.int64), "right": NodeField(np.int64), "catmask": NodeField(np.uint32, 8),
            "is_cat": NodeField(np.bool_), "value": NodeField(np.float64, max(1, K_)),
            "weight": NodeField(np.float64), "gain": NodeField(np.float64), "impurity": NodeField(np.float64),
            "depth": NodeField(np.int64)}


class Forest:
    """Struct-of-arrays node store for an ensemble (host), + cached device arrays.

    Every node field is a :class:`NodeField` (list-like over a growable numpy array): ``value[i]`` is the node's
    k outputs, ``catmask[i]`` its uint32[8] category bitmask."""

    def __init__(self, K_: int):
        # bookkeeping a trainer left to run later (settle()): the last level's node lists, appended while the
        # GPU predicts instead of between the last split and the predict launch (the node-list fields below are
        # properties that settle first, so every reader sees the complete forest)
        self._pending: list = []
        self._settling = None            # ident of the thread running settle(), or None
        self._settle_lock = threading.RLock()
        self.K = K_
        for n_, f_ in _fields(K_).items():
            self.__dict__["_" + n_] = f_
        self.roots: List[int] = []
        self._dev = {}
        self._heap_np = None  # (struct [T, 2^(D+1)-1, 2] int32, leaf values [T, 2^(D+1)-1] f64, D) built by
        # ForestTrainer.train (Forest.heap_struct's arrays), or None
        self._fit_bins: Optional[FitBins] = None

    def settle(self) -> None:
        """Run the deferred bookkeeping (idempotent; a no-op when nothing is pending).

        Re-entrant for the settling thread (the pending closures read node fields, which call back here);
        any OTHER thread blocks on the lock until the forest is complete (ForestPredictor serves worker threads)."""
        if not self._pending or self._settling == threading.get_ident():
            return
        with self._settle_lock:
            self._settling = threading.get_ident()
            try:
                while self._pending:
                    self._pending[0]()      # dequeued only once done: other threads see work pending and wait
                    self._pending.pop(0)
            finally:
                self._settling = None

    def __getstate__(self):
        self.settle()
        st = dict(self.__dict__)
        st["_pending"] = []
        st["_settling"] = None
        st.pop("_settle_lock", None)
        st.pop("_fit_bins", None)   # device bins of the training tensor: process-local
        return st

    def __setstate__(self, st):
        # forests pickled before the node fields were NodeFields hold plain lists: convert them
        K_ = int(st.get("K", 1))
        for n_, f_ in _fields(K_).items():
            v = st.get("_" + n_)
            if v is not None and not isinstance(v, NodeField):
                f_.extend(np.asarray(v, dtype=f_._a.dtype).reshape((-1,) + f_._a.shape[1:]) if len(v) else [])
                st["_" + n_] = f_
        st.pop("_np", None)
        pre = st.get("_heap_np")
        if pre is not None and len(pre) != 3:
            st["_heap_np"] = None   # an older (table, D) heap: rebuilt through heap_struct on demand
        st["_settling"] = None
        st.setdefault("_pending", [])
        st.setdefault("_fit_bins", None)
        self.__dict__.update(st)
        self.__dict__["_settle_lock"] = threading.RLock()

    def lists(self) -> dict:
        """The node-list fields (settled) as a dict name -> list, for loops that touch many nodes (one settle check
        instead of one property call per access)."""
        if self._pending:
            self.settle()
        d = self.__dict__
        return {n: d["_" + n] for n in _NODE_FIELDS}

    def add(self, value, weight, depth, impurity=float("nan")) -> int:
        if self._pending:
            self.settle()
        d = self.__dict__
        i = len(d["_feat"])
        d["_feat"].append(-1)
        d["_thr"].append(0.0)
        d["_bin"].append(0)
        d["_left"].append(-1)
        d["_right"].append(-1)
        d["_catmask"].append(0)
        d["_is_cat"].append(False)
        d["_value"].append(np.asarray(value, dtype=np.float64).reshape(-1))
        d["_weight"].append(float(weight))
        d["_gain"].append(0.0)
        d["_impurity"].append(float(impurity))
        d["_depth"].append(depth)
        return i

    def add_many(self, values: np.ndarray, weights: np.ndarray, depth: int, impurity: np.ndarray) -> np.ndarray:
        """Append N leaf nodes at once (values [N, k]); returns their ids."""
        i0, N = len(self.feat), len(weights)
        if N == 0:  # a level whose splits all failed produces no children
            return np.zeros(0, dtype=np.int64)
        values = np.asarray(values, dtype=np.float64).reshape(N, -1)
        self.feat.extend(np.full(N, -1, dtype=np.int64))
        self.thr.extend(np.zeros(N))
        self.bin.extend(np.zeros(N, dtype=np.int64))
        self.left.extend(np.full(N, -1, dtype=np.int64))
        self.right.extend(np.full(N, -1, dtype=np.int64))
        self.catmask.extend(np.zeros((N, 8), dtype=np.uint32))
        self.is_cat.extend(np.zeros(N, dtype=bool))
        self.value.extend(values)
        self.weight.extend(np.asarray(weights, dtype=np.float64))
        self.gain.extend(np.zeros(N))
        self.impurity.extend(np.asarray(impurity, dtype=np.float64))
        self.depth.extend(np.full(N, depth, dtype=np.int64))
        return np.arange(i0, i0 + N, dtype=np.int64)

    def set_splits(self, fids, feats, gains, bins, thrs, has_thr, lefts, rights) -> None:
        """Turn leaves ``fids`` into split nodes (numeric ones, ``has_thr``, also get bin + threshold).

        A level's split nodes lie in one contiguous id range (its active nodes were appended together), so each
        field is updated as one numpy slice of that range instead of a Python loop per node (the last level's
        loop ran while the GPU idled before the transform)."""
        fids = np.asarray(fids, dtype=np.int64)
        if fids.size == 0:
            return
        lo, hi = int(fids.min()), int(fids.max()) + 1
        rel = fids - lo
        h = np.asarray(has_thr, dtype=bool)
        for name, vals, sel in (("feat", feats, None), ("gain", gains, None), ("left", lefts, None),
                                ("right", rights, None), ("bin", bins, h), ("thr", thrs, h)):
            a = getattr(self, name)
            a._check()
            seg = a.array()[lo:hi]  # a view: the assignments land in the field
            v = np.asarray(vals)
            if sel is None:
                seg[rel] = v
            else:
                seg[rel[sel]] = v[sel]

    @property
    def num_nodes(self):
        return len(self.feat)

    def tree_nodes(self, t: int) -> List[int]:
        L = self.lists()
        feat, left, right = L["feat"].array(), L["left"].array(), L["right"].array()
        out, stack = [], [int(self.roots[t])]
        while stack:
            i = stack.pop()
            out.append(i)
            if feat[i] >= 0:
                stack.extend([int(right[i]), int(left[i])])
        return out

    def _layout(self, feat: Optional[np.ndarray] = None):
        """Per node: tree index (-1 if unreachable), heap slot (root 0, children 2i+1 / 2i+2) and, per tree,
        its depth -- one vectorised sweep per level instead of a Python walk per node."""
        N = len(self.feat)
        tree_of = np.full(N, -1, dtype=np.int64)
        slot = np.zeros(N, dtype=np.int64)
        T = len(self.roots)
        dep = np.zeros(T, dtype=np.int64)
        if T == 0:
            return tree_of, slot, dep
        feat = np.asarray(self.feat, dtype=np.int64) if feat is None else feat
        left = np.asarray(self.left, dtype=np.int64)
        right = np.asarray(self.right, dtype=np.int64)
        fr = np.asarray(self.roots, dtype=np.int64)
        tree_of[fr] = np.arange(T)
        level = 0
        while len(fr):
            dep[tree_of[fr]] = level
            inner = fr[feat[fr] >= 0]
            if not len(inner):
                break
            lc, rc = left[inner], right[inner]
            tree_of[lc] = tree_of[inner]
            tree_of[rc] = tree_of[inner]
            if level < 62:
                slot[lc] = 2 * slot[inner] + 1
                slot[rc] = 2 * slot[inner] + 2
            fr = np.concatenate([lc, rc])
            level += 1
        return tree_of, slot, dep

    def tree_depths(self) -> np.ndarray:
        return self._layout()[2]

    def tree_depth(self, t: int) -> int:
        return max(self.depth[i] for i in self.tree_nodes(t)) - self.depth[self.roots[t]]

    # ----------------------------------------------------------- device
    def device_arrays(self, device, values_kind: str = "value"):
        key = (str(device), values_kind)
        if key in self._dev:
            return self._dev[key]
        N = self.num_nodes
        nodes = np.zeros((N, 4), dtype=np.int32)
        L = self.lists()
        feat = L["feat"].array().astype(np.int32)
        leaf = feat < 0
        isc = L["is_cat"].array() & ~leaf
        num = ~leaf & ~isc
        left, right = L["left"].array(), L["right"].array()
        lid = np.nonzero(leaf)[0]
        V = L["value"].array()[lid] if len(lid) else np.zeros((0, self.K))
        if values_kind != "value" and len(lid):
            V = V * L["weight"].array()[lid][:, None]
        kv = V.shape[1] if V.ndim == 2 else 1
        nodes[lid, 0] = -1
        nodes[lid, 1] = np.arange(len(lid), dtype=np.int32) * kv
        cid = np.nonzero(isc)[0]
        nodes[cid, 0] = -(feat[cid] + 2)
        nodes[cid, 1] = np.arange(len(cid), dtype=np.int32)
        nid = np.nonzero(num)[0]
        nodes[nid, 0] = feat[nid]
        thr = L["thr"].array()
        nodes[nid, 1] = thr[nid].astype(np.float32).view(np.int32)
        inner = ~leaf
        nodes[inner, 2] = left[inner]
        nodes[inner, 3] = right[inner]
        vals = V.reshape(-1).astype(np.float64) if V.size else np.zeros(1, np.float64)
        masks = (L["catmask"].array()[cid].view(np.int32).reshape(-1) if len(cid) else np.zeros(8, np.int32))
        out = tuple(K.upload(device, nodes, np.asarray(self.roots, dtype=np.int32), vals, masks))
        self._dev[key] = out
        return out

    def _binned_arrays_contiguous(self, tree: int):
        """binned_arrays' tables with numpy when the tree's nodes are the contiguous id range [root, end) (a
        boosting round grows its one tree there) and it has no categorical split; else None.  The per-node Python
        loop cost ~0.45 ms per depth-8 tree, an idle GPU gap between every GBDT round's last split and its margin
        update."""
        r0 = self.roots[tree]
        r1 = self.roots[tree + 1] if tree + 1 < len(self.roots) else len(self.feat)
        if r1 - r0 < 1 or any(self.is_cat[r0:r1]):
            return None
        feat = np.asarray(self.feat[r0:r1], dtype=np.int64)
        left = np.asarray(self.left[r0:r1], dtype=np.int64)
        right = np.asarray(self.right[r0:r1], dtype=np.int64)
        sp = feat >= 0
        kids = np.concatenate([left[sp], right[sp]])
        if len(kids) != r1 - r0 - 1 or not np.array_equal(np.sort(kids), np.arange(r0 + 1, r1)):
            return None  # not exactly the nodes reachable from this root
        leaf = ~sp
        nodes = np.zeros((r1 - r0, 4), dtype=np.int32)
        nodes[:, 0] = np.where(sp, feat, -1)
        nodes[sp, 1] = np.asarray(self.bin[r0:r1], dtype=np.int64)[sp]
        nodes[sp, 2] = left[sp] - r0
        nodes[sp, 3] = right[sp] - r0
        nodes[leaf, 1] = np.arange(int(leaf.sum()))
        vals = self.value.array()[r0 + np.nonzero(leaf)[0], 0].astype(np.float32)
        return nodes, vals.reshape(-1), np.zeros(8, np.int32)

    def binned_arrays(self, device, tree: int):
        """Single tree with bin thresholds (GBDT training-set margin update)."""
        key = ("bin", str(device), tree)
        if key in self._dev:
            return self._dev[key]
        fast = self._binned_arrays_contiguous(tree)
        if fast is not None:
            out = tuple(K.upload(device, *fast))
            self._dev[key] = out
            return out
        idx = self.tree_nodes(tree)
        pos = {g: j for j, g in enumerate(idx)}
        nodes = np.zeros((len(idx), 4), dtype=np.int32)
        vals, masks = [], []
        for j, g in enumerate(idx):
            if self.feat[g] < 0:
                nodes[j] = (-1, len(vals), 0, 0)
                vals.append(float(self.value[g][0]))
            elif self.is_cat[g]:
                nodes[j] = (-(self.feat[g] + 2), len(masks), pos[self.left[g]], pos[self.right[g]])
                masks.append(self.catmask[g].view(np.int32))
            else:
                nodes[j] = (self.feat[g], self.bin[g], pos[self.left[g]], pos[self.right[g]])
        out = tuple(K.upload(device, nodes, np.asarray(vals, dtype=np.float32).reshape(-1),
                             np.concatenate(masks) if masks else np.zeros(8, np.int32)))
        self._dev[key] = out
        return out

    def heap_arrays(self, device, values_kind: str = "value"):
        """Single-output forests of depth <= 8: the packed predict heap (``K.pack_heap``: int32 [T, 2^(D+2)-2],
        internal slots {feature | -1 pass-through | -(f+2) categorical, threshold / mask-offset bits} with the
        children of slot i at 2i+1 / 2i+2, then the depth-D leaf values as fp64) plus the categorical masks, or
        None."""
        key = ("heap", str(device), values_kind)
        if key in self._dev:
            return self._dev[key]
        pre = getattr(self, "_heap_np", None)
        if values_kind == "value" and pre is not None and pre[0].shape[0] == len(self.roots):
            # filled level by level by the trainer (the same table as below; tests/test_engine_heap.py)
            h_t, m_t = K.upload(device, K.pack_heap(pre[0], pre[1], pre[2]), np.zeros(8, np.int32))
            res = (h_t, pre[2], m_t)
            self._dev[key] = res
            return res
        res = None
        hs = self.heap_struct(values_kind)
        if hs is not None:
            struct, vals, D, masks = hs
            h_t, m_t = K.upload(device, K.pack_heap(struct, vals, D), masks)
            res = (h_t, D, m_t)
        self._dev[key] = res
        return res

    def heap_struct(self, values_kind: str = "value"):
        """(struct int32 [T, 2^(D+1)-1, 2], leaf values f64 [T, 2^(D+1)-1], D, masks) of a single-output forest
        of depth <= 8 (``K.pack_heap``'s input; the trainer fills the same arrays level by level), else None."""
        feat = self.feat.array()
        tree_of, slot, dep = self._layout(feat)
        D = int(dep.max()) if self.roots else 0
        if not (self.K == 1 and self.roots and D <= 8):
            return None
        S = 2 ** (D + 1) - 1
        heap = np.zeros((len(self.roots), S, 2), dtype=np.int32)
        heap[:, :, 0] = -1
        hv = np.zeros((len(self.roots), S), dtype=np.float64)
        live = np.nonzero(tree_of >= 0)[0]
        lt, ls = tree_of[live], slot[live]
        fl = feat[live].astype(np.int32)
        leaf = fl < 0
        v = self.value.array()[live[leaf], 0]
        if values_kind != "value":
            v = v * np.asarray(self.weight, dtype=np.float64)[live[leaf]]
        hv[lt[leaf], ls[leaf]] = v
        sp = ~leaf
        isc = np.asarray(self.is_cat, dtype=bool)[live] & sp
        num = sp & ~isc
        heap[lt[num], ls[num], 0] = fl[num]
        heap[lt[num], ls[num], 1] = np.asarray(self.thr, dtype=np.float64)[live[num]].astype(
            np.float32).view(np.int32)
        cat_ids = live[isc]
        masks = self.catmask.array()[cat_ids].view(np.int32).reshape(-1)
        heap[lt[isc], ls[isc], 0] = -(fl[isc] + 2)
        heap[lt[isc], ls[isc], 1] = np.arange(len(cat_ids), dtype=np.int32)
        return heap, hv, D, (masks if len(cat_ids) else np.zeros(8, np.int32))

    def predict(self, X: torch.Tensor, tree_w: np.ndarray, base=None, values_kind="value") -> torch.Tensor:
        """[n, K] float64 predictions: base + sum_t tree_w[t] * leaf value, all fp64 in one fixed tree order on
        every device (K.ordered_tree_sum)."""
        tw, = K.upload(X.device, np.asarray(tree_w, np.float64).reshape(-1))
        if self.K == 1 and X.device.type == "cuda" and HEAP_PREDICT:
            ha = self.heap_arrays(X.device, values_kind)
            if ha is not None:
                b0 = 0.0 if base is None else float(np.asarray(base, np.float64).reshape(-1)[0])
                out = K.tree_predict_heap(X, ha[0], ha[1], tw, ha[2], b0)
                if out is not None:
                    return out
        nodes, roots, vals, masks = self.device_arrays(X.device, values_kind)
        b = None if base is None else K.upload(X.device, np.asarray(base, np.float64).reshape(-1))[0]
        return K.tree_predict(X, nodes, roots, tw, vals, masks, self.K, b)

    def predict_leaf_index(self, X: torch.Tensor) -> torch.Tensor:
        """Host reference traversal returning leaf ids [n, T] (small inputs only)."""
        Xn = X.double().cpu().numpy()
        out = np.zeros((Xn.shape[0], len(self.roots)), dtype=np.int64)
        for t, r in enumerate(self.roots):
            for i in range(Xn.shape[0]):
                j = r
                while self.feat[j] >= 0:
                    x = Xn[i, self.feat[j]]
                    if self.is_cat[j]:
                        c = int(x)
                        go_left = 0 <= c < 256 and (int(self.catmask[j][c >> 5]) >> (c & 31)) & 1
                    else:
                        go_left = x <= self.thr[j]
                    j = self.left[j] if go_left else self.right[j]
                out[i, t] = j
        return torch.from_numpy(out)

    # ----------------------------------------------------------- persistence
    def state(self, prefix="forest_"):
        L = self.lists()
        dt = {"feat": np.int32, "bin": np.int32, "left": np.int32, "right": np.int32, "depth": np.int32}
        out = {prefix + n: torch.from_numpy(np.array(L[n].array(), dtype=dt.get(n, L[n].array().dtype)))
               for n in _NODE_FIELDS}
        out[prefix + "catmask"] = torch.from_numpy(L["catmask"].array().view(np.int32).copy())
        out[prefix + "roots"] = torch.tensor(list(self.roots), dtype=torch.int32)
        return out

    @classmethod
    def from_state(cls, st, prefix="forest_"):
        vals = st[prefix + "value"].numpy()
        f = cls(vals.shape[1] if vals.ndim == 2 else 1)
        for n in _NODE_FIELDS:
            a = st[prefix + n].numpy()
            setattr(f, n, a.view(np.uint32) if n == "catmask" else a)
        f.roots = st[prefix + "roots"].tolist()
        return f

    def feature_importances(self, d: int, trees: Optional[List[int]] = None) -> np.ndarray:
        """Spark semantics: per-tree gain×count, normalised per tree, averaged, normalised."""
        total = np.zeros(d)
        trees = range(len(self.roots)) if trees is None else trees
        L = self.lists()
        feat, gain, weight = L["feat"].array(), L["gain"].array(), L["weight"].array()
        for t in trees:
            imp = np.zeros(d)
            for i in self.tree_nodes(t):
                if feat[i] >= 0:
                    imp[feat[i]] += gain[i] * weight[i]
            s = imp.sum()
            if s > 0:
                imp /= s
            total += imp
        s = total.sum()
        return total / s if s > 0 else total


def _settled_list(name: str):
    key = "_" + name

    def get(self):
        if self._pending:
            self.settle()
        return self.__dict__[key]

    def set_(self, v):
        cur = self.__dict__[key]
        f = NodeField(cur._a.dtype, cur._w)
        f.extend(v)
        self.__dict__[key] = f
    return property(get, set_)


class _FrozenList(list):
    """The root list of a forest cut by the fused tuner (truncate_forest): reads are plain list reads; every
    in-place mutation raises (the cut shares its node layout with the models the tuner scores)."""

    def _frozen(self, *a, **k):
        raise TypeError("the node lists of a cut forest are immutable; build a new Forest instead")

    __setitem__ = __delitem__ = __iadd__ = __imul__ = append = extend = insert = pop = remove = clear = \
        sort = reverse = _frozen

    def __reduce__(self):  # pickle / deepcopy rebuild from a plain list (the default would extend())
        return (_FrozenList, (list(self),))


def freeze_cut(forest: "Forest") -> None:
    """Freeze a cut forest's node fields and roots (in-place mutations raise; reassigning a field still works)."""
    d = forest.__dict__
    for n in _NODE_FIELDS:
        d["_" + n].frozen = True
    d["roots"] = _FrozenList(d["roots"])


_NODE_FIELDS = ("feat", "thr", "bin", "left", "right", "catmask", "is_cat", "value", "weight", "gain", "impurity",
                "depth")
for _name in _NODE_FIELDS:
    setattr(Forest, _name, _settled_list(_name))
del _name


def _forest_level_ops(forest, add_args, split_args, first_id, count):
    """One level's forest bookkeeping (ForestTrainer.train defers it to the next level's decision sync): append
    the children, then turn the split nodes into splits pointing at them."""
    got = forest.add_many(*add_args)
    assert len(got) == count and (not count or got[0] == first_id)
    forest.set_splits(*split_args)


from ...ops import tune as _tune  # noqa: E402  (CDNAML_TUNE overrides of the constants above)
_tune.apply(__import__(__name__, fromlist=["_"]))
