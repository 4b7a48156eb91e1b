"""Forest storage: the struct-of-arrays node store of an ensemble on the host, the device
tables the predictors read (node arrays, the packed predict heap), the pending bookkeeping a trainer leaves to run
while the GPU predicts (``Forest.settle``) and the frozen node lists of a tuner-cut forest."""
from __future__ import annotations

from typing import List, Optional

import numpy as np
import torch

from ...ops import kernels as K

# single-output forests of depth <= 8 predict from a heap layout (8-byte nodes, fixed-step walks)
HEAP_PREDICT = True
# predictor tables of tuner-cut forests from the arrays truncate_forest computed (0: from the node lists)
CUT_ARRAYS = True


# ============================================================ forest storage
_ZERO_MASK = np.zeros(8, dtype=np.uint32)
_ZERO_MASK.flags.writeable = False


class Forest:
    """Struct-of-arrays node store for an ensemble (host), + cached device arrays.

    ``value[i]``: the node's k outputs (a float sequence: numpy array or list); ``catmask[i]``: uint32[8] bitmask
    (leaves share one read-only zero mask)."""

    def __init__(self, K_: int):
        # bookkeeping a trainer left to run later (settle()): the last level's node lists, appended while the
        # GPU predicts instead of between the last split and the predict launch (the node-list fields below are
        # properties that settle first, so every reader sees the complete forest)
        self._pending: list = []
        self._settling = False
        self.K = K_
        self.feat: List[int] = []
        self.thr: List[float] = []
        self.bin: List[int] = []
        self.left: List[int] = []
        self.right: List[int] = []
        self.catmask: List[np.ndarray] = []
        self.is_cat: List[bool] = []
        self.value: List[np.ndarray] = []
        self.weight: List[float] = []
        self.gain: List[float] = []
        self.impurity: List[float] = []
        self.depth: List[int] = []
        self.roots: List[int] = []
        self._dev = {}
        self._heap_np = None  # (struct [T, 2^(D+1)-1, 2] int32, leaf values [T, 2^(D+1)-1] f64, D) built by
        # ForestTrainer.train (Forest.heap_struct's arrays), or None

    def settle(self) -> None:
        """Run the deferred bookkeeping (idempotent; a no-op when nothing is pending)."""
        if self._settling:
            return
        self._settling = True
        try:
            while self._pending:
                self._pending.pop(0)()
        finally:
            self._settling = False

    def __getstate__(self):
        self.settle()
        st = dict(self.__dict__)
        st["_pending"] = []
        return st

    def lists(self) -> dict:
        """The node-list fields (settled) as a dict name -> list, for loops that touch many nodes (one settle check
        instead of one property call per access)."""
        if self._pending and not self._settling:
            self.settle()
        d = self.__dict__
        return {n: d["_" + n] for n in _NODE_FIELDS}

    def add(self, value, weight, depth, impurity=float("nan")) -> int:
        if self._pending and not self._settling:
            self.settle()
        d = self.__dict__
        i = len(d["_feat"])
        d["_feat"].append(-1)
        d["_thr"].append(0.0)
        d["_bin"].append(0)
        d["_left"].append(-1)
        d["_right"].append(-1)
        d["_catmask"].append(np.zeros(8, dtype=np.uint32))
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
        self.feat.extend([-1] * N)
        self.thr.extend([0.0] * N)
        self.bin.extend([0] * N)
        self.left.extend([-1] * N)
        self.right.extend([-1] * N)
        # leaves share one read-only zero mask (a categorical split assigns its own) and take their values as
        # float lists: N fresh numpy rows per field cost ~0.2 ms at the headline's last level (640 leaves) while
        # the GPU waits for the predict launch
        self.catmask.extend([_ZERO_MASK] * N)
        self.is_cat.extend([False] * N)
        self.value.extend(values.tolist())
        self.weight.extend(np.asarray(weights, dtype=np.float64).tolist())
        self.gain.extend([0.0] * N)
        self.impurity.extend(np.asarray(impurity, dtype=np.float64).tolist())
        self.depth.extend([depth] * N)
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
        if hi - lo == fids.size and bool(h.all()) and bool((rel[1:] > rel[:-1]).all()):
            # every node of the range splits, in order, on a threshold: plain slice assignments
            for name, vals in (("feat", feats), ("gain", gains), ("left", lefts), ("right", rights), ("bin", bins),
                               ("thr", thrs)):
                getattr(self, name)[lo:hi] = np.asarray(vals, dtype=np.float64 if name in ("gain", "thr")
                                                        else np.int64).tolist()
            return
        for name, vals, sel in (("feat", feats, None), ("gain", gains, None), ("left", lefts, None),
                                ("right", rights, None), ("bin", bins, h), ("thr", thrs, h)):
            lst = getattr(self, name)
            seg = np.array(lst[lo:hi], dtype=np.float64 if name in ("gain", "thr") else np.int64)
            v = np.asarray(vals)
            if sel is None:
                seg[rel] = v
            else:
                seg[rel[sel]] = v[sel]
            lst[lo:hi] = seg.tolist()

    @property
    def num_nodes(self):
        return len(self.feat)

    def tree_nodes(self, t: int) -> List[int]:
        L = self.lists()
        feat, left, right = L["feat"], L["left"], L["right"]
        out, stack = [], [self.roots[t]]
        while stack:
            i = stack.pop()
            out.append(i)
            if feat[i] >= 0:
                stack.extend([right[i], left[i]])
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
        # a forest cut by the fused tuner carries its node fields as arrays (truncate_forest): no list round trip
        npa = self.__dict__.get("_np") if CUT_ARRAYS else None
        if npa is not None and (len(npa["feat"]) != N or npa["is_cat"] is None or npa["value"] is None):
            npa = None
        feat = npa["feat"].astype(np.int32) if npa is not None else np.asarray(self.feat, dtype=np.int32)
        leaf = feat < 0
        isc = (npa["is_cat"] if npa is not None else np.asarray(self.is_cat, dtype=bool)) & ~leaf
        num = ~leaf & ~isc
        left = npa["left"].astype(np.int32) if npa is not None else np.asarray(self.left, dtype=np.int32)
        right = npa["right"].astype(np.int32) if npa is not None else np.asarray(self.right, dtype=np.int32)
        lid = np.nonzero(leaf)[0]
        if npa is not None:
            V = npa["value"][lid] if len(lid) else np.zeros((0, self.K))
        else:
            V = (np.stack([self.value[i] for i in lid.tolist()]).astype(np.float64) if len(lid)
                 else np.zeros((0, self.K)))
        if values_kind != "value" and len(lid):
            w_all = npa["weight"] if npa is not None else np.asarray(self.weight, dtype=np.float64)
            V = V * w_all[lid][:, None]
        kv = V.shape[1] if V.ndim == 2 else 1
        nodes[lid, 0] = -1
        nodes[lid, 1] = np.arange(len(lid), dtype=np.int32) * kv
        cid = np.nonzero(isc)[0]
        nodes[cid, 0] = -(feat[cid] + 2)
        nodes[cid, 1] = np.arange(len(cid), dtype=np.int32)
        nid = np.nonzero(num)[0]
        nodes[nid, 0] = feat[nid]
        thr = npa["thr"] if npa is not None else np.asarray(self.thr, dtype=np.float64)
        nodes[nid, 1] = thr[nid].astype(np.float32).view(np.int32)
        inner = ~leaf
        nodes[inner, 2] = left[inner]
        nodes[inner, 3] = right[inner]
        vals = V.reshape(-1).astype(np.float64) if V.size else np.zeros(1, np.float64)
        masks = (np.stack([self.catmask[i] for i in cid.tolist()]).view(np.int32).reshape(-1) if len(cid)
                 else np.zeros(8, np.int32))
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
        vals = np.array([self.value[r0 + j][0] for j in np.nonzero(leaf)[0].tolist()], dtype=np.float32)
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
        feat = np.asarray(self.feat, dtype=np.int64)  # one list conversion shared with _layout (~1.3k nodes)
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
        vl = self.value
        v = (np.concatenate([vl[i] for i in live[leaf].tolist()]) if leaf.any()
             else np.zeros(0)).astype(np.float64)
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
        masks = [self.catmask[i].view(np.int32) for i in cat_ids.tolist()]
        heap[lt[isc], ls[isc], 0] = -(fl[isc] + 2)
        heap[lt[isc], ls[isc], 1] = np.arange(len(cat_ids), dtype=np.int32)
        return heap, hv, D, (np.concatenate(masks) if masks else np.zeros(8, np.int32))

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
        catm = np.stack(self.catmask) if self.catmask else np.zeros((0, 8), np.uint32)
        vals = np.stack(self.value) if self.value else np.zeros((0, self.K))
        return {
            prefix + "feat": torch.tensor(self.feat, dtype=torch.int32),
            prefix + "thr": torch.tensor(self.thr, dtype=torch.float64),
            prefix + "bin": torch.tensor(self.bin, dtype=torch.int32),
            prefix + "left": torch.tensor(self.left, dtype=torch.int32),
            prefix + "right": torch.tensor(self.right, dtype=torch.int32),
            prefix + "catmask": torch.from_numpy(catm.view(np.int32).copy()),
            prefix + "is_cat": torch.tensor(self.is_cat, dtype=torch.bool),
            prefix + "value": torch.from_numpy(vals),
            prefix + "weight": torch.tensor(self.weight, dtype=torch.float64),
            prefix + "gain": torch.tensor(self.gain, dtype=torch.float64),
            prefix + "impurity": torch.tensor(self.impurity, dtype=torch.float64),
            prefix + "depth": torch.tensor(self.depth, dtype=torch.int32),
            prefix + "roots": torch.tensor(self.roots, dtype=torch.int32),
        }

    @classmethod
    def from_state(cls, st, prefix="forest_"):
        vals = st[prefix + "value"].numpy()
        f = cls(vals.shape[1] if vals.ndim == 2 else 1)
        f.feat = st[prefix + "feat"].tolist()
        f.thr = st[prefix + "thr"].tolist()
        f.bin = st[prefix + "bin"].tolist()
        f.left = st[prefix + "left"].tolist()
        f.right = st[prefix + "right"].tolist()
        f.catmask = [r.view(np.uint32).copy() for r in st[prefix + "catmask"].numpy()]
        f.is_cat = st[prefix + "is_cat"].tolist()
        f.value = [v for v in vals]
        f.weight = st[prefix + "weight"].tolist()
        f.gain = st[prefix + "gain"].tolist()
        f.impurity = st[prefix + "impurity"].tolist()
        f.depth = st[prefix + "depth"].tolist()
        f.roots = st[prefix + "roots"].tolist()
        return f

    def feature_importances(self, d: int, trees: Optional[List[int]] = None) -> np.ndarray:
        """Spark semantics: per-tree gain×count, normalised per tree, averaged, normalised."""
        total = np.zeros(d)
        trees = range(len(self.roots)) if trees is None else trees
        for t in trees:
            imp = np.zeros(d)
            for i in self.tree_nodes(t):
                if self.feat[i] >= 0:
                    imp[self.feat[i]] += self.gain[i] * self.weight[i]
            s = imp.sum()
            if s > 0:
                imp /= s
            total += imp
        s = total.sum()
        return total / s if s > 0 else total


def _settled_list(name: str):
    key = "_" + name

    def get(self):
        if self._pending and not self._settling:
            self.settle()
        return self.__dict__[key]

    def set_(self, v):
        self.__dict__[key] = v
        self.__dict__.pop("_np", None)  # a reassigned node list invalidates a cut's array snapshot
    return property(get, set_)


class _FrozenList(list):
    """A node list of a forest cut by the fused tuner (truncate_forest): its node fields are also held as an
    array snapshot (``Forest._np``) that the predictor reads instead of the lists, so the lists must not change
    after the cut.  Reads are plain list reads; every in-place mutation raises."""

    def _frozen(self, *a, **k):
        raise TypeError("the node lists of a cut forest are immutable (its array snapshot feeds the predictor); "
                        "build a new Forest instead")

    __setitem__ = __delitem__ = __iadd__ = __imul__ = append = extend = insert = pop = remove = clear = \
        sort = reverse = _frozen

    def __reduce__(self):  # pickle / deepcopy rebuild from a plain list (the default would extend())
        return (_FrozenList, (list(self),))


def freeze_cut(forest: "Forest", arrays: dict) -> None:
    """Attach the cut's node arrays (read-only) to ``forest`` and freeze its node lists (see _FrozenList)."""
    d = forest.__dict__
    for n in _NODE_FIELDS:
        d["_" + n] = _FrozenList(d["_" + n])
    d["roots"] = _FrozenList(d["roots"])
    for a in arrays.values():
        if isinstance(a, np.ndarray):
            a.flags.writeable = False
    d["_np"] = arrays


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
