"""Alternating least squares.

One process: each half-iteration accumulates, for every rating, the per-entity normal equations Σ v vᵀ and
Σ r v on device (K12 als.hip, no [nnz, r, r] temporary) and solves them as a BATCH on the GPU -- Cholesky by
default, coordinate-descent NNLS when ``nonnegative=True`` (MLE 01 - Collaborative Filtering Lab.py:136-202).
Regularisation follows MLlib's ALS-WR scaling (λ · n_u).  ``coldStartStrategy="drop"`` removes rows with
unknown users/items from ``transform`` output.

Several ranks (block ALS, MLlib's in/out-block design re-done for one process per GPU): users and items are
hash-partitioned over the ranks by dense id (owner = id % W) and the ratings are shuffled twice with
``all_to_all_v`` -- one copy grouped by user owner, one by item owner.  A user half-step on rank p needs the
item factors its users rated: every rank sends each peer exactly the rows of its own items that peer needs
(an ``all_to_all_v`` of [m, rank] factor blocks, routing lists built once), and p then solves only its own
users.  No rank holds or all-reduces the dense [n_entities, rank, rank] systems; the result equals the
one-rank fit up to the fp64 summation order.  Factors are all-gathered once at the end for the model.
"""
from __future__ import annotations

import numpy as np
import torch

from ..sql import types as T
from ..sql.batch import ColumnData
from ..sql.dataframe import MapPlan
from .base import Estimator, Model
from .param import NO_DEFAULT, TypeConverters as TC, keyword_init
from .regression import _default_seed
from .util import local_batch


# K12 HIP path (als.hip) for ranks <= 32 on the GPU; the torch path is the reference
ALS_NATIVE = True
# several ranks: block-partitioned users / items with all-to-all factor exchange (else replicated + all-reduce)
ALS_BLOCK = __import__("os").environ.get("CDNAML_ALS_BLOCK", "1") != "0"


class _LocalComm:
    """No-op reducer: block ALS half-steps solve rank-local systems."""
    distributed = False

    @staticmethod
    def all_reduce_many(tensors, op="sum"):
        return list(tensors)

    @staticmethod
    def all_reduce(t, op="sum"):
        return t

class ALS(Estimator):
    _params = {
        "rank": ("rank of the factorization", 10, TC.toInt),
        "maxIter": ("max number of iterations (>= 0)", 10, TC.toInt),
        "regParam": ("regularization parameter (>= 0)", 0.1, TC.toFloat),
        "numUserBlocks": ("number of user blocks", 10, TC.toInt),
        "numItemBlocks": ("number of item blocks", 10, TC.toInt),
        "implicitPrefs": ("whether to use implicit preference", False, TC.toBoolean),
        "alpha": ("alpha for implicit preference", 1.0, TC.toFloat),
        "userCol": ("column name for user ids. Ids must be within the integer value range.", "user", TC.toString),
        "itemCol": ("column name for item ids. Ids must be within the integer value range.", "item", TC.toString),
        "ratingCol": ("column name for ratings", "rating", TC.toString),
        "predictionCol": ("prediction column name", "prediction", TC.toString),
        "nonnegative": ("whether to use nonnegative constraint for least squares", False, TC.toBoolean),
        "checkpointInterval": ("checkpoint interval", 10, TC.toInt),
        "seed": ("random seed", None, TC.toInt),
        "intermediateStorageLevel": ("storage level for intermediate datasets", "MEMORY_AND_DISK", TC.toString),
        "finalStorageLevel": ("storage level for ALS model factors", "MEMORY_AND_DISK", TC.toString),
        "coldStartStrategy": ("strategy for dealing with unknown or new users/items at prediction time: nan, drop",
                              "nan", TC.toString),
        "blockSize": ("block size for stacking input data in matrices", 4096, TC.toInt),
    }

    def __init__(self, **kwargs):
        super().__init__()
        keyword_init(self, kwargs)

    @staticmethod
    def _solve(A: torch.Tensor, b: torch.Tensor, nonneg: bool) -> torch.Tensor:
        """Batched SPD solve [E, r, r] x = [E, r] on device."""
        if not nonneg:
            L, info = torch.linalg.cholesky_ex(A)
            x = torch.cholesky_solve(b.unsqueeze(-1), L).squeeze(-1)
            bad = info != 0
            if bool(bad.any()):
                x[bad] = torch.linalg.lstsq(A[bad], b[bad].unsqueeze(-1)).solution.squeeze(-1)
            return x
        # batched coordinate-descent NNLS (exact per-coordinate minimisation)
        E, r = b.shape
        x = torch.zeros_like(b)
        diag = torch.diagonal(A, dim1=1, dim2=2).clamp_min(1e-12)
        for _ in range(40):
            for j in range(r):
                g = b[:, j] - (A[:, j, :] * x).sum(1) + A[:, j, j] * x[:, j]
                x[:, j] = torch.clamp(g / diag[:, j], min=0.0)
        return x

    @staticmethod
    def _csr(dst_idx: torch.Tensor, n_dst: int):
        """Ratings sorted by destination: (order, offsets[n_dst + 1])."""
        order = torch.argsort(dst_idx, stable=True)
        counts = torch.bincount(dst_idx, minlength=n_dst)
        off = torch.zeros(n_dst + 1, dtype=torch.int64, device=dst_idx.device)
        off[1:] = torch.cumsum(counts, 0)
        return order, off

    def _half_step_native(self, comm, src_idx, dst_idx, r, F_src, n_dst, lam, nonneg, implicit, alpha, csr,
                          gram=None):
        """K12 on the GPU (als.hip): per-destination Gram accumulation without an [nnz, r, r]
        temporary, one fused all-reduce, then batched in-LDS Cholesky / NNLS solves."""
        from ..ops import _lib
        from ..ops.kernels import _ptr, _stream
        rank = F_src.shape[1]
        dev = F_src.device
        order, off = csr
        src_s = src_idx[order].int().contiguous()
        r_s = r[order].double().contiguous()
        Fd = F_src.double().contiguous()
        A = torch.empty((n_dst, rank, rank), dtype=torch.float64, device=dev)
        bvec = torch.empty((n_dst, rank), dtype=torch.float64, device=dev)
        cnt = torch.empty(n_dst, dtype=torch.float64, device=dev)
        L = _lib.lib()
        _lib.check(L.cdna_als_accumulate(n_dst, _ptr(off), _ptr(src_s), _ptr(r_s), _ptr(Fd), rank, int(implicit),
                                         float(alpha), _ptr(A), _ptr(bvec), _ptr(cnt), _stream(dev)),
                   "cdna_als_accumulate")
        comm.all_reduce_many([A.view(-1), bvec.view(-1), cnt])
        has = cnt > 0
        out = torch.zeros((n_dst, rank), dtype=torch.float64, device=dev)
        hi = torch.nonzero(has).flatten()
        E = int(hi.numel())
        if E == 0:
            return out
        Ah, bh = A[hi].contiguous(), bvec[hi].contiguous()
        diag = (lam * cnt[hi].clamp_min(1)) if implicit else (lam * cnt[hi])
        G = (gram.double() if gram is not None else Fd.T @ Fd).contiguous() if implicit else None
        x = torch.empty((E, rank), dtype=torch.float64, device=dev)
        info = torch.empty(E, dtype=torch.int32, device=dev)
        _lib.check(L.cdna_als_solve(E, rank, _ptr(Ah), _ptr(bh), _ptr(diag.contiguous()), _ptr(G), int(nonneg), 40,
                                    _ptr(x), _ptr(info), _stream(dev)), "cdna_als_solve")
        bad = info != 0
        if bool(bad.any()):
            eye = torch.eye(rank, dtype=torch.float64, device=dev)
            Mb = Ah[bad] + diag[bad][:, None, None] * eye + (G[None] if G is not None else 0)
            x[bad] = torch.linalg.lstsq(Mb, bh[bad].unsqueeze(-1)).solution.squeeze(-1)
        out[hi] = x
        return out

    def _half_step(self, comm, src_idx, dst_idx, r, F_src, n_dst, lam, nonneg, implicit, alpha, csr=None,
                   gram=None):
        """gram: the implicit-feedback Y^T Y over ALL source factors (block ALS passes the all-reduced one)."""
        rank = F_src.shape[1]
        dev = F_src.device
        if csr is not None:
            return self._half_step_native(comm, src_idx, dst_idx, r, F_src, n_dst, lam, nonneg, implicit, alpha, csr,
                                          gram)
        A = torch.zeros((n_dst, rank, rank), dtype=torch.float64, device=dev)
        bvec = torch.zeros((n_dst, rank), dtype=torch.float64, device=dev)
        cnt = torch.zeros(n_dst, dtype=torch.float64, device=dev)
        chunk = 1 << 20
        for a in range(0, src_idx.numel(), chunk):
            s, d_, rr = src_idx[a:a + chunk], dst_idx[a:a + chunk], r[a:a + chunk]
            V = F_src[s]
            if implicit:
                c = 1.0 + alpha * rr.abs()
                p = (rr > 0).double()
                A.index_add_(0, d_, (c - 1.0)[:, None, None] * V[:, :, None] * V[:, None, :])
                bvec.index_add_(0, d_, (c * p)[:, None] * V)
            else:
                A.index_add_(0, d_, V[:, :, None] * V[:, None, :])
                bvec.index_add_(0, d_, rr[:, None] * V)
            cnt.index_add_(0, d_, torch.ones_like(rr))
        comm.all_reduce_many([A.view(-1), bvec.view(-1), cnt])
        eye = torch.eye(rank, dtype=torch.float64, device=dev)
        if implicit:
            YtY = gram if gram is not None else F_src.T @ F_src
            A = A + YtY[None]
            A = A + lam * cnt.clamp_min(1)[:, None, None] * eye
        else:
            A = A + (lam * cnt)[:, None, None] * eye
        has = cnt > 0
        out = torch.zeros((n_dst, rank), dtype=torch.float64, device=dev)
        if bool(has.any()):
            out[has] = self._solve(A[has], bvec[has], nonneg)
        return out

    def _fit(self, dataset):
        uc, ic, rc = self.getUserCol(), self.getItemCol(), self.getRatingCol()
        session = dataset._session
        comm = session.comm
        b = local_batch(dataset, [uc, ic, rc])
        u = b.columns[uc].values.long()
        i = b.columns[ic].values.long()
        r = b.columns[rc].values.double()
        ok = torch.ones_like(r, dtype=torch.bool)
        for c in (b.columns[uc], b.columns[ic], b.columns[rc]):
            if c.valid is not None:
                ok &= c.valid
        u, i, r = u[ok], i[ok], r[ok]
        uid = torch.unique(u)
        iid = torch.unique(i)
        if comm.distributed:
            uid = torch.unique(torch.cat(comm.all_gather_varlen(uid)))
            iid = torch.unique(torch.cat(comm.all_gather_varlen(iid)))
        ui = torch.searchsorted(uid, u)
        ii = torch.searchsorted(iid, i)
        k = self.getRank()
        seed = self.getSeed() if self.getSeed() is not None else _default_seed(type(self))
        g = torch.Generator().manual_seed(int(seed) & 0x7FFFFFFF)
        # MLlib initialises factors with |N(0,1)| / sqrt(rank)-normalised rows
        U = torch.randn((uid.numel(), k), generator=g, dtype=torch.float64).abs()
        V = torch.randn((iid.numel(), k), generator=g, dtype=torch.float64).abs()
        U = (U / torch.linalg.vector_norm(U, dim=1, keepdim=True)).to(u.device)
        V = (V / torch.linalg.vector_norm(V, dim=1, keepdim=True)).to(u.device)
        lam, nonneg = self.getRegParam(), self.getNonnegative()
        implicit, alpha = self.getImplicitPrefs(), self.getAlpha()
        native = ALS_NATIVE and u.device.type == "cuda" and k <= 32
        csr_u = self._csr(ui, uid.numel()) if native else None
        csr_i = self._csr(ii, iid.numel()) if native else None
        if comm.distributed and ALS_BLOCK:
            U, V = self._fit_blocks(comm, ui, ii, r, U, V, lam, nonneg, implicit, alpha, k)
        else:
            for _ in range(self.getMaxIter()):
                U = self._half_step(comm, ii, ui, r, V, uid.numel(), lam, nonneg, implicit, alpha, csr_u)
                V = self._half_step(comm, ui, ii, r, U, iid.numel(), lam, nonneg, implicit, alpha, csr_i)
        model = ALSModel(uid.cpu().numpy(), U.float().cpu().numpy(), iid.cpu().numpy(), V.float().cpu().numpy())
        return model

    # ------------------------------------------------------------------ block ALS (W > 1)
    @staticmethod
    def _shuffle(comm, owner, cols):
        """Route rating rows to their owner rank: returns the received columns (concatenated)."""
        W = comm.world_size
        order = torch.argsort(owner, stable=True)
        counts = torch.bincount(owner, minlength=W).tolist()
        recv = comm.all_to_all_counts(counts)  # one count exchange for all columns
        out = []
        for c in cols:
            parts = list(torch.split(c[order], counts))
            out.append(torch.cat(comm.all_to_all_v(parts, recv)))
        return out

    @staticmethod
    def _routes(comm, need_ids):
        """need_ids: sorted global ids of remote-owned (or own) entities this rank's ratings reference.
        Returns (send_lists, need_sorted): send_lists[q] = global ids this rank owns that rank q needs (in q's
        request order); need_sorted = this rank's needs ordered by (owner, id), the order replies arrive in."""
        W = comm.world_size
        own = need_ids % W
        order = torch.argsort(own * (need_ids.max() + 1 if need_ids.numel() else 1) + need_ids)
        need_sorted = need_ids[order]
        counts = torch.bincount(own, minlength=W).tolist()
        send_lists = comm.all_to_all_v(list(torch.split(need_sorted, counts)))
        return send_lists, need_sorted

    def _fit_blocks(self, comm, ui, ii, r, U0, V0, lam, nonneg, implicit, alpha, k):
        W, me = comm.world_size, comm.rank
        dev = ui.device
        nu, ni = U0.shape[0], V0.shape[0]
        # the ratings twice: grouped by user owner and by item owner
        bu_u, bu_i, bu_r = self._shuffle(comm, ui % W, [ui, ii, r])
        bi_u, bi_i, bi_r = self._shuffle(comm, ii % W, [ui, ii, r])
        my_u = torch.arange(me, nu, W, device=dev)          # owned users (global ids), local index = id // W
        my_i = torch.arange(me, ni, W, device=dev)
        U = U0[my_u].clone()
        V = V0[my_i].clone()
        # routing: which item factors each rank needs for its user step (and users for the item step)
        need_i = torch.unique(bu_i)
        send_i, need_i_sorted = self._routes(comm, need_i)
        need_u = torch.unique(bi_u)
        send_u, need_u_sorted = self._routes(comm, need_u)
        # rating -> row of the received factor block (replies arrive in (owner, id) order)
        pos_i = torch.argsort(need_i_sorted)
        src_in_u = pos_i[torch.searchsorted(need_i_sorted[pos_i], bu_i)]
        pos_u = torch.argsort(need_u_sorted)
        src_in_i = pos_u[torch.searchsorted(need_u_sorted[pos_u], bi_u)]
        dst_u, dst_i = bu_u // W, bi_i // W
        native = ALS_NATIVE and dev.type == "cuda" and k <= 32
        csr_u = self._csr(dst_u, my_u.numel()) if native else None
        csr_i = self._csr(dst_i, my_i.numel()) if native else None
        local = _LocalComm()
        # every iteration's factor replies follow the same routing: rank q sends what this rank asked it for
        recv_i = torch.bincount(need_i_sorted % W, minlength=W).tolist()
        recv_u = torch.bincount(need_u_sorted % W, minlength=W).tolist()
        for _ in range(self.getMaxIter()):
            Vneed = torch.cat(comm.all_to_all_v([V[s // W] for s in send_i], recv_i))
            gV = comm.all_reduce(V.T @ V) if implicit else None   # implicit Y^T Y spans every rank's items
            U = self._half_step(local, src_in_u, dst_u, bu_r, Vneed, my_u.numel(), lam, nonneg, implicit, alpha,
                                csr_u, gV)
            Uneed = torch.cat(comm.all_to_all_v([U[s // W] for s in send_u], recv_u))
            gU = comm.all_reduce(U.T @ U) if implicit else None
            V = self._half_step(local, src_in_i, dst_i, bi_r, Uneed, my_i.numel(), lam, nonneg, implicit, alpha,
                                csr_i, gU)
        # assemble the replicated factors for the model (one gather each)
        Uf = torch.zeros((nu, k), dtype=torch.float64, device=dev)
        Vf = torch.zeros((ni, k), dtype=torch.float64, device=dev)
        for ids, F in zip(comm.all_gather_varlen(my_u), comm.all_gather_varlen(U)):
            Uf[ids.to(dev)] = F.to(dev)
        for ids, F in zip(comm.all_gather_varlen(my_i), comm.all_gather_varlen(V)):
            Vf[ids.to(dev)] = F.to(dev)
        return Uf, Vf


class ALSModel(Model):
    _params = {k: v for k, v in ALS._params.items() if k != "rank"}  # ALSModel.rank is a property

    def __init__(self, user_ids=None, user_factors=None, item_ids=None, item_factors=None):
        super().__init__()
        self._uid = np.asarray(user_ids if user_ids is not None else [], dtype=np.int64)
        self._U = np.asarray(user_factors if user_factors is not None else np.zeros((0, 0)), dtype=np.float32)
        self._iid = np.asarray(item_ids if item_ids is not None else [], dtype=np.int64)
        self._V = np.asarray(item_factors if item_factors is not None else np.zeros((0, 0)), dtype=np.float32)

    @property
    def rank(self):
        return int(self._U.shape[1]) if self._U.ndim == 2 else 0

    def _factor_df(self, ids, F):
        import pandas as pd
        from ..session import SparkSession
        s = SparkSession.getActiveSession()
        return s.createDataFrame(pd.DataFrame({"id": ids.astype(np.int32), "features": [list(map(float, f)) for f in F]}),
                                 schema="id int, features array<float>")

    @property
    def userFactors(self):
        return self._factor_df(self._uid, self._U)

    @property
    def itemFactors(self):
        return self._factor_df(self._iid, self._V)

    def _lookup(self, ids: torch.Tensor, table: np.ndarray):
        t = torch.from_numpy(table).to(ids.device)
        if t.numel() == 0:
            return torch.zeros_like(ids), torch.zeros_like(ids, dtype=torch.bool)
        pos = torch.searchsorted(t, ids).clamp(max=t.numel() - 1)
        return pos, t[pos] == ids

    def _transform(self, dataset):
        uc, ic, pc = self.getUserCol(), self.getItemCol(), self.getPredictionCol()
        drop = self.getColdStartStrategy() == "drop"
        U, V = torch.from_numpy(self._U), torch.from_numpy(self._V)
        model = self

        def fn(b, ctx):
            u = b.columns[uc].values.long()
            i = b.columns[ic].values.long()
            pu, oku = model._lookup(u, model._uid)
            pi, oki = model._lookup(i, model._iid)
            Ud, Vd = U.to(u.device), V.to(u.device)
            ok = oku & oki
            for c in (b.columns[uc], b.columns[ic]):
                if c.valid is not None:
                    ok &= c.valid
            pred = (Ud[pu] * Vd[pi]).sum(1).double() if u.numel() else torch.zeros(0, dtype=torch.float64,
                                                                                     device=u.device)
            pred = torch.where(ok, pred, torch.full_like(pred, float("nan")))
            nb = b.with_column(pc, ColumnData(pred.float(), T.FloatType()))
            return nb.filter(ok) if drop else nb
        return dataset._new(MapPlan(dataset._plan, "ALSModel", fn))

    def _recommend(self, src_ids, S, dst_ids, D, k, src_name, dst_name):
        import pandas as pd
        from ..session import SparkSession
        s = SparkSession.getActiveSession()
        dev = s.device
        St, Dt = torch.from_numpy(S).to(dev), torch.from_numpy(D).to(dev)
        scores = St @ Dt.T
        kk = min(k, Dt.shape[0])
        top = torch.topk(scores, kk, dim=1)
        idx, val = top.indices.cpu().numpy(), top.values.cpu().numpy()
        recs = [[{dst_name: int(dst_ids[j]), "rating": float(v)} for j, v in zip(ri, rv)] for ri, rv in zip(idx, val)]
        pdf = pd.DataFrame({src_name: src_ids.astype(np.int32), "recommendations": [str(r) for r in recs]})
        df = s.createDataFrame(pdf)
        df._recs = recs
        return df

    def recommendForAllUsers(self, numItems):
        return self._recommend(self._uid, self._U, self._iid, self._V, numItems, self.getUserCol(),
                               self.getItemCol())

    def recommendForAllItems(self, numUsers):
        return self._recommend(self._iid, self._V, self._uid, self._U, numUsers, self.getItemCol(),
                               self.getUserCol())

    def recommendForUserSubset(self, dataset, numItems):
        ids = np.array([r[0] for r in dataset.select(self.getUserCol()).distinct().collect()], dtype=np.int64)
        pos = np.searchsorted(self._uid, ids)
        ok = (pos < len(self._uid)) & (self._uid[np.minimum(pos, len(self._uid) - 1)] == ids)
        return self._recommend(ids[ok], self._U[pos[ok]], self._iid, self._V, numItems, self.getUserCol(),
                               self.getItemCol())

    def _save_state(self):
        return {}, {"uid": torch.from_numpy(self._uid), "U": torch.from_numpy(self._U),
                    "iid": torch.from_numpy(self._iid), "V": torch.from_numpy(self._V)}

    def _load_state(self, extra, tensors, stages):
        self._uid, self._U = tensors["uid"].numpy(), tensors["U"].numpy()
        self._iid, self._V = tensors["iid"].numpy(), tensors["V"].numpy()
