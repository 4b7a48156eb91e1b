"""Round checkpoints for boosted ensembles ("optional per-N-trees GBDT
checkpoints (model-so-far plus the prediction column)").

Spark's GBT takes ``checkpointInterval`` with ``SparkContext.setCheckpointDir``
(MLlib checkpoints the RDD lineage); here a checkpoint is what is needed to
resume the boosting loop exactly:

    <dir>/<fit key>/rank<r>.safetensors   forest-so-far + this rank's margins; the round, the
                                          tree weights / history and the data fingerprint ride
                                          in the file's metadata (one atomic file per rank)

``fit key`` hashes the estimator's params, the world size and a DATA
fingerprint: the bin thresholds (a function of the global quantile sample),
every rank's row count, and an all-reduced checksum of the labels.  A fit on
different data of the same shape, or with a different GPU count, therefore
never resumes from a foreign checkpoint; the fingerprint is stored in the file
and checked again on load.  The file is written to a temp name and renamed (a
crash mid-write leaves the previous checkpoint).  A successful fit removes its
checkpoints (like Spark's periodic checkpointer).  A resumed fit is
bit-identical to an uninterrupted one: the per-round seeds are derived from
the round index and the margins are restored exactly.
"""
from __future__ import annotations

import hashlib
import json
import os
from typing import Any, Dict, Optional, Tuple

import numpy as np
import torch

from .forest import Forest


def data_fingerprint(session, data, labels: Optional[torch.Tensor]) -> str:
    """Identical on every rank: thresholds + per-rank row counts + world size + label checksum."""
    comm = session.comm
    h = hashlib.sha1()
    h.update(np.ascontiguousarray(data.thresholds, dtype=np.float64).tobytes())
    h.update(np.ascontiguousarray(data.nthr, dtype=np.int64).tobytes())
    h.update(json.dumps([int(comm.world_size), comm.all_gather_object(int(data.n_local)),
                         int(data.n_global), int(data.d), int(data.B)]).encode())
    if labels is not None:
        y = labels.reshape(-1).double()
        n = y.numel()
        # position-weighted checksum (a permuted or shifted label column changes it)
        pos = torch.arange(n, dtype=torch.float64, device=y.device) + float(data.row_offset) + 1.0
        s = torch.stack([y.sum(), (y * y).sum(), (y * torch.remainder(pos, 9973.0)).sum()]) if n else \
            torch.zeros(3, dtype=torch.float64, device=y.device)
        s = s.to(comm.device)
        comm.all_reduce(s)
        h.update(np.asarray(s.cpu().numpy(), dtype=np.float64).tobytes())
    return h.hexdigest()[:20]


def fit_key(est, fingerprint: str) -> str:
    items = sorted((p.name, repr(v)) for p, v in est.extractParamMap().items()
                   if p.name not in ("checkpointInterval",))
    h = hashlib.sha1(json.dumps([type(est).__name__, items, fingerprint]).encode()).hexdigest()
    return h[:16]


class RoundCheckpointer:
    """Saves every ``interval`` rounds; ``load()`` returns the latest state or None; ``finish()`` removes
    this fit's checkpoints once the fit has completed."""

    def __init__(self, session, est, data, interval: Optional[int], labels: Optional[torch.Tensor] = None):
        root = session.sparkContext.getCheckpointDir()
        self.enabled = bool(root) and interval is not None and int(interval) >= 1
        self.interval = int(interval) if self.enabled else 0
        self.rank = session.comm.rank
        self.comm = session.comm
        self.fingerprint = data_fingerprint(session, data, labels) if self.enabled else ""
        self.dir = os.path.join(root, fit_key(est, self.fingerprint)) if self.enabled else None
        self.saved = 0

    def _path(self):
        return os.path.join(self.dir, f"rank{self.rank}.safetensors")

    def _read_meta(self, path) -> Optional[dict]:
        from safetensors import safe_open
        try:
            with safe_open(path, framework="pt") as f:
                md = f.metadata() or {}
            meta = json.loads(md.get("cdnaml", "{}"))
        except Exception:  # noqa: BLE001 - unreadable / foreign file: no resume
            return None
        if meta.get("fingerprint") != self.fingerprint or "round" not in meta:
            return None
        return meta

    def load(self) -> Optional[Tuple[int, Forest, torch.Tensor, Dict[str, Any]]]:
        if not self.enabled:
            return None
        path = self._path()
        meta = self._read_meta(path) if os.path.exists(path) else None
        # every rank must resume from the same round (or none)
        rounds = self.comm.all_gather_object(int(meta["round"]) if meta else -1)
        if min(rounds) < 0 or len(set(rounds)) != 1:
            return None
        from safetensors.torch import load_file
        st = load_file(path)
        forest = Forest.from_state(st)
        if len(forest.roots) != int(meta.get("trees", len(forest.roots))):
            return None
        return int(meta["round"]), forest, st["margins"], meta.get("extra", {})

    def maybe_save(self, rounds_done: int, forest: Forest, margins: torch.Tensor, extra: Dict[str, Any]):
        if not self.enabled or rounds_done % self.interval != 0:
            return
        from safetensors.torch import save_file
        os.makedirs(self.dir, exist_ok=True)
        path = self._path()
        st = {k: v.contiguous() for k, v in forest.state().items()}
        st["margins"] = margins.detach().float().cpu().contiguous()
        meta = {"round": int(rounds_done), "trees": len(forest.roots), "fingerprint": self.fingerprint,
                "world_size": int(self.comm.world_size), "extra": extra}
        save_file(st, path + ".tmp", metadata={"cdnaml": json.dumps(meta)})
        os.replace(path + ".tmp", path)
        self.saved += 1

    def finish(self) -> None:
        """The fit completed: drop this rank's checkpoint (and the fit directory once it is empty)."""
        if not self.enabled:
            return
        for p in (self._path(), self._path() + ".tmp"):
            if os.path.exists(p):
                os.remove(p)
        try:
            os.rmdir(self.dir)
        except OSError:
            pass  # other ranks' files still there, or never created
