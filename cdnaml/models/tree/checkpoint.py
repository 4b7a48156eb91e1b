"""Round checkpoints for boosted ensembles ("optional per-N-trees GBDT
checkpoints (model-so-far plus the prediction column)").

Spark's GBT takes ``checkpointInterval`` with ``SparkContext.setCheckpointDir``
(MLlib checkpoints the RDD lineage); here a checkpoint is what is needed to
resume the boosting loop exactly:

    <dir>/<fit key>/rank<r>.safetensors   forest-so-far + this rank's margins + round
    <dir>/<fit key>/rank<r>.json          round, tree weights / history, data fingerprint

``fit key`` hashes the estimator's params and the global data shape, so a
different fit never resumes from a foreign checkpoint.  Files are written to a
temp name and renamed (a crash mid-write leaves the previous checkpoint).  A
resumed fit is bit-identical to an uninterrupted one: the per-round seeds are
derived from the round index and the margins are restored exactly.
"""
from __future__ import annotations

import hashlib
import json
import os
from typing import Any, Dict, Optional, Tuple

import torch

from .engine import Forest


def fit_key(est, n_global: int, d: int) -> str:
    items = sorted((p.name, repr(v)) for p, v in est.extractParamMap().items()
                   if p.name not in ("checkpointInterval",))
    h = hashlib.sha1(json.dumps([type(est).__name__, items, int(n_global), int(d)]).encode()).hexdigest()
    return h[:16]


class RoundCheckpointer:
    """Saves every ``interval`` rounds; ``load()`` returns the latest state or None."""

    def __init__(self, session, est, n_global: int, d: int, interval: Optional[int]):
        root = session.sparkContext.getCheckpointDir()
        self.enabled = bool(root) and interval is not None and int(interval) >= 1
        self.interval = int(interval) if self.enabled else 0
        self.rank = session.comm.rank
        self.comm = session.comm
        self.dir = os.path.join(root, fit_key(est, n_global, d)) if self.enabled else None
        self.saved = 0

    def _paths(self):
        base = os.path.join(self.dir, f"rank{self.rank}")
        return base + ".safetensors", base + ".json"

    def load(self) -> Optional[Tuple[int, Forest, torch.Tensor, Dict[str, Any]]]:
        if not self.enabled:
            return None
        st_path, js_path = self._paths()
        ok = os.path.exists(st_path) and os.path.exists(js_path)
        # every rank must resume from the same round (or none)
        rounds = self.comm.all_gather_object(json.load(open(js_path))["round"] if ok else -1)
        if min(rounds) < 0 or len(set(rounds)) != 1:
            return None
        from safetensors.torch import load_file
        st = load_file(st_path)
        meta = json.load(open(js_path))
        forest = Forest.from_state(st)
        return meta["round"], forest, st["margins"], meta.get("extra", {})

    def maybe_save(self, rounds_done: int, forest: Forest, margins: torch.Tensor, extra: Dict[str, Any]):
        if not self.enabled or rounds_done % self.interval != 0:
            return
        from safetensors.torch import save_file
        os.makedirs(self.dir, exist_ok=True)
        st_path, js_path = self._paths()
        st = {k: v.contiguous() for k, v in forest.state().items()}
        st["margins"] = margins.detach().float().cpu().contiguous()
        save_file(st, st_path + ".tmp")
        with open(js_path + ".tmp", "w") as f:
            json.dump({"round": int(rounds_done), "extra": extra}, f)
        os.replace(st_path + ".tmp", st_path)
        os.replace(js_path + ".tmp", js_path)
        self.saved += 1
