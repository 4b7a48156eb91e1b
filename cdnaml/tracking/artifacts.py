"""Model URIs (``runs:/<id>/<path>``, ``models:/<name>/<version|stage>``) -> local paths."""
from __future__ import annotations

import os
from typing import Optional, Tuple

from .entities import TrackingException


def parse_runs_uri(uri: str) -> Tuple[Optional[str], Optional[str]]:
    if uri.startswith("runs:/"):
        rest = uri[len("runs:/"):].lstrip("/")
        rid, _, path = rest.partition("/")
        return rid, path
    return None, None


def resolve(uri: str) -> str:
    from . import fluent
    st = fluent._store()
    if uri.startswith("runs:/"):
        rid, path = parse_runs_uri(uri)
        return os.path.join(st.artifact_dir(rid), path)
    if uri.startswith("models:/"):
        rest = uri[len("models:/"):].strip("/")
        name, _, ver = rest.partition("/")
        if not ver or ver.lower() == "latest":
            vs = st.search_model_versions_for(name)
            if not vs:
                raise TrackingException(f"No versions of model {name}")
            mv = vs[-1]
        elif ver.isdigit():
            mv = st.get_model_version(name, int(ver))
        else:
            cands = [v for v in st.search_model_versions_for(name) if v.current_stage.lower() == ver.lower()]
            if not cands:
                raise TrackingException(f"No versions of model {name} in stage {ver}")
            mv = cands[-1]
        return resolve(mv.source)
    from ..utils.dbutils import to_local
    return to_local(uri)
