"""Koalas options (ML 14:120,180,201-202): ``set_option``, ``get_option`` and the
attribute namespace ``options.plotting.backend = 'matplotlib'``."""
from __future__ import annotations

import contextlib

_DEFAULTS = {
    "display.max_rows": 1000,
    "compute.max_rows": 1000,
    "compute.shortcut_limit": 1000,
    "compute.ops_on_diff_frames": False,
    "compute.default_index_type": "sequence",
    "compute.ordered_head": False,
    "plotting.max_rows": 1000,
    "plotting.sample_ratio": None,
    "plotting.backend": "matplotlib",
}
_VALID = {
    "compute.default_index_type": {"sequence", "distributed-sequence", "distributed"},
    "plotting.backend": {"matplotlib", "plotly"},
}
_state = dict(_DEFAULTS)


def get_option(key: str, default=None):
    if key not in _state:
        if default is not None:
            return default
        raise KeyError(f"No such option: '{key}'")
    return _state[key]


def set_option(key: str, value) -> None:
    if key not in _DEFAULTS:
        raise KeyError(f"No such option: '{key}'")
    if key in _VALID and value not in _VALID[key]:
        raise ValueError(f"'{key}' must be one of {sorted(_VALID[key])}, got {value!r}")
    _state[key] = value


def reset_option(key: str) -> None:
    _state[key] = _DEFAULTS[key]


@contextlib.contextmanager
def option_context(*args):
    pairs = list(zip(args[::2], args[1::2]))
    old = {k: get_option(k) for k, _ in pairs}
    try:
        for k, v in pairs:
            set_option(k, v)
        yield
    finally:
        for k, v in old.items():
            set_option(k, v)


class _Namespace:
    def __init__(self, prefix=""):
        object.__setattr__(self, "_prefix", prefix)

    def _key(self, name):
        return f"{self._prefix}.{name}" if self._prefix else name

    def __getattr__(self, name):
        k = self._key(name)
        if k in _state:
            return _state[k]
        if any(x.startswith(k + ".") for x in _state):
            return _Namespace(k)
        raise AttributeError(f"No such option: '{k}'")

    def __setattr__(self, name, value):
        set_option(self._key(name), value)

    def __dir__(self):
        p = self._prefix + "." if self._prefix else ""
        return sorted({k[len(p):].split(".")[0] for k in _state if k.startswith(p)})


options = _Namespace()
