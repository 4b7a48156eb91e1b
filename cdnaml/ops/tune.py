"""Tuning constants of the tree engine and its kernels, overridable for experiments through ONE environment knob.

The engine's kernel-path switches and sizes are plain module constants (``cdnaml.ops.kernels``,
``cdnaml.models.tree.engine``) with the measured defaults documented next to them; tests patch them as module
attributes.  For an A/B run on a GPU box without editing code::

    CDNAML_TUNE="SEG_MIN_BLOCKS=1024,LANE10_CHUNK3=1" python bench.py

sets those constants at import, each value parsed as the type of the default (bool: 0/1/true/false).  A name
that no tuned module defines is an error, so a typo does not silently measure the default."""
from __future__ import annotations

import os
from typing import Dict

_SPEC = os.environ.get("CDNAML_TUNE", "")


def _parse() -> Dict[str, str]:
    out = {}
    for item in _SPEC.split(","):
        item = item.strip()
        if not item:
            continue
        name, eq, val = item.partition("=")
        if not eq:
            raise ValueError(f"CDNAML_TUNE entries are NAME=value, got {item!r}")
        out[name.strip()] = val.strip()
    return out


_OVERRIDES = _parse()
_APPLIED = set()


def _coerce(default, text: str):
    if isinstance(default, bool):
        if text.lower() in ("1", "true", "yes", "on"):
            return True
        if text.lower() in ("0", "false", "no", "off"):
            return False
        raise ValueError(f"CDNAML_TUNE: {text!r} is not a bool")
    if isinstance(default, int):
        return int(float(text))
    if isinstance(default, float):
        return float(text)
    return text


def apply(module) -> None:
    """Set the overridden constants ``module`` defines (call at the end of the module)."""
    for name, text in _OVERRIDES.items():
        if name.isupper() and hasattr(module, name):
            setattr(module, name, _coerce(getattr(module, name), text))
            _APPLIED.add(name)


def check() -> None:
    """Every override named a constant of some tuned module (call once all of them are imported)."""
    unknown = sorted(set(_OVERRIDES) - _APPLIED)
    if unknown:
        raise ValueError(f"CDNAML_TUNE names no tuning constant: {', '.join(unknown)}")
