"""Params system.

Param objects are class attributes (``rf.maxDepth``) usable as grid and
``copy()`` keys; ``explainParams()`` documents them; ``setX``/``getX``
chain; integral floats from ``hp.quniform`` are coerced for int params
(``pipeline.copy({rf.maxDepth: 3.0, rf.numTrees: 57.0})`` — ML 08 -
Hyperopt.py:97,159).
"""
from __future__ import annotations

import copy as _copy
import uuid
from typing import Any, Callable, Dict, Optional


class TypeConverters:
    @staticmethod
    def identity(v):
        return v

    @staticmethod
    def toInt(v):
        if isinstance(v, bool):
            raise TypeError(f"Could not convert {v!r} to int")
        if isinstance(v, float):
            if not v.is_integer():
                raise TypeError(f"Could not convert {v} to int")
            return int(v)
        try:
            import numpy as np
            if isinstance(v, np.generic):
                return TypeConverters.toInt(v.item())
        except Exception:
            pass
        return int(v)

    @staticmethod
    def toFloat(v):
        if isinstance(v, bool):
            raise TypeError(f"Could not convert {v!r} to float")
        return float(v)

    @staticmethod
    def toString(v):
        if not isinstance(v, str):
            raise TypeError(f"Could not convert {v!r} to string")
        return v

    @staticmethod
    def toBoolean(v):
        if not isinstance(v, bool):
            raise TypeError(f"Boolean Param requires value of type bool. Found {type(v)}.")
        return v

    @staticmethod
    def toListString(v):
        if isinstance(v, str):
            return [v]
        return [str(x) for x in v]

    @staticmethod
    def toListFloat(v):
        return [float(x) for x in v]

    @staticmethod
    def toListInt(v):
        return [TypeConverters.toInt(x) for x in v]


class Param:
    def __init__(self, parent, name: str, doc: str, typeConverter: Optional[Callable] = None):
        self.parent = parent if isinstance(parent, str) else getattr(parent, "uid", "undefined")
        self.name = name
        self.doc = doc
        self.typeConverter = typeConverter or TypeConverters.identity

    def _copy_new_parent(self, parent):
        p = _copy.copy(self)
        p.parent = parent.uid
        return p

    def __repr__(self):
        return f"Param(parent={self.parent!r}, name={self.name!r}, doc={self.doc!r})"

    def __str__(self):
        return f"{self.parent}__{self.name}"

    def __hash__(self):
        return hash(str(self))

    def __eq__(self, other):
        return isinstance(other, Param) and self.parent == other.parent and self.name == other.name


class Params:
    """Base for everything with params.

    Subclasses declare ``_params = {name: (doc, default, converter)}``.
    """
    _params: Dict[str, tuple] = {}

    def __init_subclass__(cls, **kw):
        super().__init_subclass__(**kw)
        _install_accessors(cls)

    def __init__(self):
        self.uid = f"{type(self).__name__}_{uuid.uuid4().hex[:12]}"
        self._paramMap: Dict[str, Any] = {}
        self._defaultParamMap: Dict[str, Any] = {}
        for name, spec in self._all_specs().items():
            doc, default, conv = spec
            p = Param(self, name, doc, conv)
            object.__setattr__(self, name, p)
            if default is not _NO_DEFAULT:
                self._defaultParamMap[name] = default

    @classmethod
    def _all_specs(cls) -> Dict[str, tuple]:
        specs: Dict[str, tuple] = {}
        for c in reversed(cls.__mro__):
            specs.update(getattr(c, "_params", {}) or {})
        return specs

    # ----------------------------------------------------------- access
    @property
    def params(self):
        return [getattr(self, n) for n in sorted(self._all_specs())]

    def hasParam(self, name: str) -> bool:
        return name in self._all_specs()

    def getParam(self, name: str) -> Param:
        if not self.hasParam(name):
            raise AttributeError(f"{type(self).__name__} has no param {name}")
        return getattr(self, name)

    def _name(self, p) -> str:
        return p.name if isinstance(p, Param) else p

    def isSet(self, p) -> bool:
        return self._name(p) in self._paramMap

    def hasDefault(self, p) -> bool:
        return self._name(p) in self._defaultParamMap

    def isDefined(self, p) -> bool:
        return self.isSet(p) or self.hasDefault(p)

    def getOrDefault(self, p):
        n = self._name(p)
        if n in self._paramMap:
            return self._paramMap[n]
        if n in self._defaultParamMap:
            return self._defaultParamMap[n]
        raise KeyError(f"Failed to find a default value for {n}")

    def _get(self, name, default=None):
        n = self._name(name)
        if n in self._paramMap:
            return self._paramMap[n]
        return self._defaultParamMap.get(n, default)

    def set(self, p, value):
        n = self._name(p)
        spec = self._all_specs()[n]
        conv = spec[2] or TypeConverters.identity
        self._paramMap[n] = conv(value) if value is not None else None
        return self

    def _set(self, **kwargs):
        for k, v in kwargs.items():
            if v is not None:
                self.set(k, v)
        return self

    def _setDefault(self, **kwargs):
        self._defaultParamMap.update(kwargs)
        return self

    def clear(self, p):
        self._paramMap.pop(self._name(p), None)

    def extractParamMap(self, extra=None):
        m = {getattr(self, k): v for k, v in self._defaultParamMap.items()}
        m.update({getattr(self, k): v for k, v in self._paramMap.items()})
        if extra:
            m.update(extra)
        return m

    def explainParam(self, p) -> str:
        n = self._name(p)
        doc = self._all_specs()[n][0]
        parts = []
        if n in self._defaultParamMap:
            parts.append(f"default: {self._defaultParamMap[n]}")
        if n in self._paramMap:
            parts.append(f"current: {self._paramMap[n]}")
        tail = f" ({', '.join(parts)})" if parts else " (undefined)"
        return f"{n}: {doc}{tail}"

    def explainParams(self) -> str:
        return "\n".join(self.explainParam(n) for n in sorted(self._all_specs()))

    # ----------------------------------------------------------- copying
    def copy(self, extra: Optional[dict] = None):
        that = _copy.copy(self)
        that._paramMap = dict(self._paramMap)
        that._defaultParamMap = dict(self._defaultParamMap)
        if extra:
            for p, v in extra.items():
                if isinstance(p, Param) and p.parent != self.uid:
                    continue
                that.set(p, v)
        return that

    def _copyValues(self, to, extra=None):
        for n, v in self._paramMap.items():
            if to.hasParam(n):
                to._paramMap[n] = v
        if extra:
            for p, v in extra.items():
                if isinstance(p, Param) and to.hasParam(p.name) and p.parent == self.uid:
                    to.set(p.name, v)
        return to

    def _resolveParamMap(self, extra):
        """Return the sub-map of ``extra`` that targets this instance."""
        if not extra:
            return {}
        return {p: v for p, v in extra.items() if isinstance(p, Param) and p.parent == self.uid}


class _NoDefault:
    def __repr__(self):
        return "<no default>"


_NO_DEFAULT = _NoDefault()


def _install_accessors(cls):
    """Generate setX/getX for every declared param (idempotent)."""
    for name in cls._all_specs():
        cap = name[0].upper() + name[1:]
        if not hasattr(cls, "set" + cap):
            def setter(self, value, _n=name):
                return self.set(_n, value)
            setter.__name__ = "set" + cap
            setattr(cls, "set" + cap, setter)
        if not hasattr(cls, "get" + cap):
            def getter(self, _n=name):
                return self.getOrDefault(_n)
            getter.__name__ = "get" + cap
            setattr(cls, "get" + cap, getter)
    return cls


def params_class(cls):
    return _install_accessors(cls)


def keyword_init(self, kwargs: dict):
    for k, v in kwargs.items():
        if k == "self" or v is None:
            continue
        if not self.hasParam(k):
            raise TypeError(f"{type(self).__name__} got an unexpected keyword argument '{k}'")
        self.set(k, v)


NO_DEFAULT = _NO_DEFAULT
T = TypeConverters
