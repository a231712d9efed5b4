"""Spark-style Params (pyspark.ml.param-compatible surface).

The reference passes no hyper-parameters at all: every estimator
runs on Spark's defaults, so each estimator here declares Spark's default values
explicitly (``_params`` tables) and they are written to the saved model's
``defaultParamMap`` exactly as Spark does.

A class declares ``_params = {"maxIter": (100, "max number of iterations (>= 0)", int), ...}``;
``__init_subclass__`` materialises ``Param`` objects plus ``getX``/``setX`` methods
for every entry in the MRO, and the constructor accepts the params as keywords.
"""
from __future__ import annotations

import copy as _copy
import uuid
from typing import Any, Callable, Dict, Optional


class Param:
    def __init__(self, parent: str, name: str, doc: str, typeConverter: Optional[Callable] = None):
        self.parent = parent
        self.name = name
        self.doc = doc
        self.typeConverter = typeConverter or (lambda v: v)

    def _copy_new_parent(self, parent: str) -> "Param":
        p = _copy.copy(self)
        p.parent = parent
        return p

    def __repr__(self):
        return f"Param(parent={self.parent!r}, name={self.name!r}, doc={self.doc!r})"

    def __hash__(self):
        return hash((self.parent, self.name))

    def __eq__(self, other):
        return isinstance(other, Param) and self.parent == other.parent and self.name == other.name


class TypeConverters:
    @staticmethod
    def identity(v):
        return v

    @staticmethod
    def toInt(v):
        if isinstance(v, bool) or float(v) != int(float(v)):
            raise TypeError(f"could not convert {v!r} to int")
        return int(v)

    @staticmethod
    def toFloat(v):
        return float(v)

    @staticmethod
    def toString(v):
        if not isinstance(v, str):
            raise TypeError(f"could not convert {v!r} to string")
        return v

    @staticmethod
    def toBoolean(v):
        if not isinstance(v, bool):
            raise TypeError(f"could not convert {v!r} to bool")
        return v

    @staticmethod
    def toListString(v):
        return [TypeConverters.toString(x) for x in v]

    @staticmethod
    def toListFloat(v):
        return [float(x) for x in v]

    @staticmethod
    def toListInt(v):
        return [int(x) for x in v]


_CONV = {int: TypeConverters.toInt, float: TypeConverters.toFloat, str: TypeConverters.toString,
         bool: TypeConverters.toBoolean, list: lambda v: list(v), "liststr": TypeConverters.toListString,
         "listfloat": TypeConverters.toListFloat, None: TypeConverters.identity}


def _cap(name: str) -> str:
    return name[0].upper() + name[1:]


class Params:
    """Base of everything with parameters (estimators, models, transformers, evaluators)."""

    _params: Dict[str, tuple] = {}

    def __init_subclass__(cls, **kw):
        super().__init_subclass__(**kw)
        specs: Dict[str, tuple] = {}
        for base in reversed(cls.__mro__):
            specs.update(base.__dict__.get("_params", {}))
        cls._all_params = specs
        for name, spec in specs.items():
            getter, setter = "get" + _cap(name), "set" + _cap(name)
            if getter not in cls.__dict__ and not _defined_in_mro(cls, getter):
                setattr(cls, getter, _make_getter(name))
            if setter not in cls.__dict__ and not _defined_in_mro(cls, setter):
                setattr(cls, setter, _make_setter(name))

    def __init__(self, **kwargs):
        self.uid = self._random_uid()
        self._paramMap: Dict[str, Any] = {}
        self._defaultParamMap: Dict[str, Any] = {}
        self._param_objs: Dict[str, Param] = {}
        for name, spec in getattr(type(self), "_all_params", {}).items():
            default, doc = spec[0], spec[1]
            conv = _CONV.get(spec[2] if len(spec) > 2 else None, TypeConverters.identity)
            self._param_objs[name] = Param(self.uid, name, doc, conv)
            if default is not _NoDefault:
                self._defaultParamMap[name] = default
        self._set(**kwargs)

    @classmethod
    def _random_uid(cls) -> str:
        return f"{cls.__name__}_{uuid.uuid4().hex[-12:]}"

    def __getattr__(self, name: str):
        # pyspark exposes every param as an attribute (``dt.maxDepth`` is a Param), which is what
        # ParamGridBuilder.addGrid and fit(df, {param: value}) take. Only reached when normal
        # lookup fails, so real attributes and the generated get*/set* methods win.
        po = self.__dict__.get("_param_objs")
        if po is not None and name in po:
            return po[name]
        raise AttributeError(f"{type(self).__name__!r} object has no attribute {name!r}")

    # ------------------------------------------------------------------ pyspark API
    @property
    def params(self):
        return [self._param_objs[k] for k in sorted(self._param_objs)]

    def hasParam(self, name: str) -> bool:
        return name in self._param_objs

    def getParam(self, name: str) -> Param:
        return self._param_objs[name]

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
        raise KeyError(f"param {n} is not set and has no default")

    def get(self, name, default=None):
        try:
            return self.getOrDefault(name)
        except KeyError:
            return default

    def set(self, param, value):
        return self._set(**{self._name(param): value})

    def _set(self, **kwargs):
        for k, v in kwargs.items():
            if k not in self._param_objs:
                raise TypeError(f"{type(self).__name__} has no param {k!r}")
            if v is None:
                self._paramMap.pop(k, None)
                continue
            self._paramMap[k] = self._param_objs[k].typeConverter(v)
        return self

    def _setDefault(self, **kwargs):
        self._defaultParamMap.update(kwargs)
        return self

    def setParams(self, **kwargs):
        return self._set(**kwargs)

    def clear(self, param) -> None:
        self._paramMap.pop(self._name(param), None)

    def extractParamMap(self, extra: Optional[Dict] = None) -> Dict[Param, Any]:
        m = {self._param_objs[k]: v for k, v in self._defaultParamMap.items() if k in self._param_objs}
        m.update({self._param_objs[k]: v for k, v in self._paramMap.items()})
        if extra:
            for k, v in extra.items():
                m[k if isinstance(k, Param) else self._param_objs[k]] = v
        return m

    def explainParam(self, p) -> str:
        n = self._name(p)
        obj = self._param_objs[n]
        parts = []
        if n in self._defaultParamMap:
            parts.append(f"default: {self._defaultParamMap[n]}")
        if n in self._paramMap:
            parts.append(f"current: {self._paramMap[n]}")
        return f"{n}: {obj.doc} ({', '.join(parts) if parts else 'undefined'})"

    def explainParams(self) -> str:
        return "\n".join(self.explainParam(k) for k in sorted(self._param_objs))

    def copy(self, extra: Optional[Dict] = None):
        that = _copy.copy(self)
        that._paramMap = dict(self._paramMap)
        that._defaultParamMap = dict(self._defaultParamMap)
        if extra:
            for k, v in extra.items():
                that._set(**{self._name(k): v})
        return that

    def _copyValues(self, to: "Params", extra=None) -> "Params":
        for k, v in self._paramMap.items():
            if k in to._param_objs:
                to._paramMap[k] = v
        for k, v in self._defaultParamMap.items():
            if k in to._param_objs and k not in to._defaultParamMap:
                to._defaultParamMap[k] = v
        return to

    def __repr__(self):
        return self.uid


class _NoDefaultType:
    def __repr__(self):
        return "<no default>"


_NoDefault = _NoDefaultType()
NO_DEFAULT = _NoDefault


def _defined_in_mro(cls, attr: str) -> bool:
    for base in cls.__mro__[1:]:
        if attr in base.__dict__ and not getattr(base.__dict__[attr], "_cml_generated", False):
            return True
    return False


def _make_getter(name: str):
    def getter(self):
        return self.getOrDefault(name)
    getter.__name__ = "get" + _cap(name)
    getter._cml_generated = True
    return getter


def _make_setter(name: str):
    def setter(self, value):
        return self._set(**{name: value})
    setter.__name__ = "set" + _cap(name)
    setter._cml_generated = True
    return setter
