"""Spark-compatible data types and schemas.

Every type knows its device storage: scalar numerics are torch tensors of the
matching width, strings are dictionary codes (int32) on device plus a host
dictionary, vectors (``VectorUDT``) are dense ``[n, d]`` matrices — fp64 (Spark's
Double) at course scale, fp32 for the large shapes the MFMA/histogram kernels
stream (``models.util.VECTOR_F64_MAX``).
Reference usage: ``df.dtypes`` splits (ML 03:56,74), ``schema.fields`` /
``IntegerType()`` checks (ML 01:203), DDL strings (ML 12:131,142;
ML 13:54-59).
"""
from __future__ import annotations

import json
import re
from typing import List, Optional

import torch


class DataType:
    torch_dtype: Optional[torch.dtype] = None
    _name = "datatype"

    def simpleString(self) -> str:
        return self._name

    def typeName(self) -> str:
        return self._name

    def jsonValue(self):
        return self._name

    def __eq__(self, other):
        return type(self) is type(other)

    def __hash__(self):
        return hash(type(self).__name__)

    def __repr__(self):
        return f"{type(self).__name__}()"

    @property
    def is_numeric(self) -> bool:
        return isinstance(self, NumericType)


class NullType(DataType):
    _name = "void"
    torch_dtype = torch.float64


class NumericType(DataType):
    pass


class IntegralType(NumericType):
    pass


class FractionalType(NumericType):
    pass


class ByteType(IntegralType):
    _name = "tinyint"
    torch_dtype = torch.int8


class ShortType(IntegralType):
    _name = "smallint"
    torch_dtype = torch.int16


class IntegerType(IntegralType):
    _name = "int"
    torch_dtype = torch.int32

    def typeName(self):
        return "integer"


class LongType(IntegralType):
    _name = "bigint"
    torch_dtype = torch.int64

    def typeName(self):
        return "long"


class FloatType(FractionalType):
    _name = "float"
    torch_dtype = torch.float32


class DoubleType(FractionalType):
    _name = "double"
    torch_dtype = torch.float64


class DecimalType(FractionalType):
    _name = "decimal"
    torch_dtype = torch.float64


class BooleanType(DataType):
    _name = "boolean"
    torch_dtype = torch.bool


class StringType(DataType):
    """Stored as int32 dictionary codes on device + a host dictionary."""
    _name = "string"
    torch_dtype = torch.int32


class DateType(DataType):
    """Days since epoch (int32)."""
    _name = "date"
    torch_dtype = torch.int32


class TimestampType(DataType):
    """Microseconds since epoch (int64)."""
    _name = "timestamp"
    torch_dtype = torch.int64


class BinaryType(DataType):
    _name = "binary"
    torch_dtype = torch.int32


class VectorUDT(DataType):
    """ML vector column: dense [n, d] on device (fp64 at course scale, fp32 for large matrices)."""
    _name = "vector"
    torch_dtype = torch.float32

    def typeName(self):
        return "vector"


class ArrayType(DataType):
    """Fixed-width numeric arrays stored like vectors ([n, d])."""

    def __init__(self, elementType: DataType = None, containsNull: bool = True):
        self.elementType = elementType or DoubleType()
        self.containsNull = containsNull
        self.torch_dtype = self.elementType.torch_dtype

    def simpleString(self):
        return f"array<{self.elementType.simpleString()}>"

    def __eq__(self, other):
        return isinstance(other, ArrayType) and other.elementType == self.elementType

    def __hash__(self):
        return hash(("array", self.elementType))

    def __repr__(self):
        return f"ArrayType({self.elementType!r}, {self.containsNull})"


class StructField:
    def __init__(self, name: str, dataType: DataType, nullable: bool = True, metadata: Optional[dict] = None):
        self.name = name
        self.dataType = dataType
        self.nullable = nullable
        self.metadata = metadata or {}

    def simpleString(self):
        return f"{self.name}:{self.dataType.simpleString()}"

    def __eq__(self, other):
        """Spark's field equality: name, type, nullability and metadata all count (so
        ``set(a.schema.fields) ^ set(b.schema.fields)`` of Labs/ML 05L:257 finds schema drift)."""
        return (isinstance(other, StructField) and self.name == other.name and self.dataType == other.dataType
                and bool(self.nullable) == bool(other.nullable) and self.metadata == other.metadata)

    def __hash__(self):
        return hash((self.name, self.dataType, bool(self.nullable),
                     json.dumps(self.metadata, sort_keys=True, default=str)))

    def __repr__(self):
        return f"StructField('{self.name}', {self.dataType!r}, {self.nullable})"


class StructType(DataType):
    _name = "struct"

    def __init__(self, fields: Optional[List[StructField]] = None):
        self.fields = list(fields or [])

    def add(self, field, data_type=None, nullable=True, metadata=None):
        if isinstance(field, StructField):
            self.fields.append(field)
        else:
            if isinstance(data_type, str):
                data_type = _parse_type(data_type)
            self.fields.append(StructField(field, data_type, nullable, metadata))
        return self

    @property
    def names(self):
        return [f.name for f in self.fields]

    def fieldNames(self):
        return self.names

    def __iter__(self):
        return iter(self.fields)

    def __len__(self):
        return len(self.fields)

    def __getitem__(self, key):
        if isinstance(key, int):
            return self.fields[key]
        for f in self.fields:
            if f.name == key:
                return f
        raise KeyError(f"No StructField named {key}")

    def __contains__(self, name):
        return name in self.names

    def simpleString(self):
        return "struct<" + ",".join(f.simpleString() for f in self.fields) + ">"

    def __eq__(self, other):
        return isinstance(other, StructType) and self.fields == other.fields

    def __hash__(self):
        return hash(tuple(f.name for f in self.fields))

    def __repr__(self):
        return "StructType([" + ", ".join(repr(f) for f in self.fields) + "])"

    def jsonValue(self):
        return {"type": "struct", "fields": [
            {"name": f.name, "type": f.dataType.simpleString(), "nullable": f.nullable, "metadata": f.metadata}
            for f in self.fields]}

    def json(self):
        return json.dumps(self.jsonValue())

    @classmethod
    def fromDDL(cls, ddl: str) -> "StructType":
        return _parse_datatype_string(ddl)

    @staticmethod
    def fromJson(s):
        d = json.loads(s) if isinstance(s, str) else s
        return StructType([StructField(f["name"], _parse_type(f["type"]), f.get("nullable", True),
                                       f.get("metadata", {})) for f in d["fields"]])


_ALIASES = {
    "string": StringType, "str": StringType, "varchar": StringType, "char": StringType,
    "double": DoubleType, "float64": DoubleType, "float": FloatType, "real": FloatType, "float32": FloatType,
    "int": IntegerType, "integer": IntegerType, "int32": IntegerType,
    "bigint": LongType, "long": LongType, "int64": LongType,
    "smallint": ShortType, "short": ShortType, "tinyint": ByteType, "byte": ByteType,
    "boolean": BooleanType, "bool": BooleanType,
    "date": DateType, "timestamp": TimestampType, "binary": BinaryType,
    "vector": VectorUDT, "void": NullType, "null": NullType, "decimal": DecimalType,
}


def _parse_type(s: str) -> DataType:
    s = s.strip()
    low = s.lower()
    m = re.match(r"array\s*<(.+)>$", low)
    if m:
        return ArrayType(_parse_type(m.group(1)))
    m = re.match(r"(decimal|numeric)\s*(\(.*\))?$", low)
    if m:
        return DecimalType()
    if low.startswith("struct<"):
        return _parse_datatype_string(s[7:-1].replace(":", " "))
    if low in _ALIASES:
        return _ALIASES[low]()
    raise ValueError(f"Unsupported type string: {s!r}")


def _split_top(s: str) -> List[str]:
    out, depth, cur = [], 0, []
    for ch in s:
        if ch in "<(":
            depth += 1
        elif ch in ">)":
            depth -= 1
        if ch == "," and depth == 0:
            out.append("".join(cur))
            cur = []
        else:
            cur.append(ch)
    if cur:
        out.append("".join(cur))
    return [x.strip() for x in out if x.strip()]


def _parse_datatype_string(s: str) -> DataType:
    """Parse a DDL schema ('a int, b string') or a bare type ('double')."""
    s = s.strip()
    parts = _split_top(s)
    if len(parts) == 1 and (" " not in parts[0].strip() and ":" not in parts[0]):
        return _parse_type(parts[0])
    fields = []
    for p in parts:
        p = p.replace(":", " ", 1) if ":" in p and " " not in p.split(":")[0] else p
        name, typ = p.strip().split(None, 1)
        fields.append(StructField(name.strip("`"), _parse_type(typ)))
    return StructType(fields)


def to_schema(schema) -> Optional[StructType]:
    if schema is None or isinstance(schema, StructType):
        return schema
    if isinstance(schema, str):
        t = _parse_datatype_string(schema)
        if not isinstance(t, StructType):
            raise ValueError("expected a struct schema")
        return t
    if isinstance(schema, (list, tuple)):
        return None
    raise TypeError(f"bad schema {schema!r}")


def to_type(t) -> DataType:
    if isinstance(t, DataType):
        return t
    if isinstance(t, str):
        return _parse_type(t)
    if t is float:
        return DoubleType()
    if t is int:
        return LongType()
    if t is str:
        return StringType()
    if t is bool:
        return BooleanType()
    raise TypeError(f"bad data type {t!r}")


def from_torch(dt: torch.dtype) -> DataType:
    return {torch.float64: DoubleType(), torch.float32: FloatType(), torch.int32: IntegerType(),
            torch.int64: LongType(), torch.bool: BooleanType(), torch.int16: ShortType(),
            torch.int8: ByteType(), torch.uint8: ShortType()}[dt]


def numeric_result(a: DataType, b: DataType) -> DataType:
    order = [ByteType, ShortType, IntegerType, LongType, FloatType, DoubleType]
    ia = next((i for i, c in enumerate(order) if isinstance(a, c)), 5)
    ib = next((i for i, c in enumerate(order) if isinstance(b, c)), 5)
    return order[max(ia, ib)]()


class Row(tuple):
    """Spark Row: a tuple with named field access."""

    def __new__(cls, *args, **kwargs):
        if kwargs:
            r = tuple.__new__(cls, tuple(kwargs.values()))
            r.__fields__ = list(kwargs.keys())
            return r
        r = tuple.__new__(cls, args)
        r.__fields__ = None
        return r

    @classmethod
    def _make(cls, names, values):
        r = tuple.__new__(cls, tuple(values))
        r.__fields__ = list(names)
        return r

    def asDict(self, recursive: bool = False):
        return dict(zip(self.__fields__ or [], self))

    def __getattr__(self, item):
        if item.startswith("__"):
            raise AttributeError(item)
        f = self.__fields__ or []
        if item in f:
            return self[f.index(item)]
        raise AttributeError(item)

    def __getitem__(self, item):
        if isinstance(item, str):
            return tuple.__getitem__(self, (self.__fields__ or []).index(item))
        return tuple.__getitem__(self, item)

    def __contains__(self, item):
        return item in (self.__fields__ or [])

    def __repr__(self):
        if self.__fields__:
            return "Row(" + ", ".join(f"{k}={v!r}" for k, v in zip(self.__fields__, self)) + ")"
        return "<Row(" + ", ".join(repr(v) for v in self) + ")>"

    def __reduce__(self):
        return (Row._make, (self.__fields__, tuple(self)))
