"""Column expressions evaluated as fused device tensor ops.

An expression tree is evaluated per partition against a ``Batch``; every
node returns a ``ColumnData`` (device tensor + validity + dictionary for
strings).  String predicates are resolved against the (small, host)
dictionary and then executed as integer ops on the GPU.
Reference usage: ``col``/``lit``/``when``/``translate``/``cast``/``log``/
``exp``/``isin``/``~`` etc. (ML 01:93,203-207,234; Labs/ML 00L:96-108;
ML 10:46,179,302; ML 11:38,86; ML 13:37-41).
"""
from __future__ import annotations

import math
from typing import Any, Callable, List, Optional

import numpy as np
import torch

from . import types as T
from .batch import (ColumnData, full_column, infer_literal_type, map_dictionary, unify_dictionaries)


class EvalContext:
    """Per-partition evaluation context."""

    def __init__(self, session=None, partition_index: int = 0, row_offset: int = 0):
        self.session = session
        self.partition_index = partition_index
        self.row_offset = row_offset


class Expr:
    children: List["Expr"] = []

    def eval(self, b, ctx: EvalContext) -> ColumnData:  # pragma: no cover - abstract
        raise NotImplementedError

    def name(self) -> str:
        return str(self)

    def references(self) -> List[str]:
        out = []
        for c in self.children:
            out.extend(c.references())
        return out

    def is_aggregate(self) -> bool:
        return any(c.is_aggregate() for c in self.children)


def _and_valid(*cols: ColumnData):
    v = None
    for c in cols:
        if c.valid is not None:
            v = c.valid if v is None else (v & c.valid)
    return v


# ------------------------------------------------------------------ leaves
class ColRef(Expr):
    def __init__(self, name: str):
        self.col_name = name
        self.children = []

    def eval(self, b, ctx):
        if self.col_name in b.columns:
            return b.columns[self.col_name]
        # case-insensitive resolution (Spark default)
        for k in b.columns:
            if k.lower() == self.col_name.lower():
                return b.columns[k]
        if "." in self.col_name:
            tail = self.col_name.split(".", 1)[1]
            if tail in b.columns:
                return b.columns[tail]
        raise AnalysisException(f"cannot resolve '{self.col_name}' given input columns: {b.names}")

    def name(self):
        return self.col_name.split(".", 1)[1] if "." in self.col_name and not self.col_name.startswith("`") \
            else self.col_name

    def references(self):
        return [self.col_name]

    def __str__(self):
        return self.col_name


class Star(Expr):
    def __init__(self, table: Optional[str] = None):
        self.table = table
        self.children = []

    def __str__(self):
        return "*"


class Lit(Expr):
    def __init__(self, value, dtype: Optional[T.DataType] = None):
        self.value = value
        self.dtype = dtype or infer_literal_type(value)
        self.children = []

    def eval(self, b, ctx):
        return full_column(self.value, self.dtype, b.n, b.device)

    def __str__(self):
        return "NULL" if self.value is None else str(self.value)


class AnalysisException(Exception):
    pass


# ----------------------------------------------------------- arithmetic
_CMP = {"==": torch.eq, "!=": torch.ne, "<": torch.lt, "<=": torch.le, ">": torch.gt, ">=": torch.ge}


def _string_compare(op, lc: ColumnData, rc: ColumnData):
    lc, rc = unify_dictionaries([lc, rc])
    return _CMP[op](lc.values, rc.values)


def _to_float(c: ColumnData):
    if isinstance(c.dtype, T.BooleanType):
        return c.values.to(torch.float64)
    return c.values


class BinOp(Expr):
    def __init__(self, op: str, l: Expr, r: Expr):
        self.op, self.l, self.r = op, l, r
        self.children = [l, r]

    def __str__(self):
        return f"({self.l} {self.op} {self.r})"

    def eval(self, b, ctx):
        op = self.op
        if op in ("and", "or"):
            lc, rc = self.l.eval(b, ctx), self.r.eval(b, ctx)
            lv, rv = lc.values.bool(), rc.values.bool()
            lval, rval = lc.valid_mask(), rc.valid_mask()
            if op == "and":
                val = lv & rv
                # null AND false = false; null AND true = null
                valid = (lval & rval) | (lval & ~lv) | (rval & ~rv)
            else:
                val = lv | rv
                valid = (lval & rval) | (lval & lv) | (rval & rv)
            if lc.valid is None and rc.valid is None:
                valid = None
            return ColumnData(val & (valid if valid is not None else True), T.BooleanType(), valid)
        if isinstance(self.r, Lit) and isinstance(self.r.value, str) and op in _CMP:
            lc = self.l.eval(b, ctx)
            if isinstance(lc.dtype, T.StringType):
                return self._cmp_string_lit(op, lc, self.r.value)
        if isinstance(self.l, Lit) and isinstance(self.l.value, str) and op in _CMP:
            rc = self.r.eval(b, ctx)
            if isinstance(rc.dtype, T.StringType):
                flip = {"==": "==", "!=": "!=", "<": ">", "<=": ">=", ">": "<", ">=": "<="}[op]
                return self._cmp_string_lit(flip, rc, self.l.value)
        lc, rc = self.l.eval(b, ctx), self.r.eval(b, ctx)
        valid = _and_valid(lc, rc)
        if op == "<=>":
            lval, rval = lc.valid_mask(), rc.valid_mask()
            if isinstance(lc.dtype, T.StringType):
                eq = _string_compare("==", lc, rc)
            else:
                eq = lc.values == rc.values
            out = (lval & rval & eq) | (~lval & ~rval)
            return ColumnData(out, T.BooleanType())
        if op in _CMP:
            if isinstance(lc.dtype, T.StringType) or isinstance(rc.dtype, T.StringType):
                if isinstance(lc.dtype, T.StringType) and isinstance(rc.dtype, T.StringType):
                    out = _string_compare(op, lc, rc)
                else:
                    # string vs numeric: cast string to double (Spark semantics)
                    lf = _cast(lc, T.DoubleType()) if isinstance(lc.dtype, T.StringType) else lc
                    rf = _cast(rc, T.DoubleType()) if isinstance(rc.dtype, T.StringType) else rc
                    out = _CMP[op](lf.values, rf.values)
                    valid = _and_valid(lf, rf)
            else:
                out = _CMP[op](_to_float(lc), _to_float(rc))
            return ColumnData(out, T.BooleanType(), valid)
        if op in ("&", "|", "^") and isinstance(lc.dtype, T.BooleanType):
            f = {"&": torch.logical_and, "|": torch.logical_or, "^": torch.logical_xor}[op]
            return ColumnData(f(lc.values, rc.values), T.BooleanType(), valid)
        if isinstance(lc.dtype, T.StringType) or isinstance(rc.dtype, T.StringType):
            lc = _cast(lc, T.DoubleType()) if isinstance(lc.dtype, T.StringType) else lc
            rc = _cast(rc, T.DoubleType()) if isinstance(rc.dtype, T.StringType) else rc
            valid = _and_valid(lc, rc)
        if isinstance(lc.dtype, (T.VectorUDT,)) or isinstance(rc.dtype, (T.VectorUDT,)):
            a = lc.values if lc.values.dim() == 2 else lc.values[:, None]
            c = rc.values if rc.values.dim() == 2 else rc.values[:, None]
            f = {"+": torch.add, "-": torch.sub, "*": torch.mul, "/": torch.div}[op]
            return ColumnData(f(a.float(), c.float()), T.VectorUDT(), valid)
        lt, rt = lc.dtype, rc.dtype
        if isinstance(lt, T.NullType):
            lt = rt
        if isinstance(rt, T.NullType):
            rt = lt
        if op == "/":
            a, c = lc.values.to(torch.float64), rc.values.to(torch.float64)
            zero = c == 0
            out = a / torch.where(zero, torch.ones_like(c), c)
            v2 = ~zero if valid is None else valid & ~zero
            return ColumnData(out, T.DoubleType(), v2 if bool(zero.any()) else valid)
        res_t = T.numeric_result(lt, rt) if (isinstance(lt, T.NumericType) and isinstance(rt, T.NumericType)) \
            else T.DoubleType()
        a = lc.values.to(res_t.torch_dtype)
        c = rc.values.to(res_t.torch_dtype)
        if op == "+":
            out = a + c
        elif op == "-":
            out = a - c
        elif op == "*":
            out = a * c
        elif op == "%":
            zero = c == 0
            cc = torch.where(zero, torch.ones_like(c), c)
            out = torch.fmod(a, cc)
            if bool(zero.any()):
                valid = ~zero if valid is None else valid & ~zero
        elif op == "&":
            out = a & c
        elif op == "|":
            out = a | c
        elif op == "^":
            out = a ^ c
        elif op == "**":
            out = torch.pow(a.double(), c.double())
            res_t = T.DoubleType()
        else:
            raise AnalysisException(f"unknown operator {op}")
        return ColumnData(out, res_t, valid)

    def _cmp_string_lit(self, op, lc: ColumnData, s: str):
        d = lc.dictionary if lc.dictionary is not None else np.array([], dtype=object)
        codes = lc.values
        if op in ("==", "!="):
            hits = np.nonzero(d == s)[0] if len(d) else np.array([], dtype=np.int64)
            if len(hits):
                out = codes == int(hits[0])
            else:
                out = torch.zeros_like(codes, dtype=torch.bool)
            if op == "!=":
                out = ~out
        else:
            # dictionaries are sorted: order of codes == lexicographic order
            pos_l = int(np.searchsorted(d.astype(str), s, side="left")) if len(d) else 0
            pos_r = int(np.searchsorted(d.astype(str), s, side="right")) if len(d) else 0
            if op == "<":
                out = codes < pos_l
            elif op == "<=":
                out = codes < pos_r
            elif op == ">":
                out = codes >= pos_r
            else:
                out = codes >= pos_l
        return ColumnData(out, T.BooleanType(), lc.valid)


class Unary(Expr):
    def __init__(self, op: str, x: Expr):
        self.op, self.x = op, x
        self.children = [x]

    def __str__(self):
        return f"({self.op}{self.x})" if self.op != "not" else f"(NOT {self.x})"

    def eval(self, b, ctx):
        c = self.x.eval(b, ctx)
        if self.op == "not":
            return ColumnData(~c.values.bool(), T.BooleanType(), c.valid)
        if self.op == "-":
            return ColumnData(-c.values, c.dtype, c.valid)
        raise AnalysisException(self.op)


# ------------------------------------------------------------------ casts
def _cast(c: ColumnData, dt: T.DataType) -> ColumnData:
    src = c.dtype
    if src == dt:
        return c
    if isinstance(dt, T.StringType):
        if isinstance(src, T.StringType):
            return c
        vals = c.to_numpy()
        strs = np.array([None if v is None else _fmt(v, src) for v in vals], dtype=object)
        from .batch import column_from_numpy
        return column_from_numpy(strs, T.StringType(), c.device)
    if isinstance(src, T.StringType):
        d = c.dictionary if c.dictionary is not None else np.array([], dtype=object)
        conv, ok = [], []
        for s in d.tolist():
            try:
                if isinstance(dt, T.BooleanType):
                    v = {"true": 1.0, "false": 0.0, "1": 1.0, "0": 0.0}[s.strip().lower()]
                elif isinstance(dt, T.DateType):
                    import datetime as _dt
                    v = float((_dt.date.fromisoformat(s.strip()[:10]) - _dt.date(1970, 1, 1)).days)
                else:
                    v = float(s.strip())
                    if isinstance(dt, T.IntegralType):
                        if math.isnan(v) or math.isinf(v):
                            raise ValueError
                        v = float(math.trunc(v))
                conv.append(v)
                ok.append(True)
            except (ValueError, KeyError, AttributeError):
                conv.append(0.0)
                ok.append(False)
        lut = torch.tensor(conv + [0.0], dtype=torch.float64, device=c.device)
        okt = torch.tensor(ok + [False], dtype=torch.bool, device=c.device)
        codes = c.values.long()
        codes = torch.where(codes < 0, torch.full_like(codes, len(d)), codes)
        vals = lut[codes]
        valid = okt[codes]
        if c.valid is not None:
            valid = valid & c.valid
        out_t = dt.torch_dtype if not isinstance(dt, T.BooleanType) else torch.bool
        return ColumnData(vals.to(out_t) if out_t != torch.bool else vals != 0, dt,
                          None if bool(valid.all()) else valid)
    if isinstance(dt, (T.VectorUDT, T.ArrayType)):
        v = c.values if c.values.dim() == 2 else c.values[:, None]
        return ColumnData(v.float(), dt, c.valid, meta=c.meta)
    if isinstance(dt, T.BooleanType):
        return ColumnData(c.values != 0, dt, c.valid)
    if isinstance(dt, T.IntegralType) and c.values.dtype.is_floating_point:
        v = c.values
        bad = torch.isnan(v) | torch.isinf(v)
        vals = torch.trunc(torch.where(bad, torch.zeros_like(v), v)).to(dt.torch_dtype)
        valid = c.valid
        if bool(bad.any()):
            valid = ~bad if valid is None else valid & ~bad
        return ColumnData(vals, dt, valid)
    if isinstance(dt, T.NullType):
        return c
    return ColumnData(c.values.to(dt.torch_dtype), dt, c.valid, meta=c.meta)


def _fmt(v, src):
    if isinstance(v, bool) or isinstance(src, T.BooleanType):
        return "true" if v else "false"
    if isinstance(v, float):
        if v == int(v) and abs(v) < 1e15:
            return f"{v:.1f}"
        return repr(v)
    return str(v)


class Cast(Expr):
    def __init__(self, x: Expr, dt: T.DataType):
        self.x, self.dt = x, dt
        self.children = [x]

    def eval(self, b, ctx):
        return _cast(self.x.eval(b, ctx), self.dt)

    def name(self):
        return f"CAST({self.x.name()} AS {self.dt.simpleString().upper()})"

    def __str__(self):
        return self.name()


class Alias(Expr):
    def __init__(self, x: Expr, alias: str, metadata: Optional[dict] = None):
        self.x, self.alias, self.metadata = x, alias, metadata
        self.children = [x]

    def eval(self, b, ctx):
        c = self.x.eval(b, ctx)
        if self.metadata:
            c = c.with_meta(dict(self.metadata))
        return c

    def name(self):
        return self.alias

    def __str__(self):
        return f"{self.x} AS {self.alias}"


class IsNull(Expr):
    def __init__(self, x: Expr, negate: bool = False):
        self.x, self.negate = x, negate
        self.children = [x]

    def eval(self, b, ctx):
        c = self.x.eval(b, ctx)
        m = c.valid_mask()
        return ColumnData(m if self.negate else ~m, T.BooleanType())

    def __str__(self):
        return f"({self.x} IS {'NOT ' if self.negate else ''}NULL)"


class IsNaN(Expr):
    def __init__(self, x: Expr):
        self.x = x
        self.children = [x]

    def eval(self, b, ctx):
        c = self.x.eval(b, ctx)
        v = c.values
        out = torch.isnan(v) if v.dtype.is_floating_point else torch.zeros_like(v, dtype=torch.bool)
        return ColumnData(out, T.BooleanType(), c.valid)

    def __str__(self):
        return f"isnan({self.x})"


class IsIn(Expr):
    def __init__(self, x: Expr, values: list):
        self.x, self.values = x, list(values)
        self.children = [x]

    def eval(self, b, ctx):
        c = self.x.eval(b, ctx)
        if isinstance(c.dtype, T.StringType):
            d = c.dictionary if c.dictionary is not None else np.array([], dtype=object)
            s = set(str(v) for v in self.values)
            lut = torch.tensor([v in s for v in d.tolist()] + [False], dtype=torch.bool, device=c.device)
            codes = c.values.long()
            codes = torch.where(codes < 0, torch.full_like(codes, len(d)), codes)
            return ColumnData(lut[codes], T.BooleanType(), c.valid)
        vals = torch.tensor([float(v) for v in self.values], dtype=torch.float64, device=c.device)
        out = torch.isin(c.values.to(torch.float64), vals)
        return ColumnData(out, T.BooleanType(), c.valid)

    def __str__(self):
        return f"({self.x} IN ({', '.join(map(str, self.values))}))"


class CaseWhen(Expr):
    def __init__(self, branches, otherwise: Optional[Expr] = None):
        self.branches = list(branches)
        self.otherwise = otherwise
        self.children = [e for br in self.branches for e in br] + ([otherwise] if otherwise is not None else [])

    def eval(self, b, ctx):
        vals = [v.eval(b, ctx) for _, v in self.branches]
        other = self.otherwise.eval(b, ctx) if self.otherwise is not None else None
        allc = vals + ([other] if other is not None else [])
        dts = [c.dtype for c in allc if not isinstance(c.dtype, T.NullType)]
        dt = dts[0] if dts else T.NullType()
        if any(isinstance(x, T.StringType) for x in dts):
            dt = T.StringType()
            allc = [(_cast(c, dt) if not isinstance(c.dtype, T.StringType) and not isinstance(c.dtype, T.NullType)
                     else c) for c in allc]
            fixed = []
            for c in allc:
                if isinstance(c.dtype, T.NullType):
                    c = full_column(None, T.StringType(), b.n, b.device)
                fixed.append(c)
            allc = unify_dictionaries(fixed)
        else:
            for x in dts:
                if isinstance(x, T.NumericType) and isinstance(dt, T.NumericType):
                    dt = T.numeric_result(dt, x)
            allc = [(_cast(c, dt) if not isinstance(c.dtype, T.NullType) else c) for c in allc]
        vals = allc[: len(vals)]
        other = allc[len(vals)] if other is not None else None
        if other is None:
            out_v = torch.zeros_like(vals[0].values)
            out_valid = torch.zeros(b.n, dtype=torch.bool, device=b.device)
        else:
            out_v = other.values.to(vals[0].values.dtype).clone()
            out_valid = other.valid_mask().clone()
        decided = torch.zeros(b.n, dtype=torch.bool, device=b.device)
        for (cond, _), v in zip(self.branches, vals):
            cc = cond.eval(b, ctx)
            take = cc.values.bool() & cc.valid_mask() & ~decided
            if out_v.dim() == 2:
                out_v = torch.where(take[:, None], v.values.to(out_v.dtype), out_v)
            else:
                out_v = torch.where(take, v.values.to(out_v.dtype), out_v)
            out_valid = torch.where(take, v.valid_mask(), out_valid)
            decided |= take
        dic = vals[0].dictionary if isinstance(dt, T.StringType) else None
        return ColumnData(out_v, dt, None if bool(out_valid.all()) else out_valid, dic)

    def __str__(self):
        s = " ".join(f"WHEN {c} THEN {v}" for c, v in self.branches)
        return f"CASE {s}{' ELSE ' + str(self.otherwise) if self.otherwise is not None else ''} END"


class Func(Expr):
    """Generic elementwise function over evaluated argument columns."""

    def __init__(self, fname: str, fn: Callable, args: List[Expr], display: Optional[str] = None):
        self.fname, self.fn, self.args = fname, fn, list(args)
        self.children = list(args)
        self.display = display
        self.fuse = None  # K18 opcode tag when the function has a fused-kernel equivalent (sql/fused.py)

    def eval(self, b, ctx):
        return self.fn(b, ctx, [a.eval(b, ctx) for a in self.args])

    def name(self):
        if self.display:
            return self.display
        return f"{self.fname}({', '.join(a.name() for a in self.args)})"

    def __str__(self):
        return self.name()


class RowFunc(Expr):
    """Function needing partition context (rand, monotonically_increasing_id, ...)."""

    def __init__(self, fname: str, fn: Callable, display: Optional[str] = None):
        self.fname, self.fn, self.display = fname, fn, display
        self.children = []

    def eval(self, b, ctx):
        return self.fn(b, ctx)

    def name(self):
        return self.display or f"{self.fname}()"

    def __str__(self):
        return self.name()


class SortOrder(Expr):
    def __init__(self, x: Expr, ascending: bool = True, nulls_first: Optional[bool] = None):
        self.x, self.ascending = x, ascending
        self.nulls_first = ascending if nulls_first is None else nulls_first
        self.children = [x]

    def eval(self, b, ctx):
        return self.x.eval(b, ctx)

    def name(self):
        return self.x.name()

    def __str__(self):
        return f"{self.x} {'ASC' if self.ascending else 'DESC'}"


# -------------------------------------------------------------- Column API
def _to_expr(x) -> Expr:
    if isinstance(x, Column):
        return x._expr
    if isinstance(x, Expr):
        return x
    return Lit(x)


class Column:
    """PySpark-compatible Column wrapper around an expression tree."""

    def __init__(self, expr: Expr):
        self._expr = expr

    # -- naming
    def alias(self, *names, metadata=None) -> "Column":
        return Column(Alias(self._expr, names[0], metadata))

    name = alias

    def cast(self, dt) -> "Column":
        return Column(Cast(self._expr, T.to_type(dt)))

    astype = cast

    # -- arithmetic
    def _bin(self, op, other, reverse=False):
        a, b = _to_expr(self), _to_expr(other)
        return Column(BinOp(op, b, a) if reverse else BinOp(op, a, b))

    def __add__(self, o):
        return self._bin("+", o)

    def __radd__(self, o):
        return self._bin("+", o, True)

    def __sub__(self, o):
        return self._bin("-", o)

    def __rsub__(self, o):
        return self._bin("-", o, True)

    def __mul__(self, o):
        return self._bin("*", o)

    def __rmul__(self, o):
        return self._bin("*", o, True)

    def __truediv__(self, o):
        return self._bin("/", o)

    def __rtruediv__(self, o):
        return self._bin("/", o, True)

    __div__ = __truediv__

    def __mod__(self, o):
        return self._bin("%", o)

    def __rmod__(self, o):
        return self._bin("%", o, True)

    def __pow__(self, o):
        return self._bin("**", o)

    def __rpow__(self, o):
        return self._bin("**", o, True)

    def __neg__(self):
        return Column(Unary("-", self._expr))

    # -- comparison
    def __eq__(self, o):  # type: ignore[override]
        return self._bin("==", o)

    def __ne__(self, o):  # type: ignore[override]
        return self._bin("!=", o)

    def __lt__(self, o):
        return self._bin("<", o)

    def __le__(self, o):
        return self._bin("<=", o)

    def __gt__(self, o):
        return self._bin(">", o)

    def __ge__(self, o):
        return self._bin(">=", o)

    def eqNullSafe(self, o):
        return self._bin("<=>", o)

    # -- boolean
    def __and__(self, o):
        return self._bin("and", o)

    def __rand__(self, o):
        return self._bin("and", o, True)

    def __or__(self, o):
        return self._bin("or", o)

    def __ror__(self, o):
        return self._bin("or", o, True)

    def __invert__(self):
        return Column(Unary("not", self._expr))

    def __bool__(self):
        raise ValueError("Cannot convert column into bool: use '&' for 'and', '|' for 'or', '~' for 'not'")

    __hash__ = object.__hash__

    # -- predicates
    def isNull(self):
        return Column(IsNull(self._expr))

    def isNotNull(self):
        return Column(IsNull(self._expr, negate=True))

    def isin(self, *vals):
        if len(vals) == 1 and isinstance(vals[0], (list, tuple, set)):
            vals = tuple(vals[0])
        return Column(IsIn(self._expr, list(vals)))

    def between(self, lo, hi):
        return (self >= lo) & (self <= hi)

    def _str_pred(self, fname, fn):
        def ev(b, ctx, args):
            c = args[0]
            if not isinstance(c.dtype, T.StringType):
                c = _cast(c, T.StringType())
            d = c.dictionary if c.dictionary is not None else np.array([], dtype=object)
            lut = torch.tensor([bool(fn(s)) for s in d.tolist()] + [False], dtype=torch.bool, device=c.device)
            codes = c.values.long()
            codes = torch.where(codes < 0, torch.full_like(codes, len(d)), codes)
            return ColumnData(lut[codes], T.BooleanType(), c.valid)
        return Column(Func(fname, ev, [self._expr]))

    def contains(self, s):
        return self._str_pred("contains", lambda v: s in v)

    def startswith(self, s):
        return self._str_pred("startswith", lambda v: v.startswith(s))

    def endswith(self, s):
        return self._str_pred("endswith", lambda v: v.endswith(s))

    def like(self, pattern):
        import re
        rx = re.compile("^" + re.escape(pattern).replace("%", ".*").replace("_", ".") + "$", re.S)
        return self._str_pred("like", lambda v: rx.match(v) is not None)

    def rlike(self, pattern):
        import re
        rx = re.compile(pattern)
        return self._str_pred("rlike", lambda v: rx.search(v) is not None)

    def substr(self, start, length):
        from . import functions as F
        return F.substring(self, start, length)

    def getItem(self, key):
        def ev(b, ctx, args):
            c = args[0]
            if c.values.dim() == 2:
                return ColumnData(c.values[:, int(key)].double(), T.DoubleType(), c.valid)
            raise AnalysisException("getItem on non-array column")
        return Column(Func("getItem", ev, [self._expr], display=f"{self._expr.name()}[{key}]"))

    def __getitem__(self, k):
        return self.getItem(k)

    def __getattr__(self, item):
        if item.startswith("_"):
            raise AttributeError(item)
        raise AttributeError(f"Column has no attribute {item}")

    # -- ordering
    def asc(self):
        return Column(SortOrder(self._expr, True))

    def desc(self):
        return Column(SortOrder(self._expr, False))

    def asc_nulls_first(self):
        return Column(SortOrder(self._expr, True, True))

    def asc_nulls_last(self):
        return Column(SortOrder(self._expr, True, False))

    def desc_nulls_first(self):
        return Column(SortOrder(self._expr, False, True))

    def desc_nulls_last(self):
        return Column(SortOrder(self._expr, False, False))

    # -- conditional chaining
    def when(self, cond, value):
        e = self._expr
        if not isinstance(e, CaseWhen) or e.otherwise is not None:
            raise AnalysisException("when() can only be applied on a Column previously generated by when()")
        return Column(CaseWhen(e.branches + [(_to_expr(cond), _to_expr(value))]))

    def otherwise(self, value):
        e = self._expr
        if not isinstance(e, CaseWhen):
            raise AnalysisException("otherwise() can only be applied on a Column previously generated by when()")
        return Column(CaseWhen(e.branches, _to_expr(value)))

    def over(self, window):
        from .window import WindowExpr
        return Column(WindowExpr(self._expr, window))

    def __repr__(self):
        return f"Column<'{self._expr}'>"

    def __str__(self):
        return str(self._expr)

    def __iter__(self):
        raise TypeError("Column is not iterable")
