"""K18 fused elementwise expressions.

``evaluate(expr, batch, ctx)`` is what the projection / filter / withColumn paths call.  On a GPU batch it
compiles numeric expression trees -- arithmetic, comparisons, three-valued and/or/not, casts, when /
otherwise, isnull / isnan, log / exp / sqrt / abs / floor / ceil / round / signum / trig -- into a postfix
program that ``expr.hip`` runs in ONE kernel (inputs read once, intermediates in an LDS operand stack,
result and validity written once) instead of one torch kernel per operator.  Anything it cannot express
with the torch path's exact numerics (string columns, float32 or integer-typed arithmetic, vectors, UDFs,
row functions) falls back to ``expr.eval``.  Programs are cached per (expression, input schema).

Typing mirrors ``column.py``: arithmetic fuses only when its result type is double (so computing in fp64 is
the torch path's own arithmetic), comparisons of any numeric types (exact fp64 compares), casts to
double / float / int / long / boolean, and the null rules of each torch operator.
"""
from __future__ import annotations

import ctypes
import math
import os
import weakref
from typing import Dict, List, Optional, Tuple

import numpy as np
import torch

from . import types as T
from .column import (Alias, BinOp, Cast, CaseWhen, ColRef, ColumnData, Expr, Func, IsNaN, IsNull, Lit, Unary)

FUSE = os.environ.get("CDNAML_FUSE", "1") != "0"
FUSE_MIN_ROWS = int(os.environ.get("CDNAML_FUSE_MIN_ROWS", "4096"))

# opcodes: keep in sync with csrc/kernels/expr.hip
OP = dict(LOAD=1, CONST=2, NULL=3, ADD=10, SUB=11, MUL=12, DIV=13, MOD=14, POW=15, EQ=20, NE=21, LT=22, LE=23,
          GT=24, GE=25, EQNS=26, AND=30, OR=31, NOT=39, BAND=33, BOR=34, BXOR=35, NEG=40, ABS=41, LN=42, LOG10=43,
          LOG2=44, LOG1P=45, EXP=46, EXPM1=47, SQRT=48, FLOOR=49, CEIL=50, SIGNUM=51, SIN=52, COS=53, TAN=54,
          ROUND=55, TO_I32=60, TO_I64=61, TO_BOOL=62, TO_F32=63, ISNULL=70, ISNOTNULL=71, ISNAN=72, CASE=80)
_BIN = {"+": "ADD", "-": "SUB", "*": "MUL", "/": "DIV", "%": "MOD", "**": "POW", "==": "EQ", "!=": "NE",
        "<": "LT", "<=": "LE", ">": "GT", ">=": "GE", "<=>": "EQNS", "and": "AND", "or": "OR"}
_MATH = {"ln": "LN", "log10": "LOG10", "log2": "LOG2", "log1p": "LOG1P", "exp": "EXP", "expm1": "EXPM1",
         "sqrt": "SQRT", "signum": "SIGNUM", "sin": "SIN", "cos": "COS", "tan": "TAN"}
_MAX_STACK = 16
_DT_CODE = {torch.float64: 0, torch.float32: 1, torch.int32: 2, torch.int64: 3, torch.bool: 4}
_OUT_T = {T.DoubleType: torch.float64, T.FloatType: torch.float32, T.IntegerType: torch.int32,
          T.LongType: torch.int64, T.BooleanType: torch.bool}


class _LongIn(T.LongType):
    """Static type of a 64-bit integer INPUT (a LongType column, or a long literal of magnitude >= 2^53).

    The kernel's operand stack is fp64, so such a value is exact only below 2^53 (monotonically_increasing_id
    on rank >= 1 is far above it).  Flowing into double arithmetic / math functions / a cast to double is what
    Spark itself does (long -> double promotion), so that fuses; anything that must keep the value as a long --
    the result, a CASE value, a cast to int/long, abs/round, an ordering or equality test against another long
    -- stays on the int64 operator path."""


_NUM_IN = (T.DoubleType, T.FloatType, T.IntegerType, T.LongType, T.BooleanType, _LongIn)


class _Unfusable(Exception):
    pass


class _Prog:
    __slots__ = ("code", "consts", "inputs", "depth", "maxdepth", "nullable")

    def __init__(self):
        self.code: List[int] = []
        self.consts: List[float] = []
        self.inputs: List[str] = []
        self.depth = 0
        self.maxdepth = 0
        self.nullable = False

    def emit(self, op: str, arg: int = 0, pops: int = 0, pushes: int = 1):
        self.code.append(OP[op] | (arg << 8))
        self.depth += pushes - pops
        self.maxdepth = max(self.maxdepth, self.depth)
        if self.maxdepth > _MAX_STACK or len(self.code) > 256:
            raise _Unfusable("program too large")


def _is(t, *classes) -> bool:
    return any(type(t) is c for c in classes)


def _compile(e: Expr, b, p: _Prog) -> T.DataType:
    """Emit e's postfix code; returns its static type (raises _Unfusable)."""
    if isinstance(e, Alias):
        return _compile(e.x, b, p)
    if isinstance(e, ColRef):
        c = e.eval(b, None)
        if not _is(c.dtype, *_NUM_IN) or c.values.dim() != 1 or c.values.dtype not in _DT_CODE:
            raise _Unfusable("column type")
        name = e.col_name
        if name not in p.inputs:
            p.inputs.append(name)
        p.nullable |= c.valid is not None
        p.emit("LOAD", p.inputs.index(name))
        return _LongIn() if _is(c.dtype, T.LongType) else c.dtype
    if isinstance(e, Lit):
        v = e.value
        if v is None:
            p.nullable = True
            p.emit("NULL")
            return T.NullType()
        if isinstance(v, bool) or isinstance(v, (int, float)) and not isinstance(v, bool):
            if not _is(e.dtype, *_NUM_IN):
                raise _Unfusable("literal type")
            p.consts.append(float(v))
            p.emit("CONST", len(p.consts) - 1)
            if isinstance(v, int) and not isinstance(v, bool) and abs(v) >= 2 ** 53:
                return _LongIn()
            return e.dtype
        raise _Unfusable("literal")
    if isinstance(e, BinOp):
        op = e.op
        if (isinstance(e.r, Lit) and isinstance(e.r.value, str)) or (isinstance(e.l, Lit) and isinstance(e.l.value,
                                                                                                           str)):
            raise _Unfusable("string literal")
        lt = _compile(e.l, b, p)
        rt = _compile(e.r, b, p)
        for t in (lt, rt):
            if not (_is(t, *_NUM_IN) or isinstance(t, T.NullType)):
                raise _Unfusable("operand type")
        if op in ("and", "or"):
            p.emit(_BIN[op], pops=2)
            return T.BooleanType()
        if op in ("==", "!=", "<", "<=", ">", ">=", "<=>"):
            if isinstance(lt, _LongIn) and _is(rt, T.LongType, _LongIn) or \
                    isinstance(rt, _LongIn) and _is(lt, T.LongType, _LongIn):
                raise _Unfusable("long comparison")   # two 64-bit values: fp64 rounding can merge them
            p.emit(_BIN[op], pops=2)
            return T.BooleanType()
        if op in ("&", "|", "^"):
            if _is(lt, T.BooleanType) and _is(rt, T.BooleanType):
                p.emit({"&": "BAND", "|": "BOR", "^": "BXOR"}[op], pops=2)
                return T.BooleanType()
            raise _Unfusable("integer bit ops")
        if op == "/":
            p.nullable = True
            p.emit("DIV", pops=2)
            return T.DoubleType()
        if op == "**":
            p.emit("POW", pops=2)
            return T.DoubleType()
        if op in ("+", "-", "*", "%"):
            l2 = rt if isinstance(lt, T.NullType) else lt
            r2 = lt if isinstance(rt, T.NullType) else rt
            res = T.numeric_result(l2, r2) if (isinstance(l2, T.NumericType) and isinstance(r2, T.NumericType)) \
                else T.DoubleType()
            if not _is(res, T.DoubleType):
                raise _Unfusable("non-double arithmetic")  # fp32 / integer ops round differently than fp64
            if op == "%":
                p.nullable = True
            p.emit(_BIN[op], pops=2)
            return res
        raise _Unfusable(op)
    if isinstance(e, Unary):
        t = _compile(e.x, b, p)
        if e.op == "not":
            p.emit("NOT", pops=1)
            return T.BooleanType()
        if e.op == "-":
            if not _is(t, T.DoubleType, T.FloatType, T.IntegerType):
                raise _Unfusable("neg type")
            p.emit("NEG", pops=1)
            return t
        raise _Unfusable(e.op)
    if isinstance(e, Cast):
        t = _compile(e.x, b, p)
        dt = e.dt
        if not (_is(t, *_NUM_IN) or isinstance(t, T.NullType)):
            raise _Unfusable("cast source")
        if isinstance(t, _LongIn) and not _is(dt, T.DoubleType, T.FloatType, T.BooleanType):
            raise _Unfusable("long cast")
        if _is(dt, T.DoubleType):
            return dt
        if _is(dt, T.FloatType):
            if not _is(t, T.FloatType):
                p.emit("TO_F32", pops=1)
            return dt
        if _is(dt, T.BooleanType):
            p.emit("TO_BOOL", pops=1)
            return dt
        if _is(dt, T.IntegerType, T.LongType):
            if _is(t, T.DoubleType, T.FloatType):
                p.nullable = True
                p.emit("TO_I32" if _is(dt, T.IntegerType) else "TO_I64", pops=1)
            return dt
        raise _Unfusable("cast target")
    if isinstance(e, IsNull):
        _compile(e.x, b, p)
        p.emit("ISNOTNULL" if e.negate else "ISNULL", pops=1)
        return T.BooleanType()
    if isinstance(e, IsNaN):
        t = _compile(e.x, b, p)
        if _is(t, T.DoubleType, T.FloatType):
            p.emit("ISNAN", pops=1)
        else:
            p.emit("NOT", pops=1)   # non-float: never NaN (0 where valid); NOT of x then AND 0 below
            p.consts.append(0.0)
            p.emit("CONST", len(p.consts) - 1)
            p.emit("BAND", pops=2)
        return T.BooleanType()
    if isinstance(e, CaseWhen):
        # first-match semantics: acc = otherwise, then branches folded in REVERSE so the first wins last
        vts = []
        if e.otherwise is not None:
            vts.append(_compile(e.otherwise, b, p))
        else:
            p.nullable = True
            p.emit("NULL")
        for cond, val in reversed(e.branches):
            ct = _compile(cond, b, p)
            if not (_is(ct, *_NUM_IN) or isinstance(ct, T.NullType)):
                raise _Unfusable("case condition")
            vts.append(_compile(val, b, p))
            p.emit("CASE", pops=3)
        dts = [t for t in vts if not isinstance(t, T.NullType)]
        if any(isinstance(t, _LongIn) for t in dts):
            raise _Unfusable("long case value")
        if not dts or any(not _is(t, *_NUM_IN) for t in dts):
            raise _Unfusable("case value type")
        dt = dts[0]
        for t in dts:
            if isinstance(t, T.NumericType) and isinstance(dt, T.NumericType):
                dt = T.numeric_result(dt, t)
        if any(_is(t, T.BooleanType) for t in dts) and not all(_is(t, T.BooleanType) for t in dts):
            raise _Unfusable("mixed bool case")
        if _is(dt, T.FloatType) and not all(_is(t, T.FloatType) for t in dts):
            raise _Unfusable("float case promotion")
        return dt
    if isinstance(e, Func):
        tag = getattr(e, "fuse", None)
        if tag is None or len(e.args) != 1:
            raise _Unfusable("function")
        t = _compile(e.args[0], b, p)
        if not _is(t, *_NUM_IN):
            raise _Unfusable("function arg")
        name, extra = tag if isinstance(tag, tuple) else (tag, None)
        if isinstance(t, _LongIn) and name in ("abs", "round"):
            raise _Unfusable("long abs/round")
        if name in _MATH:
            if name in ("ln", "log10", "log2", "log1p", "sqrt"):
                p.nullable = True
            p.emit(_MATH[name], pops=1)
            return T.DoubleType()
        if name == "abs":
            if _is(t, T.BooleanType):
                raise _Unfusable("abs bool")
            p.emit("ABS", pops=1)
            return t
        if name in ("floor", "ceil"):
            p.emit("FLOOR" if name == "floor" else "CEIL", pops=1)
            return T.LongType()
        if name == "round":
            if _is(t, T.IntegerType, T.LongType) and extra >= 0:
                return t
            if not _is(t, T.DoubleType) or not (-100 < extra < 100):
                raise _Unfusable("round type")
            p.emit("ROUND", extra + 128, pops=1)
            return T.DoubleType()
        raise _Unfusable(name)
    raise _Unfusable(type(e).__name__)


def _op_count(p: _Prog) -> int:
    return sum(1 for ins in p.code if (ins & 0xFF) not in (OP["LOAD"], OP["CONST"], OP["NULL"]))


# expression object -> {input-schema signature: (program, type) or None}; weak keys: plans own their Exprs
_CACHE: "weakref.WeakKeyDictionary[Expr, Dict[Tuple, Optional[Tuple]]]" = weakref.WeakKeyDictionary()


def _program(e: Expr, b):
    key_cols = tuple(sorted(set(e.references())))
    sig = []
    for nme in key_cols:
        c = b.columns.get(nme)
        sig.append((nme, None if c is None else (type(c.dtype).__name__, str(c.values.dtype), c.valid is not None,
                                                  c.values.dim())))
    key = tuple(sig)
    per = _CACHE.setdefault(e, {})
    if key in per:
        return per[key]
    try:
        p = _Prog()
        rt = _compile(e, b, p)
        if _op_count(p) < 2 or not _is(rt, *_NUM_IN) or isinstance(rt, _LongIn):
            res = None                     # a single torch op is already one kernel
        else:
            res = (p, rt)
    except (_Unfusable, KeyError, AttributeError):
        res = None
    except Exception as err:  # noqa: BLE001 -- e.g. unresolved columns: let eval raise the real error
        if type(err).__name__ == "AnalysisException":
            res = None
        else:
            raise
    per[key] = res
    return res


def _run(p: _Prog, rt: T.DataType, b) -> ColumnData:
    from ..ops import _lib
    from ..ops.kernels import _ptr, _stream, upload
    dev = b.device
    n = b.n
    cols = [b.columns[nm] if nm in b.columns else _resolve(b, nm) for nm in p.inputs]
    ins = [c.values.contiguous() for c in cols]
    vals = [None if c.valid is None else c.valid.contiguous() for c in cols]
    out_t = _OUT_T[type(rt)]
    out = torch.empty(n, dtype=out_t, device=dev)
    outv = torch.empty(n, dtype=torch.bool, device=dev) if p.nullable else None
    prog_t, cons_t = upload(dev, np.asarray(p.code, dtype=np.int32),
                            np.asarray(p.consts if p.consts else [0.0], dtype=np.float64))
    k = len(ins)
    in_arr = (ctypes.c_void_p * max(k, 1))(*[x.data_ptr() for x in ins])
    inv_arr = (ctypes.c_void_p * max(k, 1))(*[(v.data_ptr() if v is not None else None) for v in vals])
    dt_arr = (ctypes.c_int * max(k, 1))(*[_DT_CODE[x.dtype] for x in ins])
    _lib.check(_lib.lib().cdna_expr_eval(_ptr(prog_t), len(p.code), _ptr(cons_t), k, in_arr, inv_arr, dt_arr, n,
                                         _ptr(out), _DT_CODE[out_t], _ptr(outv) if outv is not None else None,
                                         _stream(dev)), "cdna_expr_eval")
    return ColumnData(out, rt, outv)


def _resolve(b, name):
    return ColRef(name).eval(b, None)


def evaluate(e: Expr, b, ctx) -> ColumnData:
    """Evaluate ``e`` on batch ``b``: one fused HIP kernel when possible, else the operator-at-a-time path."""
    if FUSE and b.n >= FUSE_MIN_ROWS and b.device.type == "cuda":
        prog = _program(e, b)
        if prog is not None:
            from ..ops import _lib
            if _lib.available():
                return _run(prog[0], prog[1], b)
    return e.eval(b, ctx)


def can_fuse(e: Expr, b) -> bool:
    """Whether ``evaluate`` would run ``e`` as one fused kernel on a GPU batch shaped like ``b``."""
    return _program(e, b) is not None


__all__ = ["evaluate", "can_fuse", "FUSE", "FUSE_MIN_ROWS", "math"]


def interpret(p: _Prog, rt: T.DataType, b) -> ColumnData:
    """Host reference of expr.hip's program semantics (numpy, fp64): the CPU tests run every compiled program
    through it and compare with the operator path, so compiler bugs surface without a GPU."""
    n = b.n
    cols = [b.columns[nm] if nm in b.columns else _resolve(b, nm) for nm in p.inputs]
    ins = [c.values.detach().cpu().numpy().astype(np.float64) for c in cols]
    vin = [np.ones(n, bool) if c.valid is None else c.valid.cpu().numpy().astype(bool) for c in cols]
    inv = {v: k for k, v in OP.items()}
    sv, sm = [], []
    with np.errstate(all="ignore"):
        for ins_ in p.code:
            op, arg = inv[ins_ & 0xFF], ins_ >> 8
            if op == "LOAD":
                sv.append(ins[arg].copy()); sm.append(vin[arg].copy()); continue
            if op in ("CONST", "NULL"):
                sv.append(np.full(n, p.consts[arg] if op == "CONST" else 0.0)); sm.append(np.full(n, op == "CONST"))
                continue
            if op == "CASE":
                bv, mb = sv.pop(), sm.pop()
                c, mc = sv.pop(), sm.pop()
                take = mc & (c != 0)
                sv[-1] = np.where(take, bv, sv[-1]); sm[-1] = np.where(take, mb, sm[-1]); continue
            if OP[op] >= OP["ADD"] and OP[op] <= OP["BXOR"]:
                y, my = sv.pop(), sm.pop()
                x, mx = sv[-1], sm[-1]
                m = mx & my
                bx, by = x != 0, y != 0
                if op == "DIV":
                    v = x / np.where(y == 0, 1.0, y); m = m & (y != 0)
                elif op == "MOD":
                    v = np.fmod(x, np.where(y == 0, 1.0, y)); m = m & (y != 0)
                elif op == "AND":
                    m = (mx & my) | (mx & ~bx) | (my & ~by); v = (bx & by & m).astype(float)
                elif op == "OR":
                    m = (mx & my) | (mx & bx) | (my & by); v = ((bx | by) & m).astype(float)
                elif op == "EQNS":
                    v = ((mx & my & (x == y)) | (~mx & ~my)).astype(float); m = np.ones(n, bool)
                else:
                    f = {"ADD": np.add, "SUB": np.subtract, "MUL": np.multiply, "POW": np.power,
                         "EQ": np.equal, "NE": np.not_equal, "LT": np.less, "LE": np.less_equal,
                         "GT": np.greater, "GE": np.greater_equal}.get(op)
                    if f is not None:
                        v = f(x, y).astype(float)
                    else:
                        v = {"BAND": bx & by, "BOR": bx | by, "BXOR": bx != by}[op].astype(float)
                sv[-1], sm[-1] = v, m
                continue
            x, m = sv[-1], sm[-1]
            if op == "NOT":
                v = (x == 0).astype(float)
            elif op in ("LN", "LOG10", "LOG2", "LOG1P"):
                v = {"LN": np.log, "LOG10": np.log10, "LOG2": np.log2, "LOG1P": np.log1p}[op](x)
                m = m & ((x > -1) if op == "LOG1P" else (x > 0))
            elif op == "SQRT":
                v = np.sqrt(x); m = m & ~(x < 0)
            elif op == "ROUND":
                pw = 10.0 ** (arg - 128)
                v = np.where(x > 0, 1.0, np.where(x < 0, -1.0, x)) * np.floor(np.abs(x) * pw + 0.5) / pw
            elif op in ("TO_I32", "TO_I64"):
                bad = ~np.isfinite(x); v = np.where(bad, 0.0, np.trunc(x)); m = m & ~bad
            elif op == "ISNULL":
                v = (~m).astype(float); m = np.ones(n, bool)
            elif op == "ISNOTNULL":
                v = m.astype(float); m = np.ones(n, bool)
            else:
                v = {"NEG": np.negative, "ABS": np.abs, "EXP": np.exp, "EXPM1": np.expm1, "FLOOR": np.floor,
                     "CEIL": np.ceil, "SIGNUM": np.sign, "SIN": np.sin, "COS": np.cos, "TAN": np.tan,
                     "TO_BOOL": lambda a: (a != 0).astype(float), "TO_F32": lambda a: a.astype(np.float32),
                     "ISNAN": lambda a: np.isnan(a).astype(float)}[op](x).astype(float)
            sv[-1], sm[-1] = v, m
    out_t = _OUT_T[type(rt)]
    vals = torch.from_numpy(sv[0]).to(out_t) if out_t != torch.bool else torch.from_numpy(sv[0] != 0)
    return ColumnData(vals, rt, torch.from_numpy(sm[0]) if p.nullable else None)
