"""Minimal SQL front-end → DataFrame plans.

Covers what the course issues: ``SELECT … FROM … [JOIN … ON …] WHERE …
GROUP BY … HAVING … ORDER BY … LIMIT`` (MLE 01 - Collaborative Filtering
Lab.py:241-252,349-374), temp-view queries (ML 00b:59-64), ``CREATE
DATABASE IF NOT EXISTS`` / ``USE`` / ``DROP DATABASE … CASCADE``
(Includes/Class-Utility-Methods.py:134-150), ``CREATE TABLE … USING DELTA
LOCATION`` (ML 00c:178-179), ``DESCRIBE HISTORY`` (ML 00c:183; Labs/ML
05L:85), ``SELECT current_user()``, plus ``expr()`` / ``selectExpr``.
"""
from __future__ import annotations

import getpass
import re
from typing import List, Optional, Tuple

from . import functions as F
from . import types as T
from .column import (AnalysisException, BinOp, CaseWhen, Cast, ColRef, Column, Expr, IsIn, IsNull, Lit, SortOrder,
                     Star, Unary)

_TOKEN = re.compile(r"""
    (?P<ws>\s+)|
    (?P<comment>--[^\n]*)|
    (?P<num>\d+\.\d*(?:[eE][-+]?\d+)?|\.\d+(?:[eE][-+]?\d+)?|\d+(?:[eE][-+]?\d+)?[LDF]?)|
    (?P<str>'(?:[^'\\]|\\.|'')*'|"(?:[^"\\]|\\.)*")|
    (?P<bq>`[^`]*`)|
    (?P<id>[A-Za-z_][A-Za-z0-9_$]*)|
    (?P<op><=>|<=|>=|<>|!=|==|\|\||[-+*/%=<>(),.;!&|^~\[\]])
""", re.X)

_KEYWORDS = {"select", "from", "where", "group", "by", "having", "order", "limit", "join", "inner", "left", "right",
             "full", "outer", "cross", "on", "as", "and", "or", "not", "is", "null", "in", "between", "like", "rlike",
             "case", "when", "then", "else", "end", "cast", "asc", "desc", "distinct", "true", "false", "union",
             "all", "semi", "anti", "using", "nulls", "first", "last"}


class Tok:
    def __init__(self, kind, val):
        self.kind, self.val = kind, val

    def __repr__(self):
        return f"{self.kind}:{self.val}"


def tokenize(s: str) -> List[Tok]:
    out, pos = [], 0
    while pos < len(s):
        m = _TOKEN.match(s, pos)
        if not m:
            raise AnalysisException(f"SQL syntax error near: {s[pos:pos + 20]!r}")
        pos = m.end()
        k = m.lastgroup
        v = m.group(k)
        if k in ("ws", "comment"):
            continue
        if k == "str":
            q = v[0]
            v = v[1:-1].replace(q + q, q).replace("\\" + q, q)
        if k == "bq":
            k, v = "id", v[1:-1]
            out.append(Tok("qid", v))
            continue
        out.append(Tok(k, v))
    out.append(Tok("eof", None))
    return out


class Parser:
    def __init__(self, s: str, session=None):
        self.toks = tokenize(s)
        self.i = 0
        self.session = session

    # ------------------------------------------------------------ helpers
    def peek(self, k=0) -> Tok:
        return self.toks[min(self.i + k, len(self.toks) - 1)]

    def next(self) -> Tok:
        t = self.toks[self.i]
        self.i += 1
        return t

    def is_kw(self, *kws, k=0) -> bool:
        t = self.peek(k)
        return t.kind == "id" and t.val.lower() in kws

    def accept_kw(self, *kws) -> bool:
        if self.is_kw(*kws):
            self.i += 1
            return True
        return False

    def expect_kw(self, kw):
        if not self.accept_kw(kw):
            raise AnalysisException(f"expected {kw.upper()} but found {self.peek().val!r}")

    def accept_op(self, op) -> bool:
        t = self.peek()
        if t.kind == "op" and t.val == op:
            self.i += 1
            return True
        return False

    def expect_op(self, op):
        if not self.accept_op(op):
            raise AnalysisException(f"expected '{op}' but found {self.peek().val!r}")

    def ident(self) -> str:
        t = self.next()
        if t.kind not in ("id", "qid"):
            raise AnalysisException(f"expected identifier, found {t.val!r}")
        return t.val

    # --------------------------------------------------------- expressions
    def expression(self) -> Expr:
        return self.or_expr()

    def or_expr(self):
        e = self.and_expr()
        while self.accept_kw("or"):
            e = BinOp("or", e, self.and_expr())
        return e

    def and_expr(self):
        e = self.not_expr()
        while self.accept_kw("and"):
            e = BinOp("and", e, self.not_expr())
        return e

    def not_expr(self):
        if self.accept_kw("not"):
            return Unary("not", self.not_expr())
        return self.predicate()

    def predicate(self):
        e = self.additive()
        while True:
            t = self.peek()
            if t.kind == "op" and t.val in ("=", "==", "!=", "<>", "<", "<=", ">", ">=", "<=>"):
                self.next()
                op = {"=": "==", "<>": "!="}.get(t.val, t.val)
                e = BinOp(op, e, self.additive())
                continue
            neg = False
            if self.is_kw("not") and self.is_kw("in", "between", "like", "rlike", k=1):
                self.next()
                neg = True
            if self.accept_kw("is"):
                n = self.accept_kw("not")
                self.expect_kw("null")
                e = IsNull(e, negate=n)
                continue
            if self.accept_kw("in"):
                self.expect_op("(")
                vals = [self._literal_value(self.expression())]
                while self.accept_op(","):
                    vals.append(self._literal_value(self.expression()))
                self.expect_op(")")
                e = IsIn(e, vals)
            elif self.accept_kw("between"):
                lo = self.additive()
                self.expect_kw("and")
                hi = self.additive()
                e = BinOp("and", BinOp(">=", e, lo), BinOp("<=", e, hi))
            elif self.accept_kw("like"):
                pat = self._literal_value(self.additive())
                e = Column(e).like(pat)._expr
            elif self.accept_kw("rlike"):
                pat = self._literal_value(self.additive())
                e = Column(e).rlike(pat)._expr
            else:
                return e
            if neg:
                e = Unary("not", e)

    @staticmethod
    def _literal_value(e):
        if isinstance(e, Lit):
            return e.value
        if isinstance(e, Unary) and e.op == "-" and isinstance(e.x, Lit):
            return -e.x.value
        raise AnalysisException("expected a literal")

    def additive(self):
        e = self.multiplicative()
        while True:
            t = self.peek()
            if t.kind == "op" and t.val in ("+", "-"):
                self.next()
                e = BinOp(t.val, e, self.multiplicative())
            elif t.kind == "op" and t.val == "||":
                self.next()
                e = F.concat(Column(e), Column(self.multiplicative()))._expr
            else:
                return e

    def multiplicative(self):
        e = self.unary()
        while True:
            t = self.peek()
            if t.kind == "op" and t.val in ("*", "/", "%"):
                self.next()
                e = BinOp(t.val, e, self.unary())
            else:
                return e

    def unary(self):
        if self.accept_op("-"):
            x = self.unary()
            if isinstance(x, Lit) and isinstance(x.value, (int, float)):
                return Lit(-x.value)
            return Unary("-", x)
        if self.accept_op("+"):
            return self.unary()
        if self.accept_op("!"):
            return Unary("not", self.unary())
        return self.primary()

    def primary(self) -> Expr:
        t = self.peek()
        if t.kind == "num":
            self.next()
            v = t.val
            if v[-1] in "LDF":
                v = v[:-1]
            if re.fullmatch(r"\d+", v):
                return Lit(int(v))
            return Lit(float(v))
        if t.kind == "str":
            self.next()
            return Lit(t.val)
        if t.kind == "op" and t.val == "(":
            self.next()
            e = self.expression()
            self.expect_op(")")
            return e
        if t.kind == "op" and t.val == "*":
            self.next()
            return Star()
        if t.kind == "qid":
            self.next()
            return self._qualified(t.val)
        if t.kind != "id":
            raise AnalysisException(f"unexpected token {t.val!r}")
        low = t.val.lower()
        if low in ("true", "false"):
            self.next()
            return Lit(low == "true")
        if low == "null":
            self.next()
            return Lit(None)
        if low == "case":
            self.next()
            return self.case_expr()
        if low == "cast" and self.peek(1).kind == "op" and self.peek(1).val == "(":
            self.next()
            self.expect_op("(")
            x = self.expression()
            self.expect_kw("as")
            typ = self.type_name()
            self.expect_op(")")
            return Cast(x, T._parse_type(typ))
        if low in ("date", "timestamp") and self.peek(1).kind == "str":
            self.next()
            s = self.next().val
            import datetime as _dt
            return Lit(_dt.date.fromisoformat(s) if low == "date" else _dt.datetime.fromisoformat(s))
        self.next()
        if self.peek().kind == "op" and self.peek().val == "(":
            return self.func_call(t.val)
        return self._qualified(t.val)

    def _qualified(self, name):
        while self.peek().kind == "op" and self.peek().val == ".":
            self.next()
            if self.accept_op("*"):
                return Star(name)
            name = name + "." + self.ident()
        return ColRef(name)

    def type_name(self) -> str:
        parts = [self.ident()]
        if self.accept_op("<"):
            inner = self.type_name()
            self.expect_op(">")
            return f"{parts[0]}<{inner}>"
        if self.accept_op("("):
            while not self.accept_op(")"):
                self.next()
        return parts[0]

    def case_expr(self):
        base = None
        if not self.is_kw("when"):
            base = self.expression()
        branches = []
        while self.accept_kw("when"):
            c = self.expression()
            if base is not None:
                c = BinOp("==", base, c)
            self.expect_kw("then")
            branches.append((c, self.expression()))
        other = self.expression() if self.accept_kw("else") else None
        self.expect_kw("end")
        return CaseWhen(branches, other)

    def func_call(self, name) -> Expr:
        self.expect_op("(")
        low = name.lower()
        distinct = self.accept_kw("distinct")
        args: List[Expr] = []
        if not self.accept_op(")"):
            args.append(self.expression())
            while self.accept_op(","):
                args.append(self.expression())
            self.expect_op(")")
        return build_function(low, args, distinct, self.session)

    # ------------------------------------------------------------ statements
    def select_item(self) -> Expr:
        e = self.expression()
        if self.accept_kw("as"):
            return F.Column(e).alias(self.ident())._expr
        t = self.peek()
        if t.kind in ("id", "qid") and t.val.lower() not in _KEYWORDS:
            self.next()
            return F.Column(e).alias(t.val)._expr
        return e


def build_function(low: str, args: List[Expr], distinct: bool, session=None) -> Expr:
    C = [Column(a) for a in args]
    aggs = {"count": F.count, "sum": F.sum, "avg": F.avg, "mean": F.avg, "min": F.min, "max": F.max,
            "stddev": F.stddev, "stddev_samp": F.stddev_samp, "stddev_pop": F.stddev_pop, "variance": F.variance,
            "var_samp": F.var_samp, "var_pop": F.var_pop, "first": F.first, "last": F.last,
            "collect_list": F.collect_list, "collect_set": F.collect_set}
    if low in aggs:
        if low == "count" and args and isinstance(args[0], Star):
            return F.count("*")._expr
        if low == "count" and args and isinstance(args[0], Lit):
            return F.count("*")._expr
        e = aggs[low](C[0])._expr
        if distinct:
            e.distinct = True
        return e
    if low in ("percentile_approx", "percentile", "approx_percentile"):
        return F.percentile_approx(C[0], Parser._literal_value(args[1]))._expr
    if low == "median":
        return F.median(C[0])._expr
    if low == "current_user":
        return Lit(_current_user())
    if low in ("current_database", "current_schema"):
        return Lit(session.catalog.currentDatabase() if session else "default")
    simple = {"lower": F.lower, "upper": F.upper, "lcase": F.lower, "ucase": F.upper, "trim": F.trim,
              "ltrim": F.ltrim, "rtrim": F.rtrim, "length": F.length, "exp": F.exp, "sqrt": F.sqrt, "abs": F.abs,
              "floor": F.floor, "ceil": F.ceil, "ceiling": F.ceil, "log10": F.log10, "log2": F.log2,
              "log1p": F.log1p, "year": F.year, "month": F.month, "day": F.dayofmonth, "dayofmonth": F.dayofmonth,
              "to_date": F.to_date, "isnan": F.isnan, "isnull": F.isnull, "initcap": F.initcap,
              "reverse": F.reverse, "signum": F.signum, "sin": F.sin, "cos": F.cos}
    if low in simple:
        return simple[low](*C)._expr
    if low in ("ln",):
        return F.log(C[0])._expr
    if low == "log":
        return (F.log(C[0]) if len(C) == 1 else F.log(Parser._literal_value(args[0]), C[1]))._expr
    if low in ("pow", "power"):
        return F.pow(C[0], C[1])._expr
    if low == "round":
        return F.round(C[0], Parser._literal_value(args[1]) if len(args) > 1 else 0)._expr
    if low in ("coalesce", "ifnull", "nvl"):
        return F.coalesce(*C)._expr
    if low in ("concat",):
        return F.concat(*C)._expr
    if low in ("substring", "substr"):
        return F.substring(C[0], Parser._literal_value(args[1]), Parser._literal_value(args[2]))._expr
    if low == "translate":
        return F.translate(C[0], Parser._literal_value(args[1]), Parser._literal_value(args[2]))._expr
    if low == "regexp_replace":
        return F.regexp_replace(C[0], Parser._literal_value(args[1]), Parser._literal_value(args[2]))._expr
    if low == "rand":
        return F.rand(Parser._literal_value(args[0]) if args else None)._expr
    if low == "randn":
        return F.randn(Parser._literal_value(args[0]) if args else None)._expr
    if low == "monotonically_increasing_id":
        return F.monotonically_increasing_id()._expr
    if low == "hash":
        return F.hash(*C)._expr
    if low in ("greatest", "least"):
        return getattr(F, low)(*C)._expr
    if low == "if":
        return CaseWhen([(args[0], args[1])], args[2])
    if low == "datediff":
        return F.datediff(C[0], C[1])._expr
    if low in ("double", "int", "float", "string", "bigint", "boolean"):
        return Cast(args[0], T._parse_type(low))
    if session is not None and low in session.catalog._functions:
        return session.catalog._functions[low](*C)._expr
    raise AnalysisException(f"Undefined function: '{low}'")


def _current_user() -> str:
    try:
        return getpass.getuser()
    except Exception:
        return "user"


def parse_expression(s: str) -> Column:
    p = Parser(s)
    e = p.select_item()
    if p.peek().kind != "eof":
        raise AnalysisException(f"unexpected trailing tokens in expression {s!r}")
    return Column(e)


# ===================================================================== SQL
def run_sql(session, query: str):
    q = query.strip().rstrip(";").strip()
    p = Parser(q, session)
    if p.is_kw("select") or (p.peek().kind == "op" and p.peek().val == "(") or p.is_kw("with"):
        df = _select(p, session)
        if p.peek().kind != "eof":
            raise AnalysisException(f"unexpected trailing input near {p.peek().val!r}")
        return df
    low = q.lower()
    words = low.split()
    if words[:2] == ["create", "database"] or words[:2] == ["create", "schema"]:
        m = re.match(r"create\s+(?:database|schema)\s+(if\s+not\s+exists\s+)?([`\w.]+)", q, re.I)
        session.catalog.createDatabase(m.group(2).strip("`"), ifNotExists=bool(m.group(1)))
        return _empty(session)
    if words[0] == "use":
        name = words[-1].strip("`")
        session.catalog.setCurrentDatabase(name)
        return _empty(session)
    if words[:2] in (["drop", "database"], ["drop", "schema"]):
        m = re.match(r"drop\s+(?:database|schema)\s+(if\s+exists\s+)?([`\w.]+)(\s+cascade)?", q, re.I)
        session.catalog.dropDatabase(m.group(2).strip("`"), ifExists=bool(m.group(1)), cascade=bool(m.group(3)))
        return _empty(session)
    if words[:2] == ["drop", "table"] or words[:2] == ["drop", "view"]:
        m = re.match(r"drop\s+(?:table|view)\s+(if\s+exists\s+)?([`\w.]+)", q, re.I)
        name = m.group(2).strip("`")
        if not session.catalog.dropTempView(name):
            session.catalog.dropTable(name, ifExists=bool(m.group(1)))
        return _empty(session)
    if words[:2] == ["create", "table"] or words[:4] == ["create", "or", "replace", "table"]:
        m = re.match(r"create\s+(?:or\s+replace\s+)?table\s+(if\s+not\s+exists\s+)?([`\w.]+)\s*(.*)$", q, re.I | re.S)
        name, rest = m.group(2).strip("`"), m.group(3)
        ml = re.search(r"location\s+['\"]([^'\"]+)['\"]", rest, re.I)
        mu = re.search(r"using\s+(\w+)", rest, re.I)
        fmt = (mu.group(1).lower() if mu else "delta")
        mas = re.search(r"\bas\s+(select.*)$", rest, re.I | re.S)
        if mas:
            df = run_sql(session, mas.group(1))
            w = df.write.format(fmt).mode("overwrite")
            if ml:
                w.save(ml.group(1))
                session.catalog._register_table(name, ml.group(1), fmt, managed=False)
            else:
                w.saveAsTable(name)
            return _empty(session)
        if ml:
            from .readwriter import _strip_dbfs
            session.catalog._register_table(name, _strip_dbfs(ml.group(1)), fmt, managed=False)
            return _empty(session)
        raise AnalysisException("CREATE TABLE needs LOCATION or AS SELECT")
    if words[:2] == ["describe", "history"]:
        target = q.split(None, 2)[2].strip()
        from ..storage.delta import DeltaTable
        path = _table_path(session, target)
        return DeltaTable(session, path).history()
    if words[0] in ("describe", "desc"):
        target = q.split(None, 1)[1].strip()
        if target.lower().startswith("table "):
            target = target[6:]
        df = session.table(target.strip("`"))
        import pandas as pd
        return session.createDataFrame(pd.DataFrame({"col_name": df.columns,
                                                     "data_type": [t for _, t in df.dtypes],
                                                     "comment": [None] * len(df.columns)}),
                                       "col_name string, data_type string, comment string")
    if words[:2] == ["show", "tables"]:
        import pandas as pd
        ts = session.catalog.listTables()
        return session.createDataFrame(pd.DataFrame({"database": [t.database or "" for t in ts],
                                                     "tableName": [t.name for t in ts],
                                                     "isTemporary": [t.isTemporary for t in ts]}))
    if words[:2] == ["show", "databases"]:
        import pandas as pd
        return session.createDataFrame(pd.DataFrame({"namespace": [d.name for d in
                                                                   session.catalog.listDatabases()]}))
    if words[0] == "cache" or words[0] == "uncache" or words[:2] == ["refresh", "table"]:
        return _empty(session)
    if words[0] == "set":
        kv = q[3:].strip()
        if "=" in kv:
            k, v = kv.split("=", 1)
            session.conf.set(k.strip(), v.strip())
        return _empty(session)
    if words[0] == "vacuum":
        m = re.match(r"vacuum\s+(\S+)(?:\s+retain\s+([\d.]+)\s+hours)?", q, re.I)
        from ..storage.delta import DeltaTable
        return DeltaTable(session, _table_path(session, m.group(1))).vacuum(float(m.group(2) or 168))
    raise AnalysisException(f"unsupported SQL statement: {q[:60]}")


def _empty(session):
    import pandas as pd
    return session.createDataFrame(pd.DataFrame())


def _table_path(session, target: str) -> str:
    m = re.match(r"delta\.`([^`]+)`", target.strip(), re.I)
    if m:
        from .readwriter import _strip_dbfs
        return _strip_dbfs(m.group(1))
    info = session.catalog._table_info(target.strip("`"))
    if info is None:
        raise AnalysisException(f"Table not found: {target}")
    return info["location"]


def _resolve(name: str, columns: List[str]) -> str:
    base = name.split(".")[-1] if "." in name else name
    for c in columns:
        if c == base:
            return c
    for c in columns:
        if c.lower() == base.lower():
            return c
    raise AnalysisException(f"cannot resolve column {name!r} among {columns}")


def _from_source(p: Parser, session):
    """Parse a table reference; returns (DataFrame, alias, table name or None)."""
    tname = None
    if p.accept_op("("):
        df = _select(p, session)
        p.expect_op(")")
    else:
        t = p.next()
        name = t.val
        if t.kind == "id" and name.lower() in ("delta", "parquet", "csv", "json") and p.peek().kind == "op" \
                and p.peek().val == ".":
            p.next()
            path = p.next().val
            from .readwriter import _strip_dbfs
            df = session.read.format(name.lower()).load(_strip_dbfs(path))
        else:
            while p.peek().kind == "op" and p.peek().val == ".":
                p.next()
                name += "." + p.ident()
            df = session.table(name)
            tname = name.split(".")[-1]
    alias = None
    if p.accept_kw("as"):
        alias = p.ident()
    elif p.peek().kind in ("id", "qid") and p.peek().val.lower() not in _KEYWORDS:
        alias = p.next().val
    return df, alias, tname


def _map_expr(e: Expr, fn) -> Expr:
    """Rebuild ``e`` bottom-up; ``fn(node)`` may return a replacement for a node (else None = recurse)."""
    import copy
    r = fn(e)
    if r is not None:
        return r
    e2 = copy.copy(e)
    kids = None
    for attr in ("l", "r", "x", "otherwise"):
        if isinstance(getattr(e2, attr, None), Expr):
            setattr(e2, attr, _map_expr(getattr(e2, attr), fn))
    if hasattr(e2, "args"):
        e2.args = [_map_expr(a, fn) for a in e2.args]
        kids = list(e2.args)
    elif hasattr(e2, "branches"):
        e2.branches = [(_map_expr(c, fn), _map_expr(v, fn)) for c, v in e2.branches]
        kids = [k for br in e2.branches for k in br] + ([e2.otherwise] if e2.otherwise is not None else [])
    else:
        kids = [getattr(e2, a) for a in ("l", "r", "x") if isinstance(getattr(e2, a, None), Expr)]
    e2.children = kids
    return e2


def _collect_aggs(e: Expr, out: list):
    from .functions import AggExpr
    if isinstance(e, AggExpr):
        if all(a is not e for a in out):
            out.append(e)
        return
    for c in e.children:
        if c is not None:
            _collect_aggs(c, out)


def _replace_aggs(e: Expr, mapping: dict) -> Expr:
    return _map_expr(e, lambda x: ColRef(mapping[id(x)]) if id(x) in mapping else None)


def _display(e: Expr) -> str:
    """Spark's output name of an un-aliased select item: column references lose their qualifier."""
    return _map_expr(e, lambda x: ColRef(x.col_name.split(".")[-1]) if isinstance(x, ColRef) else None).name()


class _Scope:
    """Name resolution over the FROM clause (Spark's analyzer, the part SQL queries over joins need).

    Every source's columns are renamed to unique internal names (``__s<i>_<col>``), so both sides of
    a join stay addressable: ``alias.col`` resolves to that source's column, a bare name must match
    exactly one source column (else ``AnalysisException: Reference 'x' is ambiguous``, as in Spark),
    and ``JOIN … USING (k)`` merges the key into one column visible under both qualifiers.
    """

    def __init__(self):
        self.entries: List[Tuple[Optional[str], str, str]] = []  # (qualifier lower, column, internal name)
        self.nsrc = 0

    def add(self, df, alias, tname):
        i = self.nsrc
        self.nsrc += 1
        qual = (alias or tname)
        qual = qual.lower() if qual else None
        internal = [f"__s{i}_{c}" for c in df.columns]
        for c, n in zip(df.columns, internal):
            self.entries.append((qual, c, n))
        return df.toDF(*internal), qual

    def columns(self, qual=None):
        seen, out = set(), []
        for q, c, n in self.entries:
            if (qual is None or q == qual) and n not in seen:
                seen.add(n)
                out.append((c, n))
        return out

    def lookup(self, name: str) -> Optional[str]:
        parts = name.split(".")
        if len(parts) >= 2:
            q, c = parts[-2].lower(), parts[-1].lower()
            hits = {n for qq, cc, n in self.entries if qq == q and cc.lower() == c}
            if len(hits) == 1:
                return hits.pop()
        c = name.lower()
        hits = {n for _, cc, n in self.entries if cc.lower() == c}
        if not hits and len(parts) >= 2:
            if parts[-2].lower() in {qq for qq, _, _ in self.entries if qq}:
                # a known source qualifier whose source has no such column: Spark cannot resolve it (no
                # fallback to another source's column of that name)
                return None
            c = parts[-1].lower()
            hits = {n for _, cc, n in self.entries if cc.lower() == c}
        if len(hits) > 1:
            raise AnalysisException(f"Reference '{name}' is ambiguous, could be: "
                                    f"{sorted(q + '.' + cc if q else cc for q, cc, n in self.entries if n in hits)}")
        return hits.pop() if hits else None

    def bind(self, e: Expr, extra: Optional[dict] = None) -> Expr:
        def fn(x):
            if isinstance(x, ColRef):
                if extra is not None and "." not in x.col_name and x.col_name.lower() in extra:
                    return extra[x.col_name.lower()]
                n = self.lookup(x.col_name)
                if n is None:
                    raise AnalysisException(f"cannot resolve column '{x.col_name}' given input columns "
                                            f"{[c for c, _ in self.columns()]}")
                return ColRef(n)
            return None
        return _map_expr(e, fn)


def _join_keys(cond: Expr, scope: _Scope, left_names: set, lk, rk):
    """Equi-join conditions (AND of col = col) bound to internal names, left side first."""
    if isinstance(cond, BinOp) and cond.op == "and":
        _join_keys(cond.l, scope, left_names, lk, rk)
        _join_keys(cond.r, scope, left_names, lk, rk)
        return
    if isinstance(cond, BinOp) and cond.op == "==" and isinstance(cond.l, ColRef) and isinstance(cond.r, ColRef):
        a, b = scope.bind(cond.l).col_name, scope.bind(cond.r).col_name
        if a in left_names and b not in left_names:
            lk.append(a)
            rk.append(b)
            return
        if b in left_names and a not in left_names:
            lk.append(b)
            rk.append(a)
            return
    raise AnalysisException("only equality join conditions between the two sides (combined with AND) are supported")


def _select(p: Parser, session):
    if p.accept_op("("):
        df = _select(p, session)
        p.expect_op(")")
        return df
    p.expect_kw("select")
    distinct = p.accept_kw("distinct")
    items = [p.select_item()]
    while p.accept_op(","):
        items.append(p.select_item())
    scope = _Scope()
    if p.accept_kw("from"):
        df, _ = scope.add(*_from_source(p, session))
        while True:
            how = None
            if p.is_kw("join"):
                how = "inner"
            elif p.is_kw("inner", "left", "right", "full", "cross"):
                how = p.next().val.lower()
                if how in ("left", "right", "full") and p.accept_kw("outer"):
                    pass
                if how == "left" and p.is_kw("semi", "anti"):
                    how = "left_" + p.next().val.lower()
            else:
                break
            p.expect_kw("join")
            left_names = set(df.columns)
            n_before = len(scope.entries)
            other, oq = scope.add(*_from_source(p, session))
            if how == "cross":
                df = df.crossJoin(other)
                continue
            if p.accept_kw("using"):
                p.expect_op("(")
                keys = [p.ident()]
                while p.accept_op(","):
                    keys.append(p.ident())
                p.expect_op(")")
                ren = {}
                for k in keys:
                    ln = [n for q, c, n in scope.entries[:n_before] if c.lower() == k.lower()]
                    rn = [n for q, c, n in scope.entries[n_before:] if c.lower() == k.lower()]
                    if len(set(ln)) != 1 or len(rn) != 1:
                        raise AnalysisException(f"USING column '{k}' cannot be resolved on both sides of the join")
                    ren[rn[0]] = ln[0]
                # the right key becomes the left key column: one merged column under both qualifiers
                other = other.toDF(*[ren.get(c, c) for c in other.columns])
                scope.entries[n_before:] = [(q, c, ren.get(n, n)) for q, c, n in scope.entries[n_before:]]
                df = df.join(other, on=[ren[r] for r in ren], how=how)
                continue
            p.expect_kw("on")
            cond = p.expression()
            lk, rk = [], []
            _join_keys(cond, scope, left_names, lk, rk)
            df = df.join(other, on=[Column(BinOp("==", ColRef(a), ColRef(b))) for a, b in zip(lk, rk)], how=how)
    else:
        df, _ = scope.add(session.createDataFrame([(1,)], ["__dummy"]), None, None)
    where = p.expression() if p.accept_kw("where") else None
    group_keys = None
    if p.accept_kw("group"):
        p.expect_kw("by")
        group_keys = [p.expression()]
        while p.accept_op(","):
            group_keys.append(p.expression())
    having = p.expression() if p.accept_kw("having") else None
    order = None
    if p.accept_kw("order"):
        p.expect_kw("by")
        order = [_order_item(p)]
        while p.accept_op(","):
            order.append(_order_item(p))
    limit = None
    if p.accept_kw("limit"):
        limit = int(p.next().val)

    # ---- bind every expression to the FROM scope; output names are Spark's (unqualified) display names
    from .column import Alias
    out_exprs: List[Expr] = []
    names: List[str] = []
    for it in items:
        if isinstance(it, Star):
            qual = it.table.lower() if it.table else None
            cols = scope.columns(qual)
            if qual is not None and not cols:
                raise AnalysisException(f"cannot resolve '{it.table}.*'")
            for c, n in cols:
                if n == "__s0___dummy":
                    continue
                out_exprs.append(ColRef(n))
                names.append(c)
            continue
        if isinstance(it, Alias):
            out_exprs.append(scope.bind(it.x))
            names.append(it.alias)
        else:
            out_exprs.append(scope.bind(it))
            names.append(_display(it))
    # duplicate output names (SELECT * over a join) stay addressable with a suffix
    seen = {}
    for i, nm in enumerate(names):
        k = nm.lower()
        if k in seen:
            seen[k] += 1
            names[i] = f"{nm}_{seen[k]}"
        else:
            seen[k] = 0
    alias_map = {nm.lower(): e for nm, e in zip(names, out_exprs)}
    if where is not None:
        df = df.filter(Column(scope.bind(where)))
    having_b = scope.bind(having, alias_map) if having is not None else None
    order_b = [scope.bind(o, alias_map) for o in order] if order else None

    aggs: list = []
    for e in out_exprs:
        _collect_aggs(e, aggs)
    if having_b is not None:
        _collect_aggs(having_b, aggs)
    for o in order_b or []:
        _collect_aggs(o, aggs)
    if group_keys is not None or aggs:
        keys = []
        for k in group_keys or []:
            kb = scope.bind(k, alias_map) if not isinstance(k, Lit) else k
            if isinstance(kb, ColRef):
                keys.append(kb.col_name)
            elif isinstance(kb, Lit) and isinstance(kb.value, int) and 1 <= kb.value <= len(out_exprs):
                keys.append(Column(out_exprs[kb.value - 1]))  # GROUP BY <ordinal>
            else:
                keys.append(Column(kb))
        mapping = {id(a): f"__agg{i}" for i, a in enumerate(aggs)}
        agg_cols = [Column(a).alias(mapping[id(a)]) for a in aggs]
        df = df.groupBy(*keys).agg(*agg_cols) if agg_cols else df.groupBy(*keys).agg(
            F.count("*").alias("__cnt"))
        # non-column group keys come out under their display name: refer to them by it
        kmap = {}
        for k in keys:
            if isinstance(k, Column) and not isinstance(k._expr, ColRef):
                kmap[str(k._expr)] = k._expr.name()

        def fix(e):
            e = _replace_aggs(e, mapping)
            if kmap:
                e = _map_expr(e, lambda x: ColRef(kmap[str(x)]) if (not isinstance(x, (ColRef, Lit)) and
                                                                    str(x) in kmap) else None)
            return e
        out_exprs = [fix(e) for e in out_exprs]
        if having_b is not None:
            df = df.filter(Column(fix(having_b)))
        if order_b:
            order_b = [fix(o) for o in order_b]
    elif having_b is not None:
        df = df.filter(Column(having_b))
    proj = [Column(e).alias(nm) for e, nm in zip(out_exprs, names)]
    if distinct:
        out = df.select(*proj).distinct()
        if order_b:
            # after DISTINCT only output columns can be ordered on
            rev = {str(e): nm for e, nm in zip(out_exprs, names)}
            fixed = [_map_expr(o, lambda x: ColRef(rev[str(x)]) if str(x) in rev and not isinstance(x, SortOrder)
                               else None) for o in order_b]
            out = out.orderBy(*[Column(o) for o in fixed])
    else:
        if order_b:
            df = df.orderBy(*[Column(o) for o in order_b])
        out = df.select(*proj)
    if limit is not None:
        out = out.limit(limit)
    return out


def _order_item(p: Parser) -> Expr:
    e = p.expression()
    asc = True
    if p.accept_kw("asc"):
        asc = True
    elif p.accept_kw("desc"):
        asc = False
    nulls_first = None
    if p.accept_kw("nulls"):
        nulls_first = p.accept_kw("first")
        if not nulls_first:
            p.expect_kw("last")
    return SortOrder(e, asc, nulls_first)
