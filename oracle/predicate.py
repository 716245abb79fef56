"""CPU ORACLE of the filtered-search predicate — test infrastructure only.

Only ``tests/`` may use this module, as the checker of the HIP library's
predicate evaluator (``duckdb-lancedb_amd/csrc/meta.cpp``) and of filtered
search.  It restates, row by row in plain Python, the Lance-SQL predicates
the reference's optimizer pushes down (paths relative to ``/root/reference``):

* ``src/lance_optimizer.cpp:137-200`` literals: ``'..'`` with ``''`` escapes,
  integers, DuckDB float text, ``true`` / ``false``, ``NULL``;
* ``src/lance_optimizer.cpp:204-344`` shapes: ``col op const`` (or
  ``const op col``) with ``= != < > <= >=``, ``AND`` / ``OR`` (OR children in
  parentheses), ``NOT (..)``, ``col IS [NOT] NULL``, ``col [NOT] IN (..)``,
  ``BETWEEN`` (written as two comparisons; the parser also accepts the
  keyword);
* LanceDB ``only_if`` = prefilter: a row is searched iff the predicate is
  TRUE under SQL three-valued logic (NULL is not TRUE).

Rows are dicts ``{column: value or None}``; the implicit ``label`` column is
the row's label.  Parity with DataFusion itself is unpinned (the crate is not
in the container); the reference's own goldens
(``test/sql/lance_optimizer_filter.test``) pin the shapes it generates.
"""
from __future__ import annotations

import math
import re

_TOK = re.compile(r"""\s*(?:
    (?P<str>'(?:[^']|'')*')
  | (?P<qid>"[^"]*"|`[^`]*`)
  | (?P<num>-?(?:\d+\.?\d*(?:[eE][+-]?\d+)?|\.\d+(?:[eE][+-]?\d+)?))
  | (?P<id>[A-Za-z_][A-Za-z0-9_]*)
  | (?P<op><=|>=|!=|<>|==|=|<|>)
  | (?P<p>[(),])
)""", re.X)

KEYWORDS = {"AND", "OR", "NOT", "IS", "NULL", "IN", "BETWEEN", "TRUE", "FALSE"}


def tokenize(s):
    out, i = [], 0
    s = s.rstrip()
    while i < len(s):
        m = _TOK.match(s, i)
        if not m or m.end() == i:
            raise ValueError(f"bad predicate near {s[i:]!r}")
        i = m.end()
        kind = m.lastgroup
        text = m.group(kind)
        if kind == "num" and text.startswith("-") and out and out[-1][0] in ("id", "qid", "num", "str") \
                and not (out[-1][0] == "id" and out[-1][1].upper() in KEYWORDS):
            raise ValueError("binary minus is not part of the predicate language")
        out.append((kind, text))
    out.append(("end", ""))
    return out


class _P:
    def __init__(self, s):
        self.t = tokenize(s)
        self.i = 0

    def peek(self):
        return self.t[self.i]

    def kw(self, k, at=0):
        kind, text = self.t[min(self.i + at, len(self.t) - 1)]
        return kind == "id" and text.upper() == k

    def take(self):
        tok = self.t[self.i]
        self.i += 1
        return tok

    def expr(self):
        a = self.and_()
        while self.kw("OR"):
            self.take()
            b = self.and_()
            a = ("or", a, b)
        return a

    def and_(self):
        a = self.not_()
        while self.kw("AND"):
            self.take()
            b = self.not_()
            a = ("and", a, b)
        return a

    def not_(self):
        if self.kw("NOT"):
            self.take()
            return ("not", self.not_())
        return self.pred()

    def operand(self):
        kind, text = self.take()
        if kind == "p" and text == "(":
            e = self.expr()
            if self.take() != ("p", ")"):
                raise ValueError("expected )")
            return e
        if kind == "str":
            return ("lit", text[1:-1].replace("''", "'"))
        if kind == "num":
            return ("lit", float(text)) if re.search(r"[.eE]", text) else ("lit", int(text))
        if kind == "qid":
            return ("col", text[1:-1])
        if kind == "id":
            u = text.upper()
            if u == "NULL":
                return ("lit", None)
            if u in ("TRUE", "FALSE"):
                return ("lit", u == "TRUE")
            if u in KEYWORDS:
                raise ValueError(f"unexpected keyword {text}")
            return ("col", text)
        raise ValueError(f"unexpected {text!r}")

    def pred(self):
        a = self.operand()
        kind, text = self.peek()
        if kind == "op":
            self.take()
            op = {"<>": "!=", "==": "="}.get(text, text)
            return ("cmp", op, a, self.operand())
        if self.kw("IS"):
            self.take()
            neg = False
            if self.kw("NOT"):
                self.take()
                neg = True
            if not self.kw("NULL"):
                raise ValueError("expected NULL")
            self.take()
            return ("isnull", neg, a)
        neg = False
        if self.kw("NOT") and (self.kw("IN", 1) or self.kw("BETWEEN", 1)):
            self.take()
            neg = True
        if self.kw("IN"):
            self.take()
            if self.take() != ("p", "("):
                raise ValueError("expected (")
            vals = [self.operand()]
            while self.peek() == ("p", ","):
                self.take()
                vals.append(self.operand())
            if self.take() != ("p", ")"):
                raise ValueError("expected )")
            return ("in", neg, a, vals)
        if self.kw("BETWEEN"):
            self.take()
            lo = self.operand()
            if not self.kw("AND"):
                raise ValueError("expected AND")
            self.take()
            hi = self.operand()
            e = ("and", ("cmp", ">=", a, lo), ("cmp", "<=", a, hi))
            return ("not", e) if neg else e
        if neg:
            raise ValueError("expected IN or BETWEEN")
        return a


def parse(s):
    p = _P(s)
    e = p.expr()
    if p.peek()[0] != "end":
        raise ValueError(f"trailing {p.peek()[1]!r}")
    return e


def _cmp(a, b, op):
    if a is None or b is None:
        return None
    if isinstance(a, str) != isinstance(b, str) or isinstance(a, bool) != isinstance(b, bool):
        raise ValueError("incomparable types")
    if isinstance(a, float) or isinstance(b, float):
        a, b = float(a), float(b)
        if math.isnan(a) or math.isnan(b):  # NaN is the largest value
            c = 0 if (math.isnan(a) and math.isnan(b)) else (1 if math.isnan(a) else -1)
        else:
            c = (a > b) - (a < b)
    else:
        if isinstance(a, str):
            a, b = a.encode(), b.encode()  # byte order
        c = (a > b) - (a < b)
    return {"=": c == 0, "!=": c != 0, "<": c < 0, "<=": c <= 0, ">": c > 0, ">=": c >= 0}[op]


def _eval(e, row):
    t = e[0]
    if t == "lit":
        return e[1]
    if t == "col":
        if e[1] in row:
            return row[e[1]]
        raise KeyError(e[1])
    if t == "and":
        a, b = _eval(e[1], row), _eval(e[2], row)
        if a is False or b is False:
            return False
        return True if (a is True and b is True) else None
    if t == "or":
        a, b = _eval(e[1], row), _eval(e[2], row)
        if a is True or b is True:
            return True
        return False if (a is False and b is False) else None
    if t == "not":
        a = _eval(e[1], row)
        return None if a is None else (not a)
    if t == "cmp":
        return _cmp(_eval(e[2], row), _eval(e[3], row), e[1])
    if t == "isnull":
        return (_eval(e[2], row) is None) != e[1]
    if t == "in":
        x = _eval(e[2], row)
        acc = False
        for v in e[3]:
            r = _cmp(x, _eval(v, row), "=")
            if r is True:
                acc = True
            elif r is None and acc is False:
                acc = None
        return (None if acc is None else (not acc)) if e[1] else acc
    raise ValueError(t)


def mask(predicate, columns, labels, live):
    """columns: {name: list of values (None = NULL)}; returns a bool list:
    live and predicate TRUE."""
    e = parse(predicate)
    n = len(labels)
    out = []
    for r in range(n):
        row = {k: v[r] for k, v in columns.items()}
        row.setdefault("label", int(labels[r]))
        out.append(bool(live[r]) and _eval(e, row) is True)
    return out
