"""Host-side jq subset for Stage selector / value queries.

The Go host evaluates ``matchExpressions`` keys and ``*From`` expressions with gojq
(pkg/utils/expression/query.go:33-69).  In this engine the host evaluates each distinct
query ONCE per ingested object (to intern its result into feature bits / value records);
the device never runs jq.  Semantics follow Query.Execute: a runtime error makes the whole
result ``None`` (nil); ``null`` outputs are dropped; JSON numbers are float64, so they never
equal a string literal (selector.go:101-111).
"""
from __future__ import annotations

import json
import re
from typing import Callable, List, Optional


class JqError(Exception):
    pass


_TOK = re.compile(r"""
    (?P<ws>\s+)
  | (?P<str>"(?:[^"\\]|\\.)*")
  | (?P<num>\d+(?:\.\d+)?(?:[eE][-+]?\d+)?)
  | (?P<op>==|!=|<=|>=|//|[<>|,()\[\]?.])
  | (?P<ident>[A-Za-z_][A-Za-z0-9_]*)
""", re.X)


def _tokens(src):
    out, i = [], 0
    while i < len(src):
        m = _TOK.match(src, i)
        if not m:
            raise JqError(f"unexpected character at {i} in {src!r}")
        i = m.end()
        if m.lastgroup != "ws":
            out.append((m.lastgroup, m.group(), m.start()))
    return out


def _type(v):
    if v is None:
        return "null"
    if isinstance(v, bool):
        return "boolean"
    if isinstance(v, (int, float)):
        return "number"
    if isinstance(v, str):
        return "string"
    if isinstance(v, list):
        return "array"
    return "object"


def _index(v, k):
    if v is None:
        return None
    if isinstance(k, str):
        if not isinstance(v, dict):
            raise JqError(f"expected an object but got: {_type(v)}")
        return v.get(k)
    if isinstance(k, (int, float)) and not isinstance(k, bool):
        if not isinstance(v, list):
            raise JqError(f"expected an array but got: {_type(v)}")
        i = int(k // 1)
        if i < 0:
            i += len(v)
        return v[i] if 0 <= i < len(v) else None
    raise JqError("cannot index with " + _type(k))


def _iter(v):
    if isinstance(v, list):
        return list(v)
    if isinstance(v, dict):
        return list(v.values())
    raise JqError(f"cannot iterate over: {_type(v)}")


def _truthy(v):
    return not (v is None or v is False)


_ORDER = {"null": 0, "boolean": 1, "number": 3, "string": 4, "array": 5, "object": 6}


def _cmp(a, b):
    ta, tb = _type(a), _type(b)
    if ta != tb:
        oa = _ORDER[ta] + (1 if ta == "boolean" and a else 0)
        ob = _ORDER[tb] + (1 if tb == "boolean" and b else 0)
        return (oa > ob) - (oa < ob)
    if ta == "boolean":
        return (a > b) - (a < b)
    if ta in ("number", "string"):
        return (a > b) - (a < b)
    if ta == "null":
        return 0
    sa, sb = json.dumps(a, sort_keys=True), json.dumps(b, sort_keys=True)
    return 0 if a == b else ((sa > sb) - (sa < sb))


Fn = Callable[[object], List[object]]


class _Parser:
    def __init__(self, src):
        self.src = src
        self.t = _tokens(src)
        self.i = 0

    def peek(self, v=None):
        if self.i >= len(self.t):
            return None
        tok = self.t[self.i]
        if v is None or tok[1] == v:
            return tok
        return None

    def eat(self, v):
        if self.peek(v):
            self.i += 1
            return True
        return False

    def expect(self, v):
        if not self.eat(v):
            raise JqError(f"expected {v!r} in {self.src!r}")

    def parse(self) -> Fn:
        f = self.pipe()
        if self.i != len(self.t):
            raise JqError(f"unexpected token {self.t[self.i][1]!r} in {self.src!r}")
        return f

    def pipe(self) -> Fn:
        left = self.comma()
        if self.eat("|"):
            right = self.pipe()
            return lambda v: [y for x in left(v) for y in right(x)]
        return left

    def comma(self) -> Fn:
        fs = [self.alt()]
        while self.eat(","):
            fs.append(self.alt())
        if len(fs) == 1:
            return fs[0]
        return lambda v: [y for f in fs for y in f(v)]

    def alt(self) -> Fn:
        left = self.orx()
        if self.eat("//"):
            right = self.alt()

            def f(v):
                try:
                    got = [x for x in left(v) if _truthy(x)]
                except JqError:
                    got = []
                return got if got else right(v)
            return f
        return left

    def orx(self) -> Fn:
        left = self.andx()
        while self.peek("or"):
            self.i += 1
            l, r = left, self.andx()
            left = lambda v, l=l, r=r: [True if _truthy(a) else _truthy(b) for a in l(v)
                                        for b in ([None] if _truthy(a) else r(v))]
        return left

    def andx(self) -> Fn:
        left = self.cmp()
        while self.peek("and"):
            self.i += 1
            l, r = left, self.cmp()
            left = lambda v, l=l, r=r: [False if not _truthy(a) else _truthy(b) for a in l(v)
                                        for b in ([None] if not _truthy(a) else r(v))]
        return left

    def cmp(self) -> Fn:
        left = self.postfix()
        tok = self.peek()
        if tok and tok[1] in ("==", "!=", "<", "<=", ">", ">="):
            self.i += 1
            op = tok[1]
            right = self.postfix()
            test = {"==": lambda c: c == 0, "!=": lambda c: c != 0, "<": lambda c: c < 0,
                    "<=": lambda c: c <= 0, ">": lambda c: c > 0, ">=": lambda c: c >= 0}[op]
            return lambda v: [test(_cmp(a, b)) for b in right(v) for a in left(v)]
        return left

    def postfix(self) -> Fn:
        f = self.term()
        while True:
            tok = self.peek()
            if tok is None:
                return f
            if tok[1] == "." and self.i + 1 < len(self.t):
                nxt = self.t[self.i + 1]
                if nxt[0] == "ident" and nxt[2] == tok[2] + 1:
                    self.i += 2
                    f = self._field(f, nxt[1])
                    continue
                if nxt[0] == "str":
                    self.i += 2
                    f = self._field(f, json.loads(nxt[1]))
                    continue
                if nxt[1] == "[":
                    self.i += 1
                    continue
                return f
            if tok[1] == "[":
                self.i += 1
                if self.eat("]"):
                    f = (lambda g: lambda v: [y for x in g(v) for y in _iter(x)])(f)
                    continue
                key = self.pipe()
                self.expect("]")
                f = (lambda g, k: lambda v: [_index(x, kk) for x in g(v) for kk in k(v)])(f, key)
                continue
            if tok[1] == "?":
                self.i += 1
                g = f

                def tried(v, g=g):
                    try:
                        return g(v)
                    except JqError:
                        return []
                f = tried
                continue
            return f

    @staticmethod
    def _field(f, name):
        return lambda v: [_index(x, name) for x in f(v)]

    def term(self) -> Fn:
        tok = self.peek()
        if tok is None:
            raise JqError(f"unexpected end of {self.src!r}")
        kind, text, pos = tok
        if text == ".":
            nxt = self.t[self.i + 1] if self.i + 1 < len(self.t) else None
            if nxt and ((nxt[0] == "ident" and nxt[2] == pos + 1) or nxt[0] == "str" or nxt[1] == "["):
                return lambda v: [v]  # postfix() consumes the .name / ."x" / .[..]
            self.i += 1
            return lambda v: [v]
        self.i += 1
        if kind == "str":
            s = json.loads(text)
            return lambda v: [s]
        if kind == "num":
            n = float(text)
            return lambda v: [n]
        if text == "(":
            f = self.pipe()
            self.expect(")")
            return f
        if text == "[":
            if self.eat("]"):
                return lambda v: [[]]
            f = self.pipe()
            self.expect("]")
            return lambda v: [f(v)]
        if kind == "ident":
            if text == "true":
                return lambda v: [True]
            if text == "false":
                return lambda v: [False]
            if text == "null":
                return lambda v: [None]
            if text == "not":
                return lambda v: [not _truthy(v)]
            if text == "empty":
                return lambda v: []
            if text == "length":
                def length(v):
                    if v is None:
                        return [0.0]
                    if isinstance(v, bool):
                        raise JqError("boolean has no length")
                    if isinstance(v, (int, float)):
                        return [abs(float(v))]
                    return [float(len(v))]
                return length
            if text == "select":
                self.expect("(")
                c = self.pipe()
                self.expect(")")
                return lambda v: [v for x in c(v) if _truthy(x)]
        raise JqError(f"unsupported jq syntax {text!r} in {self.src!r}")


class Query:
    """expression.NewQuery / Query.Execute."""

    def __init__(self, src: str):
        self.src = src
        self._f = _Parser(src).parse()

    def execute(self, v) -> Optional[list]:
        try:
            out = self._f(v)
        except (JqError, TypeError, RecursionError):
            return None
        return [x for x in out if x is not None]


def has_value(d, values) -> bool:
    """selector.go:101-111: string, bool (FormatBool) and int (FormatInt) only.  JSON numbers
    decode as float64, which never match."""
    if isinstance(d, bool):
        return ("true" if d else "false") in values
    if isinstance(d, str):
        return d in values
    return False
