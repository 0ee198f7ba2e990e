"""Host-side jq subset for Stage selector / value queries (the Python mirror of
``kwok_amd/csrc/jqc.hpp``, which the native encoder and compiler run).

The Go host evaluates ``matchExpressions`` keys and ``*From`` expressions with gojq
(pkg/utils/expression/query.go:33-69, gojq v0.12.16).  In this engine the host evaluates each
distinct query ONCE per ingested object (to intern its result into feature bits / value records);
the device never runs jq.  Semantics follow Query.Execute: a runtime error makes the whole result
``None`` (nil); ``null`` outputs are dropped.  Values are held as gojq holds them: every JSON number
of the input is a float64 (a Python float here), while number literals, ``length`` and int
arithmetic give gojq ints (Python ints) — selector.go's hasValue matches ints (FormatInt) but never
float64s.  Objects iterate and list their keys sorted, as gojq's maps do.

The subset: paths (``.a``, ``."a"``, ``.[e]``, ``.[]``, ``.a.[]``, ``?``), ``|``, ``,``, ``//``,
``and`` / ``or``, comparisons, ``+ - * / %``, unary ``-``, literals, ``[...]``, ``{...}``,
``if``-``then``-``elif``-``else``-``end``, ``try e``, the assignments ``= |= += -= *= /= %= //=`` and
the builtins listed in ``_F0`` / ``_F1``; anything else raises ``JqError`` at parse time with the
construct named (``EncoderUnsupported`` for the native encoder).
"""
from __future__ import annotations

import json
import math
from typing import Callable, List, Optional


class JqError(Exception):
    pass


class _RunError(Exception):
    """A runtime error inside a query (Execute -> nil)."""


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


def _is_int(v):
    return isinstance(v, int) and not isinstance(v, bool)


def _floats(v):
    """ToJSONStandard's json.Unmarshal: every JSON number is a float64."""
    if isinstance(v, bool) or v is None or isinstance(v, str):
        return v
    if isinstance(v, int):
        return float(v)
    if isinstance(v, float):
        return v
    if isinstance(v, list):
        return [_floats(x) for x in v]
    if isinstance(v, dict):
        return {k: _floats(x) for k, x in v.items()}
    return v


def _truthy(v):
    return not (v is None or v is False)


def _rank(v):
    t = _type(v)
    if t == "boolean":
        return 2 if v else 1
    return {"null": 0, "number": 3, "string": 4, "array": 5, "object": 6}[t]


def _skey(s: str):
    return s.encode("utf-8", "surrogatepass")


def _cmp(a, b):
    """gojq compare: null < false < true < numbers < strings < arrays < objects."""
    ra, rb = _rank(a), _rank(b)
    if ra != rb:
        return -1 if ra < rb else 1
    if ra == 3:
        return (a > b) - (a < b)
    if ra == 4:
        x, y = _skey(a), _skey(b)
        return (x > y) - (x < y)
    if ra == 5:
        for x, y in zip(a, b):
            c = _cmp(x, y)
            if c:
                return c
        return (len(a) > len(b)) - (len(a) < len(b))
    if ra == 6:
        ka, kb = sorted(a, key=_skey), sorted(b, key=_skey)
        for x, y in zip(ka, kb):
            if x != y:
                return -1 if _skey(x) < _skey(y) else 1
        if len(ka) != len(kb):
            return -1 if len(ka) < len(kb) else 1
        for k in ka:
            c = _cmp(a[k], b[k])
            if c:
                return c
        return 0
    return 0


def _sorted_items(o: dict):
    return sorted(o.items(), key=lambda kv: _skey(kv[0]))


def _enc_float(f: float) -> str:
    if f != f:
        return "null"
    f = max(min(f, 1.7976931348623157e308), -1.7976931348623157e308)
    x = abs(f)
    r = repr(f)
    if x != 0 and (x < 1e-6 or x >= 1e21):
        m, e = ("%r" % f).lower().split("e") if "e" in r.lower() else (r, "0")
        mant = m
        if "." in mant:
            mant = mant.rstrip("0").rstrip(".")
        e10 = int(e)
        return mant + ("e-" if e10 < 0 else "e+") + str(abs(e10))
    d = format(f, ".17g")
    # the shortest round-trip digits in fixed notation
    for p in range(1, 18):
        cand = format(f, ".%de" % (p - 1))
        if float(cand) == f:
            d = cand
            break
    m, e = d.split("e")
    e10 = int(e)
    neg = m.startswith("-")
    digits = m.replace("-", "").replace(".", "")
    digits = digits.rstrip("0") or "0"
    if e10 < 0:
        out = "0." + "0" * (-e10 - 1) + digits
    elif len(digits) <= e10 + 1:
        out = digits + "0" * (e10 + 1 - len(digits))
    else:
        out = digits[:e10 + 1] + "." + digits[e10 + 1:]
    return ("-" if neg else "") + out


def encode(v) -> str:
    """gojq's encoding (tostring, kwk_jq_eval's output)."""
    if v is None:
        return "null"
    if v is True:
        return "true"
    if v is False:
        return "false"
    if _is_int(v):
        return str(v)
    if isinstance(v, float):
        return _enc_float(v)
    if isinstance(v, str):
        return json.dumps(v, ensure_ascii=False)
    if isinstance(v, list):
        return "[" + ",".join(encode(x) for x in v) + "]"
    return "{" + ",".join(json.dumps(k, ensure_ascii=False) + ":" + encode(x) for k, x in _sorted_items(v)) + "}"


# ------------------------------------------------------------------ syntax tree
class N:
    __slots__ = ("k", "name", "lit", "a", "b", "args", "obj")

    def __init__(self, k, a=None, b=None, name="", lit=None):
        self.k, self.a, self.b, self.name, self.lit = k, a, b, name, lit
        self.args = []
        self.obj = []


_F0 = {"empty", "error", "not", "length", "keys", "keys_unsorted", "type", "tostring", "tonumber", "ascii_downcase",
       "ascii_upcase", "add", "any", "all", "first", "last", "values"}
_F1 = {"error", "has", "startswith", "endswith", "ltrimstr", "rtrimstr", "contains", "select", "map", "first"}
_KW_BAD = ("reduce", "foreach", "def", "label", "import", "include", "as", "__loc__")


def _idc(c):
    return c.isalnum() or c == "_"


def _isalpha(c):
    return ("a" <= c <= "z") or ("A" <= c <= "Z") or c == "_"


def _isdigit(c):
    return "0" <= c <= "9"


class _Parser:
    def __init__(self, src):
        self.s = src
        self.i = 0

    def bad(self, what):
        raise JqError(f"jq construct not supported natively: {what} in '{self.s}'")

    def ws(self):
        s = self.s
        while True:
            while self.i < len(s) and s[self.i].isspace():
                self.i += 1
            if self.i < len(s) and s[self.i] == "#":
                while self.i < len(s) and s[self.i] != "\n":
                    self.i += 1
                continue
            return

    def at(self, t):
        self.ws()
        return self.s.startswith(t, self.i)

    def eat(self, t):
        if not self.at(t):
            return False
        self.i += len(t)
        return True

    def eat_op(self, t, longer=()):
        if not self.at(t):
            return False
        if any(self.s.startswith(x, self.i) for x in longer):
            return False
        self.i += len(t)
        return True

    def at_kw(self, t):
        self.ws()
        n = len(t)
        return self.s.startswith(t, self.i) and not (self.i + n < len(self.s) and _idc(self.s[self.i + n]))

    def eat_kw(self, t):
        if not self.at_kw(t):
            return False
        self.i += len(t)
        return True

    def expect(self, t):
        if not self.eat(t):
            self.bad(f"syntax (expected '{t}')")

    def ident(self):
        self.ws()
        b = self.i
        s = self.s
        if self.i < len(s) and _isalpha(s[self.i]):
            self.i += 1
            while self.i < len(s) and _idc(s[self.i]):
                self.i += 1
        return s[b:self.i]

    def string_lit(self):
        self.ws()
        s = self.s
        if self.i >= len(s) or s[self.i] != '"':
            self.bad("syntax (expected a string)")
        b = self.i
        self.i += 1
        while self.i < len(s) and s[self.i] != '"':
            if s[self.i] == "\\":
                if self.i + 1 < len(s) and s[self.i + 1] == "(":
                    self.bad("string interpolation")
                self.i += 1
            self.i += 1
        if self.i >= len(s):
            self.bad("syntax (unterminated string)")
        self.i += 1
        try:
            v = json.loads(s[b:self.i])
        except ValueError:
            self.bad("syntax (bad string literal)")
        return v

    def parse(self):
        n = self.pipe()
        self.ws()
        if self.i != len(self.s):
            self.bad(f"unexpected '{self.s[self.i:self.i + 8]}'")
        return n

    def pipe(self):
        l = self.comma()
        if self.eat_op("|", ("|=",)):
            return N("PIPE", l, self.pipe())
        return l

    def comma(self):
        l = self.alt()
        while self.eat(","):
            l = N("COMMA", l, self.alt())
        return l

    def alt(self):
        l = self.assign()
        if self.eat_op("//", ("//=",)):
            return N("ALT", l, self.alt())
        return l

    def assign(self):
        l = self.orx()
        for op in ("|=", "+=", "-=", "*=", "/=", "%=", "//="):
            if self.eat(op):
                return N("ASSIGN", l, self.orx(), op)
        if self.eat_op("=", ("==",)):
            return N("ASSIGN", l, self.orx(), "=")
        return l

    def orx(self):
        l = self.andx()
        while self.eat_kw("or"):
            l = N("OR", l, self.andx())
        return l

    def andx(self):
        l = self.cmp()
        while self.eat_kw("and"):
            l = N("AND", l, self.cmp())
        return l

    def cmp(self):
        l = self.additive()
        for op in ("==", "!=", "<=", ">=", "<", ">"):
            if self.eat(op):
                return N("CMP", l, self.additive(), op)
        return l

    def additive(self):
        l = self.multiplicative()
        while True:
            if self.eat_op("+", ("+=",)):
                l = N("ARITH", l, self.multiplicative(), "+")
            elif self.eat_op("-", ("-=",)):
                l = N("ARITH", l, self.multiplicative(), "-")
            else:
                return l

    def multiplicative(self):
        l = self.unary()
        while True:
            if self.eat_op("*", ("*=",)):
                l = N("ARITH", l, self.unary(), "*")
            elif self.eat_op("/", ("/=", "//")):
                l = N("ARITH", l, self.unary(), "/")
            elif self.eat_op("%", ("%=",)):
                l = N("ARITH", l, self.unary(), "%")
            else:
                return l

    def unary(self):
        if self.eat_op("-", ("-=",)):
            return N("NEG", self.postfix())
        return self.postfix()

    def postfix(self):
        n = self.term()
        s = self.s
        while True:
            self.ws()
            if self.i >= len(s):
                return n
            if self.at_kw("as"):
                self.bad("'as'")
            c = s[self.i]
            if c == "?":
                if s.startswith("?//", self.i):
                    self.bad("'?//'")
                self.i += 1
                n = N("TRY", n)
                continue
            if c == "[":
                n = self.bracket(n)
                continue
            if c == "." and self.i + 1 < len(s):
                d = s[self.i + 1]
                if d == "[":
                    self.i += 1
                    n = self.bracket(n)
                    continue
                if d == '"':
                    self.i += 1
                    n = N("FIELD", n, name=self.string_lit())
                    continue
                if _isalpha(d):
                    self.i += 1
                    n = N("FIELD", n, name=self.ident())
                    continue
            return n

    def bracket(self, base):
        self.expect("[")
        if self.eat("]"):
            return N("ITER", base)
        if self.at(":"):
            self.bad("slices")
        key = self.pipe()
        if self.at(":"):
            self.bad("slices")
        self.expect("]")
        return N("INDEX", base, key)

    def term(self):
        self.ws()
        s = self.s
        if self.i >= len(s):
            self.bad("syntax (unexpected end)")
        c = s[self.i]
        if c == ".":
            if s.startswith("..", self.i):
                self.bad("'..'")
            d = s[self.i + 1] if self.i + 1 < len(s) else ""
            if d and _isalpha(d):
                self.i += 1
                return N("FIELD", N("IDENT"), name=self.ident())
            if d == '"':
                self.i += 1
                return N("FIELD", N("IDENT"), name=self.string_lit())
            if d and _isdigit(d):
                return self.number()
            self.i += 1
            return N("IDENT")
        if c == "$":
            self.bad("variables")
        if c == "@":
            self.bad("formats")
        if _isdigit(c):
            return self.number()
        if c == '"':
            return N("LIT", lit=self.string_lit())
        if c == "(":
            self.i += 1
            n = self.pipe()
            self.expect(")")
            return n
        if c == "[":
            self.i += 1
            n = N("ARRAY")
            if not self.eat("]"):
                n.a = self.pipe()
                self.expect("]")
            return n
        if c == "{":
            return self.object()
        if self.eat_kw("if"):
            return self.if_rest()
        if self.eat_kw("try"):
            body = self.postfix()
            if self.at_kw("catch"):
                self.bad("'try ... catch'")
            return N("TRY", body)
        for kw in _KW_BAD:
            if self.at_kw(kw):
                self.bad(f"'{kw}'")
        if self.eat_kw("true"):
            return N("LIT", lit=True)
        if self.eat_kw("false"):
            return N("LIT", lit=False)
        if self.eat_kw("null"):
            return N("LIT", lit=None)
        name = self.ident()
        if not name:
            self.bad(f"syntax ('{c}')")
        f = N("FUNC", name=name)
        if self.eat("("):
            while True:
                f.args.append(self.pipe())
                if self.eat(";"):
                    continue
                self.expect(")")
                break
        if not ((not f.args and name in _F0) or (len(f.args) == 1 and name in _F1)):
            self.bad(f"function {name}/{len(f.args)}")
        return f

    def number(self):
        s = self.s
        b = self.i
        while self.i < len(s) and _isdigit(s[self.i]):
            self.i += 1
        frac = False
        if self.i < len(s) and s[self.i] == ".":
            frac = True
            self.i += 1
            while self.i < len(s) and _isdigit(s[self.i]):
                self.i += 1
        if self.i < len(s) and s[self.i] in "eE":
            j = self.i + 1
            if j < len(s) and s[j] in "+-":
                j += 1
            if j < len(s) and _isdigit(s[j]):
                frac = True
                self.i = j
                while self.i < len(s) and _isdigit(s[self.i]):
                    self.i += 1
        t = s[b:self.i]
        if not frac:
            v = int(t)
            if -2**63 <= v < 2**63:
                return N("LIT", lit=v)
        return N("LIT", lit=float(t))

    def object(self):
        self.expect("{")
        n = N("OBJECT")
        if self.eat("}"):
            return n
        s = self.s
        while True:
            self.ws()
            if self.i < len(s) and s[self.i] == '"':
                key = N("LIT", lit=self.string_lit())
            elif self.i < len(s) and s[self.i] == "(":
                self.i += 1
                key = self.pipe()
                self.expect(")")
            elif self.i < len(s) and s[self.i] == "$":
                self.bad("variables")
            else:
                name = self.ident()
                if not name:
                    self.bad("syntax (object key)")
                key = N("LIT", lit=name)
            if self.eat(":"):
                val = self.objval()
            else:
                if key.k != "LIT":
                    self.bad("syntax (object key without a value)")
                val = N("FIELD", N("IDENT"), name=key.lit)
            n.obj.append((key, val))
            if self.eat(","):
                continue
            self.expect("}")
            return n

    def objval(self):
        l = self.alt()
        if self.eat_op("|", ("|=",)):
            return N("PIPE", l, self.objval())
        return l

    def if_rest(self):
        n = N("IF")
        while True:
            n.args.append(self.pipe())
            if not self.eat_kw("then"):
                self.bad("syntax (expected 'then')")
            n.args.append(self.pipe())
            if self.eat_kw("elif"):
                continue
            if self.eat_kw("else"):
                n.args.append(self.pipe())
                if not self.eat_kw("end"):
                    self.bad("syntax (expected 'end')")
                return n
            if not self.eat_kw("end"):
                self.bad("syntax (expected 'end')")
            return n


# ------------------------------------------------------------------ evaluation
def _field(v, key):
    if v is None:
        return None
    if not isinstance(v, dict):
        raise _RunError(f"expected an object but got: {_type(v)}")
    return v.get(key)


def _index(v, k):
    if isinstance(k, str):
        return _field(v, k)
    if isinstance(k, (int, float)) and not isinstance(k, bool):
        if v is None:
            return None
        if not isinstance(v, list):
            raise _RunError(f"expected an array but got: {_type(v)}")
        if k != k:
            return None
        i = math.floor(k)
        if i < 0:
            i += len(v)
        return v[i] if 0 <= i < len(v) else None
    if k is None and v is None:
        return None
    raise _RunError(f"cannot index {_type(v)} with {_type(k)}")


def _iter(v):
    if isinstance(v, list):
        return list(v)
    if isinstance(v, dict):
        return [x for _, x in _sorted_items(v)]
    raise _RunError(f"cannot iterate over: {_type(v)}")


def _i64(v):
    return -2**63 <= v < 2**63


def _arith(op, l, r):
    ints = _is_int(l) and _is_int(r)
    num = lambda x: isinstance(x, (int, float)) and not isinstance(x, bool)  # noqa: E731
    if op == "+":
        if l is None:
            return r
        if r is None:
            return l
        if num(l) and num(r):
            if ints and _i64(l + r):
                return l + r
            return float(l) + float(r)
        if isinstance(l, str) and isinstance(r, str):
            return l + r
        if isinstance(l, list) and isinstance(r, list):
            return l + r
        if isinstance(l, dict) and isinstance(r, dict):
            o = dict(l)
            o.update(r)
            return o
    elif op == "-":
        if num(l) and num(r):
            if ints and _i64(l - r):
                return l - r
            return float(l) - float(r)
        if isinstance(l, list) and isinstance(r, list):
            return [e for e in l if not any(_cmp(e, x) == 0 for x in r)]
    elif op == "*":
        if num(l) and num(r):
            if ints and _i64(l * r):
                return l * r
            return float(l) * float(r)
        if isinstance(l, dict) and isinstance(r, dict):
            o = dict(l)
            for k, v in r.items():
                o[k] = _arith("*", o[k], v) if isinstance(o.get(k), dict) and isinstance(v, dict) else v
            return o
    elif op == "/":
        if num(l) and num(r):
            if r == 0:
                raise _RunError("cannot divide by zero")
            if ints and l % r == 0 and not (r == -1 and l == -2**63):
                return int(abs(l) // abs(r)) * (1 if (l >= 0) == (r > 0) else -1)
            return float(l) / float(r)
        if isinstance(l, str) and isinstance(r, str):
            if l == "":
                return []
            if r == "":
                return list(l)
            return l.split(r)
    elif op == "%":
        if num(l) and num(r):
            if l != l or r != r:
                return float("nan")
            x, y = int(l), int(r)
            if y == 0:
                raise _RunError("cannot modulo by zero")
            z = abs(x) % abs(y)
            return -z if x < 0 else z
    raise _RunError(f"cannot {op}: {_type(l)} and {_type(r)}")


def _contains(a, b):
    if _type(a) != _type(b):
        raise _RunError(f"{_type(a)} and {_type(b)} cannot have their containment checked")
    if isinstance(a, str):
        return b in a
    if isinstance(a, list):
        return all(any(_type(x) == _type(y) and _contains(x, y) for x in a) for y in b)
    if isinstance(a, dict):
        for k, y in b.items():
            if k not in a:
                return False
            if _type(a[k]) != _type(y):
                raise _RunError("cannot have their containment checked")
            if not _contains(a[k], y):
                return False
        return True
    return _cmp(a, b) == 0


def _setpath(root, p, i, val):
    if i == len(p):
        return val
    k = p[i]
    if isinstance(k, str):
        if root is not None and not isinstance(root, dict):
            raise _RunError(f"expected an object but got: {_type(root)}")
        o = dict(root) if isinstance(root, dict) else {}
        o[k] = _setpath(o.get(k), p, i + 1, val)
        return o
    if not (isinstance(k, (int, float)) and not isinstance(k, bool)):
        raise _RunError("invalid path component")
    if root is not None and not isinstance(root, list):
        raise _RunError(f"expected an array but got: {_type(root)}")
    a = list(root) if isinstance(root, list) else []
    idx = math.floor(k)
    if idx < 0:
        idx += len(a)
    if idx < 0:
        raise _RunError("out of bounds negative array index")
    if idx > 0x7FFFFFF:
        raise _RunError("array index too large")
    while len(a) <= idx:
        a.append(None)
    a[idx] = _setpath(a[idx], p, i + 1, val)
    return a


def _getpath(root, p):
    cur = root
    for k in p:
        cur = _index(cur, k)
    return cur


def _paths(n, v, base):
    """[(path, value)] of a path expression."""
    k = n.k
    if k == "IDENT":
        return [(base, v)]
    if k == "FIELD":
        return [(p + [n.name], _field(x, n.name)) for p, x in _paths(n.a, v, base)]
    if k == "INDEX":
        return [(p + [key], _index(x, key)) for p, x in _paths(n.a, v, base) for key in _ev(n.b, v)]
    if k == "ITER":
        out = []
        for p, x in _paths(n.a, v, base):
            if isinstance(x, list):
                out += [(p + [i], e) for i, e in enumerate(x)]
            elif isinstance(x, dict):
                out += [(p + [kk], e) for kk, e in _sorted_items(x)]
            elif x is not None:
                raise _RunError(f"cannot iterate over: {_type(x)}")
        return out
    if k == "PIPE":
        return [pp for p, x in _paths(n.a, v, base) for pp in _paths(n.b, x, p)]
    if k == "COMMA":
        return _paths(n.a, v, base) + _paths(n.b, v, base)
    if k == "TRY":
        out = []
        try:
            for e in _paths_gen(n.a, v, base):
                out.append(e)
        except _RunError:
            pass
        return out
    if k == "FUNC":
        if n.name == "select":
            return [(base, v) for c in _ev(n.args[0], v) if _truthy(c)]
        if n.name == "empty":
            return []
        if n.name == "first" and n.args:
            out = []
            try:
                for e in _paths_gen(n.args[0], v, base):
                    out.append(e)
                    break
            except _RunError:
                if not out:
                    raise
            return out
    if k == "IF":
        return _if(n, v, lambda b: _paths(b, v, base), lambda: [(base, v)])
    raise _RunError("invalid path expression")


def _paths_gen(n, v, base):
    yield from _paths(n, v, base)


def _if(n, v, run, identity):
    nc = len(n.args) // 2

    def branch(i):
        if i == nc:
            return run(n.args[-1]) if len(n.args) % 2 else identity()
        out = []
        for c in _ev(n.args[2 * i], v):
            out += run(n.args[2 * i + 1]) if _truthy(c) else branch(i + 1)
        return out
    return branch(0)


def _ev(n, v) -> list:
    """All outputs of node n on input v (a _RunError propagates)."""
    return list(_gen(n, v))


def _gen(n, v):
    k = n.k
    if k == "IDENT":
        yield v
    elif k == "FIELD":
        for x in _gen(n.a, v):
            yield _field(x, n.name)
    elif k == "INDEX":
        for x in _gen(n.a, v):
            for key in _gen(n.b, v):
                yield _index(x, key)
    elif k == "ITER":
        for x in _gen(n.a, v):
            yield from _iter(x)
    elif k == "TRY":
        try:
            for x in _gen(n.a, v):
                yield x
        except _RunError:
            return
    elif k == "PIPE":
        for x in _gen(n.a, v):
            yield from _gen(n.b, x)
    elif k == "COMMA":
        yield from _gen(n.a, v)
        yield from _gen(n.b, v)
    elif k == "ALT":
        got = []
        try:
            for x in _gen(n.a, v):
                if _truthy(x):
                    got.append(x)
        except _RunError:
            pass
        if got:
            yield from got
        else:
            yield from _gen(n.b, v)
    elif k == "OR":
        for l in _gen(n.a, v):
            if _truthy(l):
                yield True
            else:
                for r in _gen(n.b, v):
                    yield _truthy(r)
    elif k == "AND":
        for l in _gen(n.a, v):
            if not _truthy(l):
                yield False
            else:
                for r in _gen(n.b, v):
                    yield _truthy(r)
    elif k == "CMP":
        test = {"==": lambda c: c == 0, "!=": lambda c: c != 0, "<": lambda c: c < 0, "<=": lambda c: c <= 0,
                ">": lambda c: c > 0, ">=": lambda c: c >= 0}[n.name]
        for r in _gen(n.b, v):
            for l in _gen(n.a, v):
                yield test(_cmp(l, r))
    elif k == "ARITH":
        for r in _gen(n.b, v):
            for l in _gen(n.a, v):
                yield _arith(n.name, l, r)
    elif k == "NEG":
        for x in _gen(n.a, v):
            if not (isinstance(x, (int, float)) and not isinstance(x, bool)):
                raise _RunError(f"cannot negate: {_type(x)}")
            yield -x if (not _is_int(x) or x != -2**63) else float(-x)
    elif k == "LIT":
        yield n.lit
    elif k == "ARRAY":
        yield [] if n.a is None else list(_gen(n.a, v))
    elif k == "OBJECT":
        def rec(i, cur):
            if i == len(n.obj):
                o = {}
                for kk, vv in cur:
                    o[kk] = vv
                yield o
                return
            for key in _gen(n.obj[i][0], v):
                if not isinstance(key, str):
                    raise _RunError(f"expected a string for object key but got: {_type(key)}")
                for val in _gen(n.obj[i][1], v):
                    yield from rec(i + 1, cur + [(key, val)])
        yield from rec(0, [])
    elif k == "IF":
        yield from _if(n, v, lambda b: _ev(b, v), lambda: [v])
    elif k == "ASSIGN":
        op = n.name
        if op == "|=":
            out = v
            for p, _ in _paths(n.a, v, []):
                old = _getpath(out, p)
                got = _ev(n.b, old)
                if not got:
                    raise _RunError("update-assignment with no output is not supported")
                out = _setpath(out, p, 0, got[0])
            yield out
            return
        for val in _gen(n.b, v):
            out = v
            for p, _ in _paths(n.a, v, []):
                if op == "=":
                    out = _setpath(out, p, 0, val)
                elif op == "//=":
                    old = _getpath(out, p)
                    out = _setpath(out, p, 0, old if _truthy(old) else val)
                else:
                    out = _setpath(out, p, 0, _arith(op[0], _getpath(out, p), val))
            yield out
    elif k == "FUNC":
        yield from _builtin(n, v)


def _builtin(n, x):
    f = n.name
    if not n.args:
        if f == "empty":
            return
        if f == "error":
            raise _RunError(x if isinstance(x, str) else "error")
        if f == "not":
            yield not _truthy(x)
        elif f == "length":
            if x is None:
                yield 0
            elif isinstance(x, bool):
                raise _RunError("length cannot be applied to: boolean")
            elif _is_int(x):
                yield abs(x) if x != -2**63 else float(2**63)
            elif isinstance(x, float):
                yield abs(x)
            else:
                yield len(x)
        elif f in ("keys", "keys_unsorted"):
            if isinstance(x, dict):
                yield [kk for kk, _ in _sorted_items(x)]
            elif isinstance(x, list):
                yield list(range(len(x)))
            else:
                raise _RunError(f"{f} cannot be applied to: {_type(x)}")
        elif f == "type":
            yield _type(x)
        elif f == "tostring":
            yield x if isinstance(x, str) else encode(x)
        elif f == "tonumber":
            if isinstance(x, (int, float)) and not isinstance(x, bool):
                yield x
            elif isinstance(x, str):
                t = x
                if t and (t.isdigit() or (t[0] in "+-" and t[1:].isdigit())) and _i64(int(t)):
                    yield int(t)
                else:
                    try:
                        v = json.loads(t)
                    except ValueError:
                        raise _RunError(f"cannot parse '{t}' as number") from None
                    if isinstance(v, bool) or not isinstance(v, (int, float)):
                        raise _RunError(f"cannot parse '{t}' as number")
                    yield float(v)
            else:
                raise _RunError(f"tonumber cannot be applied to: {_type(x)}")
        elif f in ("ascii_downcase", "ascii_upcase"):
            if not isinstance(x, str):
                raise _RunError(f"{f} cannot be applied to: {_type(x)}")
            if f == "ascii_downcase":
                yield "".join(chr(ord(c) ^ 0x20) if "A" <= c <= "Z" else c for c in x)
            else:
                yield "".join(chr(ord(c) ^ 0x20) if "a" <= c <= "z" else c for c in x)
        elif f == "add":
            acc, first = None, True
            for e in _iter(x):
                acc = e if first else _arith("+", acc, e)
                first = False
            yield acc
        elif f in ("any", "all"):
            vals = [_truthy(e) for e in _iter(x)]
            yield any(vals) if f == "any" else all(vals)
        elif f in ("first", "last"):
            yield _index(x, 0 if f == "first" else -1)
        elif f == "values":
            if x is not None:
                yield x
        return
    a0 = n.args[0]
    if f == "select":
        for c in _gen(a0, x):
            if _truthy(c):
                yield x
        return
    if f == "map":
        yield [y for e in _iter(x) for y in _gen(a0, e)]
        return
    if f == "first":
        out = []
        try:
            for y in _gen(a0, x):
                out.append(y)
                break
        except _RunError:
            if not out:
                raise
        yield from out
        return
    for y in _gen(a0, x):
        if f == "error":
            raise _RunError(y if isinstance(y, str) else "error")
        if f == "has":
            if isinstance(x, dict) and isinstance(y, str):
                yield y in x
            elif isinstance(x, list) and isinstance(y, (int, float)) and not isinstance(y, bool):
                yield False if y != y else 0 <= int(y) < len(x)
            else:
                raise _RunError(f"has({_type(y)}) cannot be applied to: {_type(x)}")
        elif f in ("startswith", "endswith"):
            if not (isinstance(x, str) and isinstance(y, str)):
                raise _RunError(f"{f}() cannot be applied to: {_type(x)}")
            yield x.startswith(y) if f == "startswith" else x.endswith(y)
        elif f in ("ltrimstr", "rtrimstr"):
            if isinstance(x, str) and isinstance(y, str):
                if f == "ltrimstr" and x.startswith(y):
                    yield x[len(y):]
                    continue
                if f == "rtrimstr" and x.endswith(y) and y:
                    yield x[:len(x) - len(y)]
                    continue
                if f == "rtrimstr" and not y:
                    yield x
                    continue
            yield x
        elif f == "contains":
            yield _contains(x, y)


Fn = Callable[[object], List[object]]


class Query:
    """expression.NewQuery / Query.Execute."""

    def __init__(self, src: str):
        self.src = src
        self.root = _Parser(src).parse()

    def execute(self, v) -> Optional[list]:
        """Query.Execute on a JSON document (its numbers taken as float64)."""
        return self.execute_std(_floats(v))

    def execute_std(self, v) -> Optional[list]:
        """Query.Execute on a value already in gojq form (floats for JSON numbers)."""
        try:
            out = list(_gen(self.root, v))
        except (_RunError, RecursionError, TypeError, ValueError, OverflowError):
            return None
        return [x for x in out if x is not None]


def has_value(d, values) -> bool:
    """selector.go:101-111: string, bool (FormatBool) and gojq int (FormatInt).  JSON numbers
    decode as float64, which never match."""
    if isinstance(d, bool):
        return ("true" if d else "false") in values
    if isinstance(d, str):
        return d in values
    if _is_int(d):
        return str(d) in values
    return False
