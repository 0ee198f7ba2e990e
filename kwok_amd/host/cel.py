"""CEL subset for kwok's Metric and ResourceUsage expressions.

kwok evaluates CEL (github.com/google/cel-go v0.17.8 through github.com/wzshiming/easycel
v0.5.0, neither under /root/reference) in an environment built by pkg/utils/cel/environment.go
and pkg/kwok/metrics/evaluator.go:51-144: variables ``node``, ``pod``, ``container`` (typed
Kubernetes objects), functions ``Now``, ``Rand``, ``SinceSecond``, ``UnixSecond``,
``Quantity`` (pkg/utils/cel/default.go, funcs.go) — every function with an argument is also a
method — plus ``Usage`` / ``CumulativeUsage`` / ``StartedContainersTotal`` methods bound to
the usage callbacks, and the ``Quantity`` / ``ResourceList`` types (pkg/utils/cel/quantity.go,
resource_list.go).  Results become float64 through ``AsFloat64`` (environment.go:117-138).

This module parses that language (the CEL grammar: ?:, ||, &&, relations incl. ``in``,
+ -, * / %, unary ! -, member / index / call, literals, lists, maps) and evaluates it with
CEL's typing rules (no implicit int <-> double arithmetic, int64 overflow is an error,
heterogeneous numeric equality, error-absorbing && / ||).  Two uses:

* ``evaluate(expr, data)`` — the host evaluation of an expression for one (node, pod,
  container) binding (the value of a ResourceUsage expression for a pod, constant folding);
* ``lower(expr)`` — the device form of a Metric value: a postfix program over the per-series
  quantities the engine keeps (usage, cumulative usage, creation times, the scrape's now) that
  ``metrics_kernel`` evaluates for every series of a scrape (engine.hip).  Sub-expressions that
  do not depend on the series fold to constants on the host.

Quantities are modelled as apimachinery's int64Amount (unscaled integer x 10^scale), with
AsApproximateFloat64, ScaledValue(Nano) and kwok's Quantity x double rule
(newQuantityFromFloat64: int64(v * 10e9) nano — the x10 quirk evaluator_test.go:95-117 pins at 18).
"""
from __future__ import annotations

import datetime as _dt
import math
import re
from dataclasses import dataclass
from typing import Any, Callable, Dict, List, Optional, Tuple

from . import quantity as Q

INT64_MIN, INT64_MAX = -(1 << 63), (1 << 63) - 1
UINT64_MAX = (1 << 64) - 1


class CELError(Exception):
    """An evaluation error (CEL error value): the metric / usage evaluation fails."""


class CELSyntaxError(ValueError):
    pass


# ------------------------------------------------------------------ values
class UInt(int):
    """CEL uint (Python int subclass to keep it apart from int)."""


@dataclass(frozen=True)
class Timestamp:
    ns: int  # unix nanoseconds

    def unix_second(self) -> float:  # funcs.go unixSecond: float64(t.UnixNano()) / float64(time.Second)
        return float(wrap_int64(self.ns)) / 1e9  # UnixNano wraps outside int64 (e.g. the zero time)


GO_ZERO_TIME = Timestamp(-62135596800 * 10**9)  # time.Time{} (0001-01-01T00:00:00Z)


def wrap_int64(v: int) -> int:
    return ((v + (1 << 63)) % (1 << 64)) - (1 << 63)


def clamp_int64(v: int) -> int:
    return max(INT64_MIN, min(INT64_MAX, v))


@dataclass(frozen=True)
class Duration:
    ns: int


class Quantity:
    """resource.Quantity as int64Amount {value, scale} (exact Python ints)."""
    __slots__ = ("value", "scale")

    def __init__(self, value: int, scale: int):
        self.value, self.scale = int(value), int(scale)

    @staticmethod
    def parse(s: str) -> "Quantity":
        try:
            Q.parse_quantity_f64(s)  # the apimachinery grammar / errors
        except Q.QuantityError as e:
            raise CELError(f"Quantity({s!r}): {e}")
        return Quantity._exact(s)

    @staticmethod
    def _exact(s: str) -> "Quantity":
        m = re.fullmatch(r"([+-]?)(\d*)(?:\.(\d*))?(.*)", s)
        sign, num, frac, suf = m.group(1), m.group(2) or "0", m.group(3) or "", m.group(4)
        base, exp, _fmt = Q._interpret(suf)
        v = int((num + frac) or "0")
        if sign == "-":
            v = -v
        if base == 10:
            q = Quantity(v, exp - len(frac))
        else:
            from fractions import Fraction
            x = Fraction(v, 10 ** len(frac)) * (1 << exp)
            if x.denominator == 1:
                q = Quantity(int(x), 0)
            else:  # rounded up to nano like the inf.Dec path
                n = x * 10**9
                q = Quantity(-((-n.numerator) // n.denominator), -9)
        if q.scale < -9:  # ParseQuantity rounds below nano up to nano
            d = 10 ** (-9 - q.scale)
            q = Quantity(-((-q.value) // d), -9)
        return q

    @staticmethod
    def nano(v: int) -> "Quantity":  # NewScaledQuantity(v, Nano)
        return Quantity(v, -9)

    def scaled_nano(self) -> int:  # ScaledValue(Nano): ceil(q / 1e-9)
        if self.scale >= -9:
            return self.value * 10 ** (self.scale + 9)
        d = 10 ** (-9 - self.scale)
        return -((-self.value) // d)

    def approx(self) -> float:  # AsApproximateFloat64
        if self.scale == 0:
            return float(self.value)
        return float(self.value) * Q.go_pow10(self.scale)

    def _aligned(self, o: "Quantity"):
        s = min(self.scale, o.scale)
        return self.value * 10 ** (self.scale - s), o.value * 10 ** (o.scale - s), s

    def add(self, o):
        a, b, s = self._aligned(o)
        return Quantity(a + b, s)

    def sub(self, o):
        a, b, s = self._aligned(o)
        return Quantity(a - b, s)

    def cmp(self, o) -> int:
        a, b, _ = self._aligned(o)
        return (a > b) - (a < b)

    def __eq__(self, o):
        return isinstance(o, Quantity) and self.cmp(o) == 0

    def __hash__(self):
        return hash(self.approx())

    def __repr__(self):
        return f"Quantity({self.value}e{self.scale})"


def _from_float(v: float) -> Quantity:
    """newQuantityFromFloat64 (quantity.go:69-72): int64(v * 10e9) nano."""
    x = v * 10e9
    if not (-9.223372036854776e18 <= x < 9.223372036854776e18) or x != x:
        return Quantity.nano(INT64_MIN)  # amd64 float->int64 of an out-of-range value
    return Quantity.nano(int(x))


class ResourceList:
    """corev1.ResourceList as the CEL ResourceList type: index of a missing key is a zero
    Quantity (resource_list.go Get)."""

    def __init__(self, d):
        self.d = d or {}

    def get(self, k):
        if not isinstance(k, str):
            raise CELError("no such overload: ResourceList index")
        if k not in self.d:
            return Quantity.nano(0)
        return Quantity.parse(str(self.d[k]))

    def contains(self, k):
        return k in self.d

    def size(self):
        return len(self.d)


class Obj:
    """A typed Kubernetes object (Node / Pod / Container / ObjectMeta / ...) over its JSON:
    unset fields read as the Go zero value of their type, as easycel's struct access does."""

    # field -> type of the Go struct field (only what the types in cel.DefaultTypes expose that
    # kwok's expressions use; anything else reads the JSON as is)
    SCHEMA: Dict[str, Dict[str, str]] = {
        "Node": {"metadata": "ObjectMeta", "spec": "NodeSpec", "status": "NodeStatus"},
        "Pod": {"metadata": "ObjectMeta", "spec": "PodSpec", "status": "PodStatus"},
        "ObjectMeta": {"name": "string", "namespace": "string", "uid": "string", "resourceVersion": "string",
                       "generateName": "string", "labels": "map", "annotations": "map",
                       "creationTimestamp": "time", "deletionTimestamp": "ptrtime"},
        "NodeSpec": {"podCIDR": "string", "providerID": "string", "unschedulable": "bool"},
        "NodeStatus": {"allocatable": "rlist", "capacity": "rlist", "phase": "string"},
        "PodSpec": {"containers": "list:Container", "initContainers": "list:Container", "nodeName": "string",
                    "hostNetwork": "bool", "schedulerName": "string", "priority": "ptrint"},
        "PodStatus": {"phase": "string", "podIP": "string", "hostIP": "string", "startTime": "ptrtime"},
        "Container": {"name": "string", "image": "string", "resources": "ResourceRequirements"},
        "ResourceRequirements": {"requests": "rlist", "limits": "rlist"},
    }

    def __init__(self, typ: str, data):
        self.typ, self.data = typ, data if isinstance(data, dict) else {}

    def field(self, name: str):
        sch = self.SCHEMA.get(self.typ, {})
        t = sch.get(name)
        v = self.data.get(name)
        if t is None:
            if name not in self.data:
                raise CELError(f"no such field {name!r} on {self.typ}")
            return from_json(v)
        return _typed(t, v)

    def has(self, name: str) -> bool:
        return self.data.get(name) not in (None, "", [], {})


def _typed(t: str, v):
    if t == "string":
        return v if isinstance(v, str) else ""
    if t == "bool":
        return bool(v) if isinstance(v, bool) else False
    if t == "map":
        return dict(v) if isinstance(v, dict) else {}
    if t == "rlist":
        return ResourceList(v if isinstance(v, dict) else {})
    if t in ("time", "ptrtime"):
        if not v:
            return GO_ZERO_TIME  # metav1.Time{} / nil -> types.Timestamp{}
        return Timestamp(_parse_time(v))
    if t == "ptrint":
        return int(v) if isinstance(v, int) and not isinstance(v, bool) else 0
    if t.startswith("list:"):
        return [Obj(t[5:], x) for x in (v or [])]
    return Obj(t, v or {})


def _parse_time(s: str) -> int:
    m = re.fullmatch(r"(\d{4})-(\d{2})-(\d{2})T(\d{2}):(\d{2}):(\d{2})(?:\.(\d+))?(Z|[+-]\d{2}:\d{2})", s)
    if not m:
        raise CELError(f"bad timestamp {s!r}")
    y, mo, d, h, mi, se = (int(m.group(i)) for i in range(1, 7))
    frac = (m.group(7) or "")[:9].ljust(9, "0")
    off = 0
    if m.group(8) != "Z":
        sg = 1 if m.group(8)[0] == "+" else -1
        off = sg * (int(m.group(8)[1:3]) * 3600 + int(m.group(8)[4:6]) * 60)
    secs = int((_dt.datetime(y, mo, d, h, mi, se) - _dt.datetime(1970, 1, 1)).total_seconds()) - off
    return secs * 10**9 + int(frac)


def from_json(v):
    if isinstance(v, bool) or v is None or isinstance(v, str):
        return v
    if isinstance(v, int):
        return v
    if isinstance(v, float):
        return v
    if isinstance(v, list):
        return [from_json(x) for x in v]
    if isinstance(v, dict):
        return {k: from_json(x) for k, x in v.items()}
    return v


def type_name(v) -> str:
    if isinstance(v, bool):
        return "bool"
    if isinstance(v, UInt):
        return "uint"
    if isinstance(v, int):
        return "int"
    if isinstance(v, float):
        return "double"
    if isinstance(v, str):
        return "string"
    if v is None:
        return "null_type"
    if isinstance(v, Quantity):
        return "kubernetes.Quantity"
    if isinstance(v, ResourceList):
        return "kubernetes.ResourceList"
    if isinstance(v, Timestamp):
        return "google.protobuf.Timestamp"
    if isinstance(v, Duration):
        return "google.protobuf.Duration"
    if isinstance(v, list):
        return "list"
    if isinstance(v, dict):
        return "map"
    if isinstance(v, Obj):
        return v.typ
    return type(v).__name__


# ------------------------------------------------------------------ lexer / parser
_TOK = re.compile(r"""
  (?P<ws>\s+)
 |(?P<float>(?:\d+\.\d*|\.\d+)(?:[eE][+-]?\d+)?|\d+[eE][+-]?\d+)
 |(?P<hex>0[xX][0-9a-fA-F]+[uU]?)
 |(?P<int>\d+[uU]?)
 |(?P<str>[rR]?(?:"(?:[^"\\\n]|\\.)*"|'(?:[^'\\\n]|\\.)*'))
 |(?P<op>==|!=|<=|>=|&&|\|\||[-+*/%!<>?:.,\[\](){}])
 |(?P<ident>[A-Za-z_][A-Za-z0-9_]*)
""", re.X)


def _lex(src: str):
    out, i = [], 0
    while i < len(src):
        m = _TOK.match(src, i)
        if not m:
            raise CELSyntaxError(f"unexpected character {src[i]!r} at {i}")
        i = m.end()
        k = m.lastgroup
        if k == "ws":
            continue
        out.append((k, m.group(k)))
    out.append(("eof", ""))
    return out


def _unescape(tok: str) -> str:
    raw = tok[0] in "rR"
    body = tok[2:-1] if raw else tok[1:-1]
    if raw:
        return body
    out, i = [], 0
    esc = {"n": "\n", "t": "\t", "r": "\r", "\\": "\\", '"': '"', "'": "'", "a": "\a", "b": "\b", "f": "\f", "v": "\v",
           "`": "`", "?": "?"}
    while i < len(body):
        c = body[i]
        if c != "\\":
            out.append(c)
            i += 1
            continue
        n = body[i + 1]
        if n in esc:
            out.append(esc[n])
            i += 2
        elif n in "xX":
            out.append(chr(int(body[i + 2:i + 4], 16)))
            i += 4
        elif n == "u":
            out.append(chr(int(body[i + 2:i + 6], 16)))
            i += 6
        elif n == "U":
            out.append(chr(int(body[i + 2:i + 10], 16)))
            i += 10
        else:
            out.append(chr(int(body[i + 1:i + 4], 8)))
            i += 4
    return "".join(out)


# AST nodes: tuples (kind, ...)
#   ("lit", value) ("ident", name) ("select", expr, field) ("index", expr, idx)
#   ("call", name, [args]) ("method", target, name, [args]) ("unary", op, expr)
#   ("binary", op, l, r) ("cond", c, a, b) ("list", [..]) ("map", [(k, v)..])
class _Parser:
    def __init__(self, src):
        self.t = _lex(src)
        self.i = 0

    def peek(self, v=None):
        k, s = self.t[self.i]
        return s if v is None else (s == v and k in ("op", "ident"))

    def eat(self, v=None):
        k, s = self.t[self.i]
        if v is not None and s != v:
            raise CELSyntaxError(f"expected {v!r}, got {s!r}")
        self.i += 1
        return k, s

    def parse(self):
        e = self.expr()
        if self.t[self.i][0] != "eof":
            raise CELSyntaxError(f"unexpected {self.t[self.i][1]!r}")
        return e

    def expr(self):
        c = self.or_()
        if self.peek("?"):
            self.eat("?")
            a = self.or_()
            self.eat(":")
            b = self.expr()
            return ("cond", c, a, b)
        return c

    def or_(self):
        e = self.and_()
        while self.peek("||"):
            self.eat()
            e = ("binary", "||", e, self.and_())
        return e

    def and_(self):
        e = self.rel()
        while self.peek("&&"):
            self.eat()
            e = ("binary", "&&", e, self.rel())
        return e

    def rel(self):
        e = self.add()
        while self.peek() in ("==", "!=", "<", "<=", ">", ">=", "in") and self.t[self.i][0] in ("op", "ident"):
            op = self.eat()[1]
            e = ("binary", op, e, self.add())
        return e

    def add(self):
        e = self.mul()
        while self.peek() in ("+", "-") and self.t[self.i][0] == "op":
            op = self.eat()[1]
            e = ("binary", op, e, self.mul())
        return e

    def mul(self):
        e = self.unary()
        while self.peek() in ("*", "/", "%") and self.t[self.i][0] == "op":
            op = self.eat()[1]
            e = ("binary", op, e, self.unary())
        return e

    def unary(self):
        if self.peek() in ("!", "-") and self.t[self.i][0] == "op":
            op = self.eat()[1]
            # negative numeric literals fold (CEL lexes -9223372036854775808 as one literal)
            k, s = self.t[self.i]
            if op == "-" and k in ("int", "float", "hex") and not self._postfix_follows():
                self.eat()
                v = self._number(k, s, neg=True)
                return ("lit", v)
            return ("unary", op, self.unary())
        return self.member()

    def _postfix_follows(self):
        return self.t[self.i + 1][1] in (".", "[") and self.t[self.i + 1][0] == "op"

    def _number(self, k, s, neg=False):
        if k == "float":
            return -float(s) if neg else float(s)
        u = s[-1] in "uU"
        body = s[:-1] if u else s
        v = int(body, 16) if k == "hex" else int(body)
        if u:
            if neg or v > UINT64_MAX:
                raise CELSyntaxError("uint literal out of range")
            return UInt(v)
        v = -v if neg else v
        if not (INT64_MIN <= v <= INT64_MAX):
            raise CELSyntaxError("int literal out of range")
        return v

    def member(self):
        e = self.primary()
        while True:
            if self.peek(".") and self.t[self.i][0] == "op":
                self.eat()
                name = self.eat()[1]
                if self.peek("(") and self.t[self.i][0] == "op":
                    e = ("method", e, name, self.args())
                else:
                    e = ("select", e, name)
            elif self.peek("[") and self.t[self.i][0] == "op":
                self.eat()
                idx = self.expr()
                self.eat("]")
                e = ("index", e, idx)
            else:
                return e

    def args(self):
        self.eat("(")
        out = []
        if not self.peek(")"):
            out.append(self.expr())
            while self.peek(","):
                self.eat()
                out.append(self.expr())
        self.eat(")")
        return out

    def primary(self):
        k, s = self.t[self.i]
        if k in ("int", "float", "hex"):
            self.eat()
            return ("lit", self._number(k, s))
        if k == "str":
            self.eat()
            return ("lit", _unescape(s))
        if k == "ident":
            self.eat()
            if s == "true":
                return ("lit", True)
            if s == "false":
                return ("lit", False)
            if s == "null":
                return ("lit", None)
            if self.peek("(") and self.t[self.i][0] == "op":
                return ("call", s, self.args())
            return ("ident", s)
        if s == "(":
            self.eat()
            e = self.expr()
            self.eat(")")
            return e
        if s == "[":
            self.eat()
            items = []
            if not self.peek("]"):
                items.append(self.expr())
                while self.peek(","):
                    self.eat()
                    if self.peek("]"):
                        break
                    items.append(self.expr())
            self.eat("]")
            return ("list", items)
        if s == "{":
            self.eat()
            items = []
            if not self.peek("}"):
                while True:
                    key = self.expr()
                    self.eat(":")
                    items.append((key, self.expr()))
                    if not self.peek(","):
                        break
                    self.eat()
                    if self.peek("}"):
                        break
            self.eat("}")
            return ("map", items)
        raise CELSyntaxError(f"unexpected {s!r}")


def parse(src: str):
    return _Parser(src).parse()


# ------------------------------------------------------------------ evaluation
@dataclass
class Env:
    """What the evaluation sees besides the variables: the metrics environment's callbacks
    (evaluator.go:35-48) and clock.  Callbacks take the same arguments as the reference's."""
    now_ns: Optional[int] = None
    started_containers_total: Optional[Callable[[str], int]] = None
    container_usage: Optional[Callable[[str, str, str, str], float]] = None
    pod_usage: Optional[Callable[[str, str, str], float]] = None
    node_usage: Optional[Callable[[str, str], float]] = None
    container_cumulative: Optional[Callable[[str, str, str, str], float]] = None
    pod_cumulative: Optional[Callable[[str, str, str], float]] = None
    node_cumulative: Optional[Callable[[str, str], float]] = None
    rand: Optional[Callable[[], float]] = None


def _checked_int(v):
    if not (INT64_MIN <= v <= INT64_MAX):
        raise CELError("integer overflow")
    return v


def _checked_uint(v):
    if not (0 <= v <= UINT64_MAX):
        raise CELError("unsigned integer overflow")
    return UInt(v)


def _is_int(v):
    return isinstance(v, int) and not isinstance(v, (bool, UInt))


def _num_eq(a, b):
    """Heterogeneous numeric equality (cel-go >= 0.10 default)."""
    nums = (int, float)
    if isinstance(a, bool) or isinstance(b, bool):
        return type(a) is type(b) and a == b
    if isinstance(a, nums) and isinstance(b, nums):
        return float(a) == float(b) if (isinstance(a, float) or isinstance(b, float)) else int(a) == int(b)
    if isinstance(a, Quantity) or isinstance(b, Quantity):
        if isinstance(a, Quantity) and isinstance(b, Quantity):
            return a.cmp(b) == 0
        raise CELError("no such overload: ==")
    if type_name(a) != type_name(b):
        return False
    return a == b


def _arith(op, a, b):
    if isinstance(a, Quantity):
        if op in ("+", "-"):
            if not isinstance(b, Quantity):
                raise CELError(f"no such overload: Quantity {op} {type_name(b)}")
            return a.add(b) if op == "+" else a.sub(b)
        if op in ("*", "/"):  # quantity.go Multiply / Divide
            if isinstance(b, bool):
                raise CELError("no such overload")
            if isinstance(b, int):  # int or uint: nano arithmetic (Go int64 wrap-around)
                n = a.scaled_nano()
                if op == "*":
                    r = ((n * int(b) + (1 << 63)) % (1 << 64)) - (1 << 63)
                else:
                    if int(b) == 0:
                        raise CELError("integer divide by zero")
                    q = abs(n) // abs(int(b))
                    r = q if (n >= 0) == (int(b) >= 0) else -q
                return Quantity.nano(r)
            if isinstance(b, float):
                return _from_float(a.approx() * b if op == "*" else a.approx() / b)
        raise CELError(f"no such overload: Quantity {op} {type_name(b)}")
    if isinstance(a, bool) or isinstance(b, bool):
        raise CELError(f"no such overload: {type_name(a)} {op} {type_name(b)}")
    if type_name(a) != type_name(b):
        if isinstance(a, Timestamp) and isinstance(b, Duration):
            return Timestamp(a.ns + b.ns if op == "+" else a.ns - b.ns)
        if isinstance(a, Duration) and isinstance(b, Timestamp) and op == "+":
            return Timestamp(a.ns + b.ns)
        raise CELError(f"no such overload: {type_name(a)} {op} {type_name(b)}")
    if isinstance(a, float):
        if op == "+":
            return a + b
        if op == "-":
            return a - b
        if op == "*":
            return a * b
        if op == "/":
            if b == 0.0:
                return math.copysign(math.inf, a) * math.copysign(1.0, b) if a != 0 and a == a else math.nan
            return a / b
        raise CELError("no such overload: double %")
    if isinstance(a, UInt):
        if op == "+":
            return _checked_uint(a + b)
        if op == "-":
            return _checked_uint(a - b)
        if op == "*":
            return _checked_uint(a * b)
        if b == 0:
            raise CELError("divide by zero" if op == "/" else "modulus by zero")
        return UInt(a // b if op == "/" else a % b)
    if isinstance(a, int):
        if op == "+":
            return _checked_int(a + b)
        if op == "-":
            return _checked_int(a - b)
        if op == "*":
            return _checked_int(a * b)
        if b == 0:
            raise CELError("divide by zero" if op == "/" else "modulus by zero")
        if op == "/":
            if a == INT64_MIN and b == -1:
                raise CELError("integer overflow")
            q = abs(a) // abs(b)
            return q if (a >= 0) == (b >= 0) else -q
        r = abs(a) % abs(b)
        return r if a >= 0 else -r
    if isinstance(a, str) and op == "+":
        return a + b
    if isinstance(a, list) and op == "+":
        return a + b
    if isinstance(a, Timestamp) and op == "-":
        return Duration(a.ns - b.ns)
    if isinstance(a, Duration) and op in ("+", "-"):
        return Duration(a.ns + b.ns if op == "+" else a.ns - b.ns)
    raise CELError(f"no such overload: {type_name(a)} {op} {type_name(b)}")


def _order(op, a, b):
    if isinstance(a, Quantity) and isinstance(b, Quantity):
        c = a.cmp(b)
    elif type_name(a) == type_name(b) and isinstance(a, (int, float, str, Timestamp, Duration)) and not isinstance(a, bool):
        ka = a.ns if isinstance(a, (Timestamp, Duration)) else a
        kb = b.ns if isinstance(b, (Timestamp, Duration)) else b
        c = (ka > kb) - (ka < kb)
    elif isinstance(a, bool) and isinstance(b, bool):
        c = (a > b) - (a < b)
    else:
        raise CELError(f"no such overload: {type_name(a)} {op} {type_name(b)}")
    return {"<": c < 0, "<=": c <= 0, ">": c > 0, ">=": c >= 0}[op]


class Evaluator:
    def __init__(self, env: Env, vars: Dict[str, Any]):
        self.env, self.vars = env, vars

    def ev(self, n):
        k = n[0]
        if k == "lit":
            return n[1]
        if k == "ident":
            if n[1] not in self.vars:
                raise CELError(f"undeclared reference to {n[1]!r}")
            return self.vars[n[1]]
        if k == "select":
            return self._select(self.ev(n[1]), n[2])
        if k == "index":
            return self._index(self.ev(n[1]), self.ev(n[2]))
        if k == "cond":
            c = self.ev(n[1])
            if not isinstance(c, bool):
                raise CELError("no such overload: ternary condition")
            return self.ev(n[2]) if c else self.ev(n[3])
        if k == "unary":
            v = self.ev(n[2])
            if n[1] == "!":
                if not isinstance(v, bool):
                    raise CELError("no such overload: !")
                return not v
            if isinstance(v, Quantity):
                return Quantity(-v.value, v.scale)
            if isinstance(v, bool) or isinstance(v, UInt) or not isinstance(v, (int, float)):
                raise CELError(f"no such overload: -{type_name(v)}")
            return _checked_int(-v) if isinstance(v, int) else -v
        if k == "binary":
            return self._binary(n)
        if k == "list":
            return [self.ev(x) for x in n[1]]
        if k == "map":
            return {self.ev(a): self.ev(b) for a, b in n[1]}
        if k == "call":
            return self._call(n[1], None, [self.ev(a) for a in n[2]])
        if k == "method":
            return self._call(n[2], self.ev(n[1]), [self.ev(a) for a in n[3]])
        raise CELError(f"bad node {k}")

    def _binary(self, n):
        op = n[1]
        if op in ("&&", "||"):  # commutative error absorption
            err = None
            vals = []
            for side in (n[2], n[3]):
                try:
                    v = self.ev(side)
                    if not isinstance(v, bool):
                        raise CELError(f"no such overload: {op}")
                except CELError as e:
                    err = e
                    continue
                if op == "&&" and v is False:
                    return False
                if op == "||" and v is True:
                    return True
                vals.append(v)
            if err is not None:
                raise err
            return op == "&&"
        a, b = self.ev(n[2]), self.ev(n[3])
        if op == "==":
            return _num_eq(a, b)
        if op == "!=":
            return not _num_eq(a, b)
        if op in ("<", "<=", ">", ">="):
            return _order(op, a, b)
        if op == "in":
            if isinstance(b, dict):
                return a in b
            if isinstance(b, ResourceList):
                return b.contains(a)
            if isinstance(b, list):
                return any(_num_eq(a, x) for x in b if type_name(x) == type_name(a) or
                           (isinstance(x, (int, float)) and isinstance(a, (int, float))))
            raise CELError("no such overload: in")
        return _arith(op, a, b)

    @staticmethod
    def _select(v, f):
        if isinstance(v, Obj):
            return v.field(f)
        if isinstance(v, dict):
            if f not in v:
                raise CELError(f"no such key: {f}")
            return v[f]
        raise CELError(f"type {type_name(v)} has no field {f!r}")

    @staticmethod
    def _index(v, i):
        if isinstance(v, ResourceList):
            return v.get(i)
        if isinstance(v, dict):
            if i not in v:
                raise CELError(f"no such key: {i}")
            return v[i]
        if isinstance(v, list):
            if isinstance(i, bool) or not isinstance(i, (int, float)) or (isinstance(i, float) and i != int(i)):
                raise CELError("invalid list index")
            i = int(i)
            if not 0 <= i < len(v):
                raise CELError(f"index out of range: {i}")
            return v[i]
        raise CELError(f"no such overload: index {type_name(v)}")

    def _now(self):
        if self.env.now_ns is None:
            raise CELError("Now is not bound")
        return Timestamp(self.env.now_ns)

    def _call(self, name, target, args):
        """Functions of cel.DefaultFuncs / the metrics environment; with a target the method form
        (FuncsToMethods: every function with an argument is also a method on its first)."""
        full = ([target] if target is not None else []) + args
        t = [type_name(a) for a in full]
        E = self.env
        if name in ("Now", "now") and not full:
            return self._now()
        if name == "Rand" and not full:
            if E.rand is None:
                raise CELError("Rand is not bound")
            return E.rand()
        if name == "Quantity" and t == ["string"]:
            return Quantity.parse(full[0])
        if name == "UnixSecond" and t == ["google.protobuf.Timestamp"]:
            return full[0].unix_second()
        if name == "SinceSecond" and len(full) == 1 and isinstance(full[0], Obj) and full[0].typ in ("Node", "Pod"):
            # funcs.go sinceSecond: time.Since(creationTimestamp).Seconds(), against the scrape's now
            ct = full[0].field("metadata").field("creationTimestamp")
            return _dur_seconds(clamp_int64(self._now().ns - ct.ns))  # Time.Sub saturates
        if name in ("StartedContainersTotal", "startedContainersTotal") and E.started_containers_total is not None:
            if t == ["string"]:
                return int(E.started_containers_total(full[0]))
            if t == ["Node"]:
                return float(E.started_containers_total(full[0].field("metadata").field("name")))
        if name in ("Usage", "CumulativeUsage") and full and isinstance(full[0], Obj):
            cum = name == "CumulativeUsage"
            o = full[0]
            md = o.field("metadata")
            if o.typ == "Pod" and t[1:] == ["string", "string"]:
                f = E.container_cumulative if cum else E.container_usage
                if f is not None:
                    return float(f(full[1], md.field("namespace"), md.field("name"), full[2]))
            if o.typ == "Pod" and t[1:] == ["string"]:
                f = E.pod_cumulative if cum else E.pod_usage
                if f is not None:
                    return float(f(full[1], md.field("namespace"), md.field("name")))
            if o.typ == "Node" and t[1:] == ["string"]:
                f = E.node_cumulative if cum else E.node_usage
                if f is not None:
                    return float(f(full[1], md.field("name")))
        if target is None and len(full) == 1:  # standard conversions
            v = full[0]
            if name == "double":
                if isinstance(v, Quantity):
                    return v.approx()
                if isinstance(v, (int, float)) and not isinstance(v, bool):
                    return float(v)
                if isinstance(v, str):
                    try:
                        return float(v)
                    except ValueError:
                        raise CELError("double conversion error")
            if name == "int" and isinstance(v, (int, float)) and not isinstance(v, bool):
                if isinstance(v, float) and not (-9.223372036854776e18 < v < 9.223372036854776e18):
                    raise CELError("int conversion range error")
                return _checked_int(int(v))
            if name == "string":
                if isinstance(v, str):
                    return v
                if isinstance(v, bool):
                    return "true" if v else "false"
                if isinstance(v, int):
                    return str(int(v))
        if name == "size" and len(full) == 1:
            v = full[0]
            if isinstance(v, (str, list, dict)):
                return len(v)
            if isinstance(v, ResourceList):
                return v.size()
        raise CELError(f"found no matching overload for '{name}' applied to ({', '.join(t)})")


def _dur_seconds(ns: int) -> float:
    """time.Duration.Seconds()"""
    sec = int(ns / 10**9)
    return float(sec) + float(ns - sec * 10**9) / 1e9


def as_float64(v) -> float:
    """AsFloat64 (environment.go:117-138)."""
    if isinstance(v, Duration):
        return float(v.ns)
    if isinstance(v, bool):
        return 1.0 if v else 0.0
    if isinstance(v, (int, float)):
        return float(v)
    if isinstance(v, Quantity):
        return v.approx()
    raise CELError(f"unsupported type: {type_name(v)}")


_PROGRAMS: Dict[str, Any] = {}


def compile(src: str):
    """Parse once per expression text (cel.Environment.Compile caches programs by source,
    environment.go:98-114)."""
    p = _PROGRAMS.get(src)
    if p is None:
        p = _PROGRAMS[src] = parse(src)
    return p


def evaluate(src: str, node=None, pod=None, container=None, env: Optional[Env] = None):
    """Evaluate for one binding (JSON objects); raises CELError like the reference's error."""
    vars = {"node": Obj("Node", node or {}), "pod": Obj("Pod", pod or {}),
            "container": Obj("Container", container or {})}
    return Evaluator(env or Env(), vars).ev(compile(src))


def evaluate_float64(src: str, **kw) -> float:
    return as_float64(evaluate(src, **kw))


# ------------------------------------------------------------------ device lowering
# Postfix program for metrics_kernel (engine.hip): one f64 stack per series.
OP_CONST, OP_LOAD, OP_ADD, OP_SUB, OP_MUL, OP_DIV, OP_NEG = 1, 2, 3, 4, 5, 6, 7
# OP_LOAD operands: per-series inputs the engine has on the device
IN_NOW_S = 0            # Now().UnixSecond() of the scrape
IN_CONTAINER_CPU, IN_CONTAINER_MEM, IN_CONTAINER_CUM_CPU, IN_CONTAINER_CUM_MEM = 1, 2, 3, 4
IN_POD_CPU, IN_POD_MEM, IN_POD_CUM_CPU, IN_POD_CUM_MEM = 5, 6, 7, 8
IN_NODE_CPU, IN_NODE_MEM, IN_NODE_CUM_CPU, IN_NODE_CUM_MEM = 9, 10, 11, 12
IN_POD_SINCE, IN_NODE_SINCE = 13, 14       # SinceSecond(): now - creationTimestamp, seconds
IN_POD_CREATED, IN_NODE_CREATED = 15, 16   # creationTimestamp.UnixSecond()
IN_STARTED_CONTAINERS = 17                 # node.StartedContainersTotal() (double)
N_INPUTS = 18


class LowerError(ValueError):
    """The expression has no device form (it reads object fields the engine does not keep):
    the host evaluates it per series instead."""


_RES = {"cpu": 0, "memory": 1}


def lower(src: str, dimension: str) -> List[Tuple[int, float]]:
    """Metric value -> postfix program [(op, operand)] over double values.  Every sub-expression
    must be a double: usage / cumulative usage calls and SinceSecond / UnixSecond are doubles in
    the reference; literals fold to doubles only where CEL would compute a double (constant
    sub-expressions are folded exactly by the host evaluator, so int / Quantity arithmetic among
    constants keeps its CEL semantics)."""
    prog: List[Tuple[int, float]] = []
    ast = compile(src)

    def dyn(n) -> bool:  # depends on the series (a variable, the clock, a callback)
        if not isinstance(n, tuple):
            return False
        k = n[0]
        if k == "ident":
            return True
        if k == "lit":
            return False
        if k == "call" and n[1] in ("Now", "now", "Rand", "StartedContainersTotal", "startedContainersTotal"):
            return True
        for x in n[1:]:
            if isinstance(x, tuple) and dyn(x):
                return True
            if isinstance(x, list):
                for y in x:
                    if isinstance(y, tuple) and (dyn(y) if isinstance(y[0], str) else any(dyn(z) for z in y)):
                        return True
        return False

    def const(n):
        v = Evaluator(Env(), {}).ev(n)
        return v

    def emit(n) -> str:
        """-> static type of the value left on the stack ("double")."""
        if not dyn(n):
            v = const(n)
            if isinstance(v, float):
                prog.append((OP_CONST, v))
                return "double"
            if isinstance(v, (int, Quantity)) and not isinstance(v, bool):
                prog.append((OP_CONST, float(v) if isinstance(v, int) else v.approx()))
                return "int" if isinstance(v, int) else "quantity"
            raise LowerError(f"constant of type {type_name(v)}")
        k = n[0]
        if k == "method" and n[2] in ("Usage", "CumulativeUsage"):
            tgt, args = n[1], n[3]
            cum = n[2] == "CumulativeUsage"
            if tgt != ("ident", "pod") and tgt != ("ident", "node"):
                raise LowerError("Usage on something other than pod / node")
            if not args or args[0][0] != "lit" or args[0][1] not in _RES:
                raise LowerError("Usage resource must be a literal cpu / memory")
            r = _RES[args[0][1]]
            if tgt == ("ident", "node") and len(args) == 1:
                if dimension not in ("node", "pod", "container"):
                    raise LowerError(dimension)
                prog.append((OP_LOAD, (IN_NODE_CUM_CPU if cum else IN_NODE_CPU) + r))
            elif tgt == ("ident", "pod") and len(args) == 1:
                if dimension not in ("pod", "container"):
                    raise LowerError("pod usage needs the pod dimension")
                prog.append((OP_LOAD, (IN_POD_CUM_CPU if cum else IN_POD_CPU) + r))
            elif tgt == ("ident", "pod") and len(args) == 2 and args[1] == ("select", ("ident", "container"), "name"):
                if dimension != "container":
                    raise LowerError("container usage needs the container dimension")
                prog.append((OP_LOAD, (IN_CONTAINER_CUM_CPU if cum else IN_CONTAINER_CPU) + r))
            else:
                raise LowerError("unsupported Usage arguments")
            return "double"
        if k == "method" and n[2] == "SinceSecond" and not n[3] and n[1] in (("ident", "pod"), ("ident", "node")):
            prog.append((OP_LOAD, IN_POD_SINCE if n[1] == ("ident", "pod") else IN_NODE_SINCE))
            return "double"
        if k == "call" and n[1] == "SinceSecond" and len(n[2]) == 1 and n[2][0] in (("ident", "pod"), ("ident", "node")):
            prog.append((OP_LOAD, IN_POD_SINCE if n[2][0] == ("ident", "pod") else IN_NODE_SINCE))
            return "double"
        if k == "method" and n[2] in ("StartedContainersTotal", "startedContainersTotal") and n[1] == ("ident", "node") \
                and not n[3]:
            prog.append((OP_LOAD, IN_STARTED_CONTAINERS))
            return "double"
        if (k == "method" and n[2] == "UnixSecond" and not n[3]) or (k == "call" and n[1] == "UnixSecond" and len(n[2]) == 1):
            t = n[1] if k == "method" else n[2][0]
            if t in (("call", "Now", []), ("call", "now", [])):
                prog.append((OP_LOAD, IN_NOW_S))
                return "double"
            if t in (("select", ("select", ("ident", "pod"), "metadata"), "creationTimestamp"),
                     ("select", ("select", ("ident", "node"), "metadata"), "creationTimestamp")):
                prog.append((OP_LOAD, IN_POD_CREATED if t[1][1][1] == "pod" else IN_NODE_CREATED))
                return "double"
            raise LowerError("UnixSecond of an unsupported timestamp")
        if k == "unary" and n[1] == "-":
            if emit(n[2]) != "double":
                raise LowerError("negation of a non-double")
            prog.append((OP_NEG, 0.0))
            return "double"
        if k == "binary" and n[1] in ("+", "-", "*", "/"):
            ta = emit(n[2])
            tb = emit(n[3])
            if ta != "double" or tb != "double":  # CEL has no mixed int / double arithmetic
                raise LowerError(f"{ta} {n[1]} {tb}")
            prog.append(({"+": OP_ADD, "-": OP_SUB, "*": OP_MUL, "/": OP_DIV}[n[1]], 0.0))
            return "double"
        raise LowerError(f"no device form for {k}")

    if not dyn(ast):  # a constant value: AsFloat64 of it
        return [(OP_CONST, as_float64(const(ast)))]
    if emit(ast) != "double":
        raise LowerError("the value is not a double")
    return prog
