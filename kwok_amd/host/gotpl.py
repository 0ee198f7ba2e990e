"""Go text/template subset renderer for Stage ``next`` patches.

Host-side mirror of ``pkg/utils/gotpl`` (renderer.go:59-124, funcs.go:42-82): the Go
host renders the text patch of every *fired* object; this Python mirror is what the
stage compiler uses to derive the device's next-state delta ops (it renders each Stage's
template against shape prototypes, see ``compiler.derive_deltas``) and what the test
harness uses to apply next states.  It is pinned against the reference's rendered golden
outputs (kustomize/stage/**/testdata/*.output.yaml, copied under tests/golden/stages).

Supported: text / actions with ``{{-``/``-}}`` trimming and comments, pipelines with
``|``, variables (``$``, ``$x :=``, ``$x =``), field chains on dot / variables /
parenthesised pipelines, string/raw/number/bool/nil literals, ``if``/``else if``/
``else``/``range``/``with``/``end``, the text/template builtins ``and or not len index
print printf eq ne lt le gt ge``, and KWOK's default funcs (Quote, Now, StartTime, YAML,
Version, NodeConditions) plus caller-supplied funcs (NodeIP, PodIPWith, ...).
"""
from __future__ import annotations

import datetime as _dt
import json
import math
import re

import yaml


class TemplateError(Exception):
    pass


class _Missing:
    """An invalid reflect.Value (missing map key): prints "<no value>", is falsy."""

    def __repr__(self):
        return "<no value>"


MISSING = _Missing()


class Num(str):
    """json.Number (the renderer decodes with UseNumber, renderer.go:85-87)."""


def _to_go_data(v):
    if isinstance(v, bool) or v is None:
        return v
    if isinstance(v, (int, float)):
        return Num(json.dumps(v))
    if isinstance(v, str):
        return v
    if isinstance(v, list):
        return [_to_go_data(x) for x in v]
    if isinstance(v, dict):
        return {str(k): _to_go_data(x) for k, x in v.items()}
    return v


def _from_go_data(v):
    if isinstance(v, Num):
        return json.loads(str(v))
    if isinstance(v, list):
        return [_from_go_data(x) for x in v]
    if isinstance(v, dict):
        return {k: _from_go_data(x) for k, x in v.items()}
    if v is MISSING:
        return None
    return v


def truth(v) -> bool:
    if v is MISSING or v is None:
        return False
    if isinstance(v, bool):
        return v
    if isinstance(v, (str, list, dict)):
        return len(v) > 0
    if isinstance(v, (int, float)):
        return v != 0
    return True


def go_sprint(v) -> str:
    """fmt.Sprint of a template value (exec.go printValue)."""
    if v is MISSING:
        return "<no value>"
    if v is None:
        return "<nil>"
    if isinstance(v, bool):
        return "true" if v else "false"
    if isinstance(v, str):
        return str(v)
    if isinstance(v, list):
        return "[" + " ".join(go_sprint(x) for x in v) + "]"
    if isinstance(v, dict):
        return "map[" + " ".join(f"{k}:{go_sprint(v[k])}" for k in sorted(v)) + "]"
    return str(v)


def _go_gostring(v) -> str:
    """fmt %#v, as used by the stage tester's placeholder funcs (pkg/tools/stage/stage.go:172-193)."""
    if v is None or v is MISSING:
        return "<nil>"
    if isinstance(v, bool):
        return "true" if v else "false"
    if isinstance(v, Num):
        return json.dumps(str(v))
    if isinstance(v, str):
        return json.dumps(v, ensure_ascii=False)
    return go_sprint(v)


def go_json_string(s: str) -> str:
    """encoding/json string encoding with escapeHTML (encode.go appendString, Go 1.22)."""
    out = ['"']
    for ch in s:
        o = ord(ch)
        if ch == '"':
            out.append('\\"')
        elif ch == "\\":
            out.append("\\\\")
        elif ch == "\n":
            out.append("\\n")
        elif ch == "\r":
            out.append("\\r")
        elif ch == "\t":
            out.append("\\t")
        elif ch == "\b":
            out.append("\\b")
        elif ch == "\f":
            out.append("\\f")
        elif o < 0x20 or ch in "<>&" or o in (0x2028, 0x2029):
            out.append("\\u%04x" % o)
        else:
            out.append(ch)
    out.append('"')
    return "".join(out)


_REPR = re.compile(r"^(\d+)(?:\.(\d+))?(?:e([-+]\d+))?$")


def go_json_float(f: float) -> str:
    """encoding/json float64 (encode.go floatEncoder): shortest digits, 'f' format unless the
    magnitude is < 1e-6 or >= 1e21, then 'e' with "e-07" cleaned to "e-7"."""
    if math.isnan(f) or math.isinf(f):
        raise ValueError("json: unsupported value")
    if f == 0:
        return "-0" if math.copysign(1.0, f) < 0 else "0"
    a = abs(f)
    m = _REPR.match(repr(a))
    ip, fp, ex = m.group(1), m.group(2) or "", int(m.group(3) or 0)
    s, point = ip + fp, len(ip) + ex
    while s.startswith("0"):
        s, point = s[1:], point - 1
    s = s.rstrip("0") or "0"
    if a < 1e-6 or a >= 1e21:
        e = point - 1
        out = s[0] + ("." + s[1:] if len(s) > 1 else "") + "e" + ("-" if e < 0 else "+") + "%02d" % abs(e)
        if e < 0 and out[-2] == "0":
            out = out[:-2] + out[-1]
    elif point <= 0:
        out = "0." + "0" * (-point) + s
    elif point >= len(s):
        out = s + "0" * (point - len(s))
    else:
        out = s[:point] + "." + s[point:]
    return ("-" if f < 0 else "") + out


def go_json_bytes(v) -> str:
    """json.Marshal of a decoded YAML / JSON value: map keys sorted, Go string / float form."""
    if v is None or v is MISSING:
        return "null"
    if v is True:
        return "true"
    if v is False:
        return "false"
    if isinstance(v, Num):
        return str(v)
    if isinstance(v, int):
        return str(v)
    if isinstance(v, float):
        return go_json_float(v)
    if isinstance(v, str):
        return go_json_string(v)
    if isinstance(v, list):
        return "[" + ",".join(go_json_bytes(x) for x in v) + "]"
    if isinstance(v, dict):
        return "{" + ",".join(go_json_string(str(k)) + ":" + go_json_bytes(v[k]) for k in sorted(v, key=str)) + "}"
    raise TypeError(f"json: unsupported type {type(v).__name__}")


def go_json_marshal(v) -> str:
    """encoding/json Marshal of a template value (json.Number keeps its text, maps sorted)."""
    return go_json_bytes(v)


def quote(s) -> str:
    """funcs.go:43-55"""
    data = go_json_marshal(s)
    if not data:
        return '""'
    if data[0] == '"':
        return data
    return json.dumps(data)  # strconv.Quote of an ASCII JSON text


class _Dumper(yaml.SafeDumper):
    pass


def yaml_func(s, *indent) -> str:
    """funcs.go:62-74 (sigs.k8s.io/yaml Marshal: JSON round trip, sorted keys, block style)."""
    data = yaml.dump(_from_go_data(s), Dumper=_Dumper, default_flow_style=False, sort_keys=True,
                     allow_unicode=True)
    if len(indent) == 1 and int(str(indent[0])) > 0:
        pad = " " * (int(str(indent[0])) * 2)
        data = ("\n" + data).replace("\n", "\n" + pad)
    return data


NODE_CONDITIONS = [  # funcs.go:85-116 (k8s.io/api NodeCondition JSON, zero times are null)
    {"type": t, "status": s, "lastHeartbeatTime": None, "lastTransitionTime": None, "reason": r, "message": m}
    for t, s, r, m in [
        ("Ready", "True", "KubeletReady", "kubelet is posting ready status"),
        ("MemoryPressure", "False", "KubeletHasSufficientMemory", "kubelet has sufficient memory available"),
        ("DiskPressure", "False", "KubeletHasNoDiskPressure", "kubelet has no disk pressure"),
        ("PIDPressure", "False", "KubeletHasSufficientPID", "kubelet has sufficient PID available"),
        ("NetworkUnavailable", "False", "RouteCreated", "RouteController created a route"),
    ]
]


def rfc3339nano(ns: int) -> str:
    """time.Time.Format(time.RFC3339Nano) in UTC (trailing zeros of the fraction trimmed)."""
    sec, frac = divmod(int(ns), 10**9)
    t = _dt.datetime(1970, 1, 1) + _dt.timedelta(seconds=sec)
    s = t.strftime("%Y-%m-%dT%H:%M:%S")
    if frac:
        s += "." + f"{frac:09d}".rstrip("0")
    return s + "Z"


def default_funcs(now_ns: int = 0, version: str = "v0.6.0"):
    return {
        "Quote": quote,
        "Now": lambda: rfc3339nano(now_ns),
        "StartTime": lambda: rfc3339nano(now_ns),
        "YAML": yaml_func,
        "Version": lambda: version,
        "NodeConditions": lambda: _to_go_data(NODE_CONDITIONS),
    }


def placeholder_funcs():
    """The stage tester's wrapFunction placeholders (pkg/tools/stage/stage.go:128-151,172-193)."""

    def wrap(name):
        def f(*args):
            if not args:
                return f"<{name}>"
            return f"<{name}(" + ", ".join(_go_gostring(a) or '""' for a in args) + ")>"
        return f

    return {n: wrap(n) for n in ["NodeIP", "NodeName", "NodePort", "PodIP", "NodeIPWith", "PodIPWith", "Now", "now",
                                 "Version"]}


# ------------------------------------------------------------------------- lexer / parser
_ACTION = re.compile(r"\{\{(-\s)?(.*?)(\s-)?\}\}", re.S)
_TOKEN = re.compile(r"""
    (?P<ws>\s+)
  | (?P<str>"(?:[^"\\]|\\.)*")
  | (?P<raw>`[^`]*`)
  | (?P<num>-?\d+(?:\.\d+)?)
  | (?P<decl>:=)
  | (?P<assign>=)
  | (?P<pipe>\|)
  | (?P<lp>\()
  | (?P<rp>\))
  | (?P<comma>,)
  | (?P<var>\$[A-Za-z0-9_]*)
  | (?P<field>(?:\.[A-Za-z_][A-Za-z0-9_]*)+)
  | (?P<dot>\.)
  | (?P<ident>[A-Za-z_][A-Za-z0-9_]*)
""", re.X)


def _tokenize(src):
    out, i = [], 0
    while i < len(src):
        m = _TOKEN.match(src, i)
        if not m:
            raise TemplateError(f"bad token at {src[i:i + 20]!r}")
        i = m.end()
        kind = m.lastgroup
        if kind == "ws":
            continue
        text = m.group()
        # a field chain directly after a ')' / var belongs to that operand
        out.append((kind, text))
    return out


class _P:
    def __init__(self, toks):
        self.t, self.i = toks, 0

    def peek(self, k=0):
        return self.t[self.i + k] if self.i + k < len(self.t) else (None, None)

    def take(self):
        tok = self.peek()
        self.i += 1
        return tok

    def pipeline(self):
        decl = None
        # $a := / $a, $b := / $a =
        if self.peek()[0] == "var":
            if self.peek(1)[0] in ("decl", "assign"):
                decl = ([self.take()[1]], self.take()[0])
            elif self.peek(1)[0] == "comma" and self.peek(2)[0] == "var" and self.peek(3)[0] == "decl":
                v1 = self.take()[1]
                self.take()
                v2 = self.take()[1]
                self.take()
                decl = ([v1, v2], "decl")
        cmds = [self.command()]
        while self.peek()[0] == "pipe":
            self.take()
            cmds.append(self.command())
        return ("pipe", decl, cmds)

    def command(self):
        args = []
        while self.peek()[0] not in (None, "pipe", "rp"):
            args.append(self.operand())
        if not args:
            raise TemplateError("empty command")
        return args

    def operand(self):
        k, v = self.take()
        if k == "field":
            node = ("field", ("dot",), v[1:].split("."))
        elif k == "dot":
            node = ("dot",)
        elif k == "var":
            node = ("var", v)
            if self.peek()[0] == "field":
                node = ("field", node, self.take()[1][1:].split("."))
        elif k == "str":
            node = ("lit", json.loads(v))
        elif k == "raw":
            node = ("lit", v[1:-1])
        elif k == "num":
            node = ("lit", Num(v))
        elif k == "lp":
            p = self.pipeline()
            if self.take()[0] != "rp":
                raise TemplateError("missing )")
            node = ("paren", p)
            if self.peek()[0] == "field":
                node = ("field", node, self.take()[1][1:].split("."))
        elif k == "ident":
            if v in ("true", "false"):
                node = ("lit", v == "true")
            elif v == "nil":
                node = ("lit", None)
            else:
                node = ("ident", v)
        else:
            raise TemplateError(f"unexpected {k} {v!r}")
        return node


def _parse(text):
    """Split into a tree of ('text', s) / ('action', pipe) / ('if'|'range'|'with', pipe, body, else)."""
    items = []
    pos = 0
    for m in _ACTION.finditer(text):
        items.append(("text", text[pos:m.start()]))
        inner = m.group(2)
        items.append(("act", inner, bool(m.group(1)), bool(m.group(3))))
        pos = m.end()
    items.append(("text", text[pos:]))
    # whitespace trimming
    for idx, it in enumerate(items):
        if it[0] == "act":
            if it[2] and idx > 0 and items[idx - 1][0] == "text":
                items[idx - 1] = ("text", items[idx - 1][1].rstrip())
            if it[3] and idx + 1 < len(items) and items[idx + 1][0] == "text":
                items[idx + 1] = ("text", items[idx + 1][1].lstrip())

    def block(i, stop):
        nodes = []
        while i < len(items):
            it = items[i]
            if it[0] == "text":
                if it[1]:
                    nodes.append(("text", it[1]))
                i += 1
                continue
            src = it[1].strip()
            if src.startswith("/*"):
                i += 1
                continue
            word = src.split(None, 1)[0] if src else ""
            rest = src[len(word):].strip()
            if word in ("end", "else"):
                if word in stop:
                    return nodes, i, src
                raise TemplateError(f"unexpected {{{{{src}}}}}")
            if word in ("if", "range", "with"):
                n, i = control(word, rest, i + 1)
                nodes.append(n)
                continue
            nodes.append(("action", _P(_tokenize(src)).pipeline()))
            i += 1
        if stop:
            raise TemplateError("missing {{end}}")
        return nodes, i, None

    def control(word, rest, i):
        pipe = _P(_tokenize(rest)).pipeline()
        body, i, term = block(i, ("end", "else"))
        els = None
        if term.startswith("else"):
            rest2 = term[4:].strip()
            if rest2.startswith("if ") or rest2.startswith("with "):
                w2, r2 = rest2.split(None, 1)
                n2, i = control(w2, r2, i + 1)
                els = [n2]
                return (word, pipe, body, els), i
            els, i, term = block(i + 1, ("end",))
        return (word, pipe, body, els), i + 1

    nodes, _, _ = block(0, ())
    return nodes


# ----------------------------------------------------------------------------- evaluation
def _field(v, name):
    if v is MISSING:
        return MISSING
    if v is None:
        raise TemplateError(f"nil pointer evaluating interface {{}}.{name}")
    if isinstance(v, dict):
        return v.get(name, MISSING)
    raise TemplateError(f"can't evaluate field {name} in type {type(v).__name__}")


def _index(x, *keys):
    for k in keys:
        if x is MISSING or x is None:
            raise TemplateError("index of untyped nil")
        if isinstance(x, dict):
            x = x.get(go_sprint(k), None)  # missing key -> zero value (nil interface)
        elif isinstance(x, (list, str)):
            i = int(str(k))
            if i < 0 or i >= len(x):
                raise TemplateError(f"index out of range: {i}")
            x = x[i]
        else:
            raise TemplateError(f"can't index item of type {type(x).__name__}")
    return x


def _basic(v):
    if v is MISSING or v is None:
        return "invalid", None
    if isinstance(v, bool):
        return "bool", v
    if isinstance(v, Num):
        return "string", str(v)
    if isinstance(v, str):
        return "string", v
    if isinstance(v, (int, float)):
        return "num", v
    return "other", v


def _eq(a, *bs):
    ka, va = _basic(a)
    for b in bs:
        kb, vb = _basic(b)
        if ka != kb:
            if ka != "invalid" and kb != "invalid":
                raise TemplateError("incompatible types for comparison")
            continue
        if ka == "other":
            raise TemplateError("non-comparable type")
        if va == vb:
            return True
    return False


def _cmp(op):
    def f(a, b):
        ka, va = _basic(a)
        kb, vb = _basic(b)
        if ka != kb or ka in ("invalid", "other", "bool"):
            raise TemplateError("incompatible types for comparison")
        return {"lt": va < vb, "le": va <= vb, "gt": va > vb, "ge": va >= vb}[op]
    return f


def _printf(fmt, *args):
    args = list(args)

    def rep(m):
        verb = m.group(1)
        if verb == "%":
            return "%"
        a = args.pop(0) if args else MISSING
        if verb in ("s", "v", "d"):
            return go_sprint(a)
        if verb == "q":
            return json.dumps(go_sprint(a))
        raise TemplateError(f"printf verb %{verb}")

    return re.sub(r"%([%svdq])", rep, str(fmt))


def _sprig_dict(*kv):
    return {go_sprint(kv[i]): (kv[i + 1] if i + 1 < len(kv) else "") for i in range(0, len(kv), 2)}


def _sprig_default(d, v=MISSING):
    return v if truth(v) else d


_BUILTINS = {
    # a few sprig (github.com/Masterminds/sprig/v3 v3.2.3) helpers used by KWOK's stages
    "dict": _sprig_dict,
    "list": lambda *a: list(a),
    "default": _sprig_default,
    "hasKey": lambda d, k: isinstance(d, dict) and go_sprint(k) in d,
    "not": lambda a: not truth(a),
    "len": lambda a: Num(str(len(a))),
    "index": _index,
    "print": lambda *a: "".join(go_sprint(x) for x in a),
    "printf": _printf,
    "eq": _eq,
    "ne": lambda a, b: not _eq(a, b),
    "lt": _cmp("lt"), "le": _cmp("le"), "gt": _cmp("gt"), "ge": _cmp("ge"),
}


class Renderer:
    """gotpl.NewRenderer(funcMap) (renderer.go:50-57); ``to_json`` = Renderer.ToJSON."""

    def __init__(self, funcs=None, now_ns: int = 0):
        self.funcs = dict(default_funcs(now_ns))
        if funcs:
            self.funcs.update(funcs)
        self._cache = {}

    def _tree(self, text):
        text = text.strip()  # renderer.go:60
        t = self._cache.get(text)
        if t is None:
            t = self._cache[text] = _parse(text)
        return t

    def to_text(self, text, data) -> str:
        root = _to_go_data(json.loads(json.dumps(data)))
        out = []
        self._exec(self._tree(text), root, [{"$": root}], out)
        return "".join(out)

    def to_json(self, text, data):
        """Render then YAMLToJSON; returns the decoded JSON value."""
        return yaml.load(self.to_text(text, data), Loader=_YamlLoader)

    # -- exec
    def _exec(self, nodes, dot, scopes, out):
        for n in nodes:
            kind = n[0]
            if kind == "text":
                out.append(n[1])
            elif kind == "action":
                v = self._pipe(n[1], dot, scopes)
                if n[1][1] is None:
                    out.append(go_sprint(v))
            elif kind == "if":
                scopes.append({})
                v = self._pipe(n[1], dot, scopes)
                if truth(v):
                    self._exec(n[2], dot, scopes, out)
                elif n[3] is not None:
                    self._exec(n[3], dot, scopes, out)
                scopes.pop()
            elif kind == "with":
                scopes.append({})
                v = self._pipe(n[1], dot, scopes)
                if truth(v):
                    self._exec(n[2], v, scopes, out)
                elif n[3] is not None:
                    self._exec(n[3], dot, scopes, out)
                scopes.pop()
            elif kind == "range":
                scopes.append({})
                pipe = n[1]
                decl = pipe[1]
                v = self._pipe(("pipe", None, pipe[2]), dot, scopes)
                if v is None:
                    raise TemplateError("range can't iterate over <nil>")
                if v is MISSING:
                    items = []
                elif isinstance(v, list):
                    items = list(enumerate(v))
                elif isinstance(v, dict):
                    items = [(k, v[k]) for k in sorted(v)]
                elif isinstance(v, Num):
                    items = [(Num(str(i)), Num(str(i))) for i in range(int(v))]
                else:
                    raise TemplateError(f"range can't iterate over {go_sprint(v)}")
                if not items:
                    if n[3] is not None:
                        self._exec(n[3], dot, scopes, out)
                for k, e in items:
                    scopes.append({})
                    if decl:
                        names = decl[0]
                        if len(names) == 1:
                            scopes[-1][names[0]] = e
                        else:
                            scopes[-1][names[0]] = Num(str(k)) if isinstance(k, int) else k
                            scopes[-1][names[1]] = e
                    self._exec(n[2], e, scopes, out)
                    scopes.pop()
                scopes.pop()

    def _lookup(self, name, scopes):
        for s in reversed(scopes):
            if name in s:
                return s[name]
        raise TemplateError(f"undefined variable {name}")

    def _pipe(self, pipe, dot, scopes):
        _, decl, cmds = pipe
        val = None
        first = True
        for cmd in cmds:
            val = self._command(cmd, dot, scopes, None if first else val, not first)
            first = False
        if decl:
            names, how = decl
            if how == "decl":
                scopes[-1][names[0]] = val
            else:
                for s in reversed(scopes):
                    if names[0] in s:
                        s[names[0]] = val
                        break
                else:
                    raise TemplateError(f"undefined variable {names[0]}")
        return val

    def _arg(self, node, dot, scopes):
        k = node[0]
        if k == "lit":
            return node[1]
        if k == "dot":
            return dot
        if k == "var":
            return self._lookup(node[1], scopes)
        if k == "field":
            v = self._arg(node[1], dot, scopes)
            for name in node[2]:
                v = _field(v, name)
            return v
        if k == "paren":
            return self._pipe(node[1], dot, scopes)
        if k == "ident":
            return self._call(node[1], [], dot, scopes)
        raise TemplateError(f"bad operand {node}")

    def _call(self, name, argnodes, dot, scopes, extra=None):
        if name in ("and", "or"):
            nodes = list(argnodes)
            vals = [lambda n=n: self._arg(n, dot, scopes) for n in nodes]
            if extra is not None:
                vals.append(lambda: extra[0])
            v = None
            for get in vals:
                v = get()
                if (name == "or") == truth(v):
                    return v
            return v
        args = [self._arg(a, dot, scopes) for a in argnodes]
        if extra is not None:
            args.append(extra[0])
        fn = self.funcs.get(name) or _BUILTINS.get(name)
        if fn is None:
            raise TemplateError(f'function "{name}" not defined')
        return fn(*args)

    def _command(self, cmd, dot, scopes, prev, has_prev):
        head = cmd[0]
        extra = (prev,) if has_prev else None
        if head[0] == "ident" and head[1] not in ("true", "false", "nil"):
            return self._call(head[1], cmd[1:], dot, scopes, extra)
        if len(cmd) > 1 or has_prev:
            raise TemplateError("can't give argument to non-function")
        return self._arg(head, dot, scopes)


class _YamlLoader(yaml.SafeLoader):
    pass


# YAMLToJSON keeps unquoted timestamps as their text (go-yaml resolves them to time.Time and
# sigs.k8s.io/yaml marshals them back to RFC3339); drop PyYAML's datetime resolver.
_YamlLoader.yaml_implicit_resolvers = {
    k: [(tag, rx) for tag, rx in v if tag != "tag:yaml.org,2002:timestamp"]
    for k, v in yaml.SafeLoader.yaml_implicit_resolvers.items()
}
