"""Precompiled merge-patch byte templates.

Reference: the per-*fired*-object patch of playStage — ``Next.Patches`` (next.go:73-160:
computePatch / computeMergePatch / wrapMergePatchData) renders each Stage patch template
with text/template + sprig (gotpl/renderer.go:59-124: JSON round trip of the object,
template Execute, sigs.k8s.io/yaml.YAMLToJSON = YAML decode + encoding/json Marshal with
sorted keys and HTML escaping) and wraps it under the patch's root key.

Here a template is compiled ONCE into a byte program for libkwok_patch.so
(kwok_amd/csrc/patch.cpp, include/kwok_patch.h).  The YAML block structure is resolved at
compile time: a mapping becomes its keys' JSON bytes in Go's sorted order, a literal scalar
its final JSON bytes, ``key:`` followed by items that all come from ranges a lazily opened
array (``null`` when nothing renders).  Only the *slots* stay dynamic:

* ``{{ x | Quote }}`` — a JSON string (funcs.go:43-55 read back by YAML);
* ``{{ x }}`` as a plain scalar — the printed text resolved as YAML would (ints, words);
* ``'...{{ range }} {{ .name }} {{ end }}...'`` — single-quoted scalars with inline ranges;
* ``range`` / ``if`` / ``else if`` / ``else`` over sequence items and mapping entries,
  variables (``$x :=``, ``$i, $e := range``), and the template functions Now,
  NodeConditions, Version, or / and / not / eq / ne / index / dict / len / Quote, plus the
  controller's functions (NodeIPWith, PodIPWith, ...) as caller functions.

The native renderer parses each fired object's JSON once and writes its patch bytes.
Anything outside that subset is rejected at compile time (``PatchUnsupported``; the stage
keeps the host renderer and is listed in ``PatchProgram.unsupported``).  A value the byte
program cannot place exactly — a printed value YAML would re-type, characters YAML treats
specially, a template execution error — gives that one object the status NEEDS_RENDER and
the caller renders it with ``render_patch_bytes``: explicit and counted, never a silent
substitute.
"""
from __future__ import annotations

import ctypes as C
import json
import math
import os
import re
from typing import Callable, Dict, List, Optional, Sequence, Tuple

import numpy as np
import yaml

from . import abi, gotpl

LIB_PATH = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "lib", "libkwok_patch.so")
STATUS_OK, STATUS_NEEDS_RENDER = 0, 1

# functions with a fixed meaning (text/template builtins, sprig, gotpl/funcs.go:42-82)
_BUILTIN = {"or", "and", "not", "eq", "ne", "index", "dict", "len", "Quote", "Now"}


class PatchUnsupported(ValueError):
    pass


go_json_string, go_json_float, go_json_bytes = gotpl.go_json_string, gotpl.go_json_float, gotpl.go_json_bytes


def render_patch_bytes(template: str, root: str, obj: dict, renderer: gotpl.Renderer) -> bytes:
    """The host renderer's patch bytes (computeMergePatch + wrapMergePatchData, next.go:132-160)."""
    body = go_json_bytes(renderer.to_json(template, obj))
    return (body if not root else "{" + go_json_string(root) + ":" + body + "}").encode()


# ------------------------------------------------------------------ template -> line entries
_KEY = re.compile(r'^(?P<key>[A-Za-z0-9_][A-Za-z0-9_./-]*|"(?:[^"\\]|\\.)*"|\'(?:[^\']|\'\')*\')[ \t]*:(?=[ \t]|$)')


def _is_ws(pieces) -> bool:
    return all(p[0] == "t" and not p[1].strip() for p in pieces)


def _body_starts_line(nodes) -> bool:
    """A control action alone on its line: its body text starts with a line break."""
    for n in nodes:
        if n[0] == "text":
            head = n[1].split("\n", 1)
            return not head[0].strip() and len(head) > 1
        return False
    return True


def _entries(nodes) -> list:
    """One AST level -> [("line", indent, pieces) | ("block", kind, pipe, body, else) |
    ("assign", pipe)]; pieces: ("t", text) | ("v", pipe) | ("r", pipe, pieces) (inline range)."""
    out, cur = [], []

    def flush():
        content = [p for p in cur if p[0] != "t" or p[1].strip()]
        if not content:
            pass
        elif any(p[0] == "a" for p in content):
            if len(content) != 1:
                raise PatchUnsupported("an assignment shares its line with content")
            out.append(("assign", content[0][1]))
        else:
            text = cur[0][1] if cur[0][0] == "t" else ""
            out.append(("line", len(text) - len(text.lstrip(" ")), list(cur)))
        cur.clear()

    for n in nodes:
        k = n[0]
        if k == "text":
            parts = n[1].split("\n")
            for i, part in enumerate(parts):
                if part:
                    if cur and cur[-1][0] == "t":
                        cur[-1] = ("t", cur[-1][1] + part)
                    else:
                        cur.append(("t", part))
                if i < len(parts) - 1:
                    flush()
        elif k == "action":
            pipe = n[1]
            cur.append(("a", pipe) if pipe[1] is not None else ("v", pipe))
        elif k in ("if", "range", "with"):
            if _is_ws(cur) and _body_starts_line(n[2]):
                cur.clear()
                if k == "with":
                    raise PatchUnsupported("{{ with }}")
                if k == "range" and n[3] is not None:
                    raise PatchUnsupported("{{ range }} ... {{ else }}")
                out.append(("block", k, n[1], _entries(n[2]), _entries(n[3]) if n[3] is not None else []))
            else:
                if k != "range" or n[3] is not None:
                    raise PatchUnsupported(f"inline {{{{ {k} }}}}")
                cur.append(("r", n[1], _inline(n[2])))
        else:
            raise PatchUnsupported(f"template node {k}")
    flush()
    return out


def _inline(nodes) -> list:
    pieces = []
    for n in nodes:
        if n[0] == "text":
            if "\n" in n[1]:
                raise PatchUnsupported("inline range spanning lines")
            pieces.append(("t", n[1]))
        elif n[0] == "action" and n[1][1] is None:
            pieces.append(("v", n[1]))
        elif n[0] == "range" and n[3] is None:
            pieces.append(("r", n[1], _inline(n[2])))
        else:
            raise PatchUnsupported("inline construct")
    return pieces


def _first_line(entries):
    for e in entries:
        if e[0] == "line":
            return e
        if e[0] == "block":
            f = _first_line(e[3]) or _first_line(e[4])
            if f:
                return f
    return None


def _lead(line) -> str:
    return line[2][0][1][line[1]:] if line[2] and line[2][0][0] == "t" else ""


def _is_item(line) -> bool:
    s = _lead(line)
    return s.startswith("- ") or s == "-"


# ------------------------------------------------------------------ compiler
class _Scope:
    def __init__(self, parent=None):
        self.parent = parent
        self.vars: Dict[str, int] = {}

    def find(self, name):
        s = self
        while s is not None:
            if name in s.vars:
                return s.vars[name]
            s = s.parent
        raise PatchUnsupported(f"undefined variable {name}")


class TemplateCompiler:
    """One template -> {"n_vars", "n_regs", "exprs", "prologue", "head", "body", "tail"}.

    Program nodes (interpreted by patch.cpp):
      ["lit", bytes] | ["q", expr] | ["raw", expr] | ["sq", pieces]
      ["map", guards, entries]   guards: [expr, then_reg, else_reg, parent_reg] in template
                                 order; entries: [key_bytes, reg (-1 = always), node] sorted
      ["seq", items]             items: ["item", node] | ["range", expr, var_i, var_e, sets, items]
                                        | ["if", expr, items, else_items]
      sets: [var, expr]; sq pieces: ["t", text] | ["v", expr] | ["r", expr, var_i, var_e, pieces]
    """

    def __init__(self, funcs: Dict[str, int], const_ids: Dict[str, int]):
        self.funcs = funcs
        self.const_ids = const_ids
        self.exprs: List = []
        self.n_vars = 0
        self.n_regs = 0
        self.reg_parent: Dict[int, int] = {}
        self.reg_sibling: Dict[int, int] = {}

    # -- expressions
    def _expr(self, e) -> int:
        self.exprs.append(e)
        return len(self.exprs) - 1

    def _var(self) -> int:
        self.n_vars += 1
        return self.n_vars - 1

    def operand(self, node, scope):
        k = node[0]
        if k == "lit":
            v = node[1]
            if isinstance(v, gotpl.Num):
                if not re.fullmatch(r"-?(0|[1-9][0-9]*)", str(v)):
                    raise PatchUnsupported(f"number literal {v}")
                return {"k": "num", "v": str(v)}
            if v is None:
                return {"k": "nil"}
            if isinstance(v, bool):
                return {"k": "bool", "v": v}
            return {"k": "str", "v": v}
        if k == "dot":
            return {"k": "dot"}
        if k == "var":
            return {"k": "root"} if node[1] == "$" else {"k": "var", "i": scope.find(node[1])}
        if k == "field":
            return {"k": "field", "a": [self.operand(node[1], scope)], "p": list(node[2])}
        if k == "paren":
            return self.pipeline(node[1], scope)
        if k == "ident":
            return self.call(node[1], [], scope)
        raise PatchUnsupported(f"operand {k}")

    def call(self, name, args, scope, piped=None):
        a = [self.operand(x, scope) for x in args]
        if piped is not None:
            a.append(piped)
        if name in self.funcs:  # the controller's functions (may override Now / Version)
            return {"k": "ext", "f": self.funcs[name], "a": a}
        if name in self.const_ids:
            if a:
                raise PatchUnsupported(f"{name} with arguments")
            return {"k": "const", "i": self.const_ids[name]}
        if name in _BUILTIN:
            if (name in ("dict", "Now") and a) or (name in ("not", "len", "Quote") and len(a) != 1) or \
                    (name in ("eq", "ne", "index") and len(a) < 2) or (name in ("or", "and") and not a):
                raise PatchUnsupported(f"{name} with {len(a)} arguments")
            return {"k": name, "a": a}
        raise PatchUnsupported(f"function {name!r}")

    def pipeline(self, pipe, scope):
        val = None
        for cmd in pipe[2]:
            head = cmd[0]
            if head[0] == "ident" and head[1] not in ("true", "false", "nil"):
                val = self.call(head[1], cmd[1:], scope, val)
            else:
                if len(cmd) > 1 or val is not None:
                    raise PatchUnsupported("argument to a non-function")
                val = self.operand(head, scope)
        return val

    def slot(self, pipe, scope):
        if pipe[1] is not None:
            raise PatchUnsupported("assignment as a value")
        cmds = pipe[2]
        last = cmds[-1]
        if last[0] == ("ident", "Quote") and len(last) == 1 and len(cmds) > 1:
            return ["q", self._expr(self.pipeline(("pipe", None, cmds[:-1]), scope))]
        if last[0] == ("ident", "Quote") and len(last) == 2 and len(cmds) == 1:
            return ["q", self._expr(self.operand(last[1], scope))]
        return ["raw", self._expr(self.pipeline(pipe, scope))]

    def assign(self, pipe, scope, sets):
        names, how = pipe[1]
        if how != "decl" or len(names) != 1:
            raise PatchUnsupported("variable re-assignment")
        e = self.pipeline(("pipe", None, pipe[2]), scope)
        v = self._var()
        scope.vars[names[0]] = v
        sets.append([v, self._expr(e)])

    def range_vars(self, pipe, scope):
        if pipe[1] is None:
            return -1, -1
        names, how = pipe[1]
        if how != "decl":
            raise PatchUnsupported("range with '='")
        if len(names) == 1:
            ve = self._var()
            scope.vars[names[0]] = ve
            return -1, ve
        vi, ve = self._var(), self._var()
        scope.vars[names[0]], scope.vars[names[1]] = vi, ve
        return vi, ve

    # -- scalars
    def scalar(self, pieces, scope):
        """The scalar after `key:` / `- `, or None when the line ends there."""
        pieces = list(pieces)
        if pieces and pieces[0][0] == "t":
            pieces[0] = ("t", pieces[0][1].lstrip())
        if pieces and pieces[-1][0] == "t":
            pieces[-1] = ("t", pieces[-1][1].rstrip())
        pieces = [p for p in pieces if p[0] != "t" or p[1]]
        if not pieces:
            return None
        if all(p[0] == "t" for p in pieces):
            text = "".join(p[1] for p in pieces)
            if text.startswith("#") or " #" in text or "\t#" in text:
                raise PatchUnsupported("YAML comment")
            try:
                v = yaml.load("k: " + text, Loader=gotpl._YamlLoader)["k"]
            except yaml.YAMLError as e:
                raise PatchUnsupported(f"YAML literal {text!r}: {e}")
            return ["lit", go_json_bytes(v)]
        if len(pieces) == 1 and pieces[0][0] == "v":
            return self.slot(pieces[0][1], scope)
        first, last = pieces[0], pieces[-1]
        if len(pieces) > 1 and first[0] == "t" and last[0] == "t" and first[1].startswith("'") \
                and last[1].endswith("'") and len(first[1]) >= 1 and len(last[1]) >= 1:
            inner = [("t", first[1][1:])] + pieces[1:-1] + [("t", last[1][:-1])]
            return ["sq", self.sq_pieces(inner, scope)]
        raise PatchUnsupported("scalar mixing text and actions outside single quotes")

    def sq_pieces(self, pieces, scope):
        out = []
        for p in pieces:
            if p[0] == "t":
                if "'" in p[1].replace("''", ""):
                    raise PatchUnsupported("quote inside a single-quoted scalar")
                if p[1]:
                    out.append(["t", p[1].replace("''", "'")])
            elif p[0] == "v":
                if p[1][1] is not None:
                    raise PatchUnsupported("assignment inside a scalar")
                out.append(["v", self._expr(self.pipeline(p[1], scope))])
            else:
                sub = _Scope(scope)
                it = self._expr(self.pipeline(("pipe", None, p[1][2]), scope))
                vi, ve = self.range_vars(p[1], sub)
                out.append(["r", it, vi, ve, self.sq_pieces(p[2], sub)])
        return out

    # -- block structure
    def value_after(self, entries, pos, indent, scope, sets):
        """Block value of a `key:` line: a sequence at >= indent, a mapping at > indent, or null."""
        nxt = _first_line(entries[pos:])
        if nxt is not None and nxt[1] >= indent and _is_item(nxt):
            return self.seq(entries, pos, nxt[1], scope, sets)
        if nxt is not None and nxt[1] > indent:
            return self.mapping(entries, pos, nxt[1], scope, sets)
        return ["lit", "null"], pos

    def mapping(self, entries, pos, indent, scope, sets, first=None):
        guards, items = [], []
        pos = self._entries_into(entries, pos, indent, scope, sets, guards, items, -1, first)
        by_key: Dict[str, List[int]] = {}
        for key, reg, _ in items:
            by_key.setdefault(key, []).append(reg)
        for key, regs in by_key.items():
            for i in range(len(regs)):
                for j in range(i + 1, len(regs)):
                    if not self._exclusive(regs[i], regs[j]):
                        raise PatchUnsupported(f"mapping key {key!r} defined twice")
        ents = [[go_json_string(k) + ":", r, node] for k, r, node in sorted(items, key=lambda it: it[0])]
        return ["map", guards, ents], pos

    def _ancestors(self, r):
        out = []
        while r != -1:
            out.append(r)
            r = self.reg_parent.get(r, -1)
        return out

    def _exclusive(self, a, b) -> bool:
        if a == -1 or b == -1:
            return False
        anc_b = set(self._ancestors(b))
        return any(self.reg_sibling.get(x) in anc_b for x in self._ancestors(a))

    def _entries_into(self, entries, pos, indent, scope, sets, guards, items, reg, first=None):
        if first is not None:
            pos = self._entry(first, entries, pos, indent, scope, sets, items, reg)
        while pos < len(entries):
            e = entries[pos]
            if e[0] == "assign":
                if reg != -1:
                    raise PatchUnsupported("assignment inside a conditional block")
                self.assign(e[1], scope, sets)
                pos += 1
                continue
            if e[0] == "block":
                fl = _first_line([e])
                if fl is None:
                    raise PatchUnsupported("control block without content")
                if fl[1] < indent or _is_item(fl):
                    return pos
                if fl[1] > indent or e[1] != "if":
                    raise PatchUnsupported(f"{{{{ {e[1]} }}}} around mapping entries")
                self._map_if(e, indent, scope, sets, guards, items, reg)
                pos += 1
                continue
            if e[1] < indent or _is_item(e):
                return pos
            if e[1] > indent:
                raise PatchUnsupported("unexpected indentation")
            pos = self._entry(e, entries, pos + 1, indent, scope, sets, items, reg)
        return pos

    def _entry(self, line, entries, pos, indent, scope, sets, items, reg):
        s = _lead(line)
        m = _KEY.match(s)
        if not m:
            raise PatchUnsupported(f"not a mapping entry: {s!r}")
        key = m.group("key")
        if key[0] in "\"'":
            key = yaml.safe_load(key)
        node = self.scalar([("t", s[m.end():])] + list(line[2][1:]), scope)
        if node is None:
            node, pos = self.value_after(entries, pos, indent, scope, sets)
        items.append((key, reg, node))
        return pos

    def _map_if(self, block, indent, scope, sets, guards, items, parent):
        cond = self._expr(self.pipeline(block[2], scope))
        rt, re_ = self.n_regs, self.n_regs + 1
        self.n_regs += 2
        self.reg_parent[rt] = self.reg_parent[re_] = parent
        self.reg_sibling[rt], self.reg_sibling[re_] = re_, rt
        guards.append([cond, rt, re_, parent])
        for body, r in ((block[3], rt), (block[4], re_)):
            pos = self._entries_into(body, 0, indent, _Scope(scope), sets, guards, items, r)
            if pos != len(body):
                raise PatchUnsupported("conditional block does not hold whole mapping entries")

    def seq(self, entries, pos, indent, scope, sets):
        items: List = []
        pos = self._items_into(entries, pos, indent, scope, sets, items, True)
        return ["seq", items], pos

    def _items_into(self, entries, pos, indent, scope, sets, items, top):
        while pos < len(entries):
            e = entries[pos]
            if e[0] == "assign":
                self.assign(e[1], scope, sets)
                pos += 1
                continue
            if e[0] == "block":
                fl = _first_line([e])
                if fl is None:
                    raise PatchUnsupported("control block without content")
                if fl[1] != indent or not _is_item(fl):
                    if fl[1] > indent:
                        raise PatchUnsupported("unexpected indentation")
                    return pos
                pos += 1
                if e[1] == "range":
                    sub = _Scope(scope)
                    it = self._expr(self.pipeline(("pipe", None, e[2][2]), scope))
                    vi, ve = self.range_vars(e[2], sub)
                    body_sets, body = [], []
                    if self._items_into(e[3], 0, indent, sub, body_sets, body, False) != len(e[3]):
                        raise PatchUnsupported("range body does not hold whole sequence items")
                    items.append(["range", it, vi, ve, body_sets, body])
                else:
                    cond = self._expr(self.pipeline(e[2], scope))
                    branches = []
                    for body in (e[3], e[4]):
                        bsets, bitems = [], []
                        if self._items_into(body, 0, indent, _Scope(scope), bsets, bitems, False) != len(body):
                            raise PatchUnsupported("if body does not hold whole sequence items")
                        if bsets:
                            raise PatchUnsupported("assignment inside a conditional block")
                        branches.append(bitems)
                    items.append(["if", cond, branches[0], branches[1]])
                continue
            if e[1] != indent or not _is_item(e):
                if e[1] > indent:
                    raise PatchUnsupported("unexpected indentation")
                return pos
            rest = _lead(e)[1:]
            inner = e[1] + 1 + len(rest) - len(rest.lstrip(" "))
            rest = rest.lstrip(" ")
            if _KEY.match(rest):
                first = ("line", inner, [("t", " " * inner + rest)] + list(e[2][1:]))
                node, pos = self.mapping(entries, pos + 1, inner, scope, sets, first=first)
            else:
                node = self.scalar([("t", rest)] + list(e[2][1:]), scope)
                if node is None:
                    raise PatchUnsupported("nested block sequence item")
                pos += 1
            items.append(["item", node])
        return pos

    def compile(self, text: str, root: str) -> dict:
        entries = _entries(gotpl._parse(text.strip()))
        fl = _first_line(entries)
        if fl is None or _is_item(fl):
            raise PatchUnsupported("template is not a mapping")
        sets: List = []
        node, pos = self.mapping(entries, 0, fl[1], _Scope(), sets)
        if pos != len(entries):
            raise PatchUnsupported("content after the top-level mapping")
        head = "{" + go_json_string(root) + ":" if root else ""
        return {"n_vars": self.n_vars, "n_regs": self.n_regs, "exprs": self.exprs, "prologue": sets,
                "head": head, "body": node, "tail": "}" if root else ""}


# ------------------------------------------------------------------ native program
_FN = C.CFUNCTYPE(C.c_int32, C.c_void_p, C.c_uint32, C.c_uint32, C.POINTER(C.c_char_p), C.POINTER(C.c_uint32),
                  C.POINTER(C.c_uint8), C.c_void_p, C.c_uint32, C.POINTER(C.c_uint32))
KIND_NAMES = {0: "missing", 1: "nil", 2: "bool", 3: "num", 4: "str", 5: "arr", 6: "obj"}

_lib = None


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise abi.EngineError(f"native patch library missing: {LIB_PATH} (run python -m kwok_amd.build)")
        L = C.CDLL(LIB_PATH)
        L.kwk_patch_last_error.restype = C.c_char_p
        L.kwk_patch_last_error.argtypes = [C.c_void_p]
        L.kwk_patcher_create.argtypes = [C.c_char_p, C.POINTER(C.c_void_p)]
        L.kwk_patcher_destroy.argtypes = [C.c_void_p]
        L.kwk_patch_render.argtypes = [C.c_void_p, C.c_uint32, C.c_void_p, C.c_char_p, C.c_void_p, C.c_int64, _FN,
                                       C.c_void_p, C.c_uint32, C.POINTER(C.c_char_p), C.c_void_p, C.c_void_p]
        L.kwk_patch_skeleton.argtypes = [C.c_void_p, C.c_uint32, C.c_char_p, C.c_uint64, C.POINTER(C.c_void_p),
                                         C.POINTER(C.c_uint64)]
        L.kwk_patch_object_values.argtypes = [C.c_void_p, C.c_uint32, C.c_uint32, C.c_char_p, C.c_void_p, C.c_char_p,
                                              C.c_uint64, _FN, C.c_void_p, C.c_uint32, C.c_uint32, C.c_uint32, C.c_void_p,
                                              C.c_void_p]
        for n in ("kwk_patcher_create", "kwk_patcher_destroy", "kwk_patch_render", "kwk_patch_skeleton",
                  "kwk_patch_object_values"):
            getattr(L, n).restype = C.c_int32
        _lib = L
    return _lib


def _check(st, what, h=None):
    """Raise for a failed call; the message is the handle's own (per handle), or the calling
    thread's for create."""
    if st != 0:
        raise abi.EngineError(f"{what} failed ({st}): {lib().kwk_patch_last_error(h).decode(errors='replace')}")


def _arg_value(kind: int, text: str):
    if kind == 2:
        return text == "true"
    if kind == 3:
        return gotpl.Num(text)
    if kind in (0, 1):
        return None
    return text


class PatchProgram:
    """The merge-patch templates of a set of Stages, compiled for libkwok_patch.

    ``funcs``: the controller's template functions by name — a string is a constant the
    native renderer returns itself; a callable is called back with the arguments (the
    Go host's funcNodeIPWith / funcPodIPWith, pod_controller.go:563-600).
    """

    def __init__(self, stages, funcs: Optional[Dict[str, object]] = None, version: str = "v0.6.0",
                 n_threads: int = 1, program=None):
        """program: a native_compiler.NativeProgram — the spec and template ids come from
        libkwok_compiler (kwk_program_patch_spec) instead of this module's compiler."""
        funcs = dict(funcs or {})
        self.n_threads = n_threads
        self.callbacks: Dict[int, Callable] = {}
        fspec, fids = [], {}
        for name in sorted(funcs):
            fids[name] = len(fspec)
            if isinstance(funcs[name], str):
                fspec.append({"name": name, "const": funcs[name]})
            else:
                self.callbacks[len(fspec)] = funcs[name]
                fspec.append({"name": name, "callback": True})
        consts = [gotpl._from_go_data(gotpl.NODE_CONDITIONS), version]
        const_ids = {"NodeConditions": 0, "Version": 1}
        self.templates: List[dict] = []
        self.template_of: Dict[Tuple[int, int], int] = {}   # (stage index, patch index) -> template id
        self.unsupported: Dict[Tuple[int, int], str] = {}
        self.stages = list(stages)
        if program is not None:
            self.spec, self.template_of = program.patch_spec(funcs, version)
            for si, st in enumerate(self.stages):
                for pi in range(len(st.next.patches)):
                    if (si, pi) not in self.template_of:
                        self.unsupported[(si, pi)] = "not compiled by libkwok_compiler"
            self.h = C.c_void_p()
            _check(lib().kwk_patcher_create(self.spec.encode(), C.byref(self.h)), "kwk_patcher_create")
            self._fn = _FN(self._callback)
            return
        for si, st in enumerate(self.stages):
            for pi, p in enumerate(st.next.patches):
                if p.type not in ("merge", "strategic"):
                    self.unsupported[(si, pi)] = f"patch type {p.type}"
                    continue
                try:
                    t = TemplateCompiler(fids, const_ids).compile(p.template, p.root)
                except (PatchUnsupported, gotpl.TemplateError) as e:
                    self.unsupported[(si, pi)] = str(e)
                    continue
                self.template_of[(si, pi)] = len(self.templates)
                self.templates.append(t)
        self.spec = json.dumps({"templates": self.templates, "funcs": fspec, "consts": consts})
        self.h = C.c_void_p()
        _check(lib().kwk_patcher_create(self.spec.encode(), C.byref(self.h)), "kwk_patcher_create")
        self._fn = _FN(self._callback)

    def _callback(self, user, fid, argc, argv, argl, kinds, out, cap, out_len):
        try:
            args = [_arg_value(kinds[i], C.string_at(argv[i], argl[i]).decode()) for i in range(argc)]
            r = gotpl.go_sprint(self.callbacks[fid](*args)).encode()
        except Exception:
            return 1
        out_len[0] = len(r)
        if len(r) > cap:
            return 2
        C.memmove(out, r, len(r))
        return 0

    def close(self):
        if self.h:
            lib().kwk_patcher_destroy(self.h)
            self.h = C.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def render_buffer(self, template_ids: np.ndarray, buf: bytes, offsets: np.ndarray, now_ns: int):
        """-> (patch bytes buffer, n + 1 offsets, per-object status)."""
        n = len(template_ids)
        tids = np.ascontiguousarray(template_ids, dtype=np.uint16)
        offsets = np.ascontiguousarray(offsets, dtype=np.uint64)
        out_offs = np.zeros(n + 1, dtype=np.uint64)
        status = np.zeros(n, dtype=np.uint8)
        data = C.c_char_p()
        _check(lib().kwk_patch_render(self.h, n, abi.ptr(tids), buf, abi.ptr(offsets), int(now_ns), self._fn, None,
                                      self.n_threads, C.byref(data), abi.ptr(out_offs), abi.ptr(status)),
               "kwk_patch_render", self.h)
        total = int(out_offs[-1])
        return (C.string_at(data, total) if total else b""), out_offs, status

    def render(self, template_ids: Sequence[int], objs: Sequence, now_ns: int) -> List[Optional[bytes]]:
        """Patch bytes per object (None = NEEDS_RENDER: use render_patch_bytes)."""
        from .encoder import pack_json
        buf, offs = pack_json(objs)
        out, o, st = self.render_buffer(np.asarray(template_ids), buf, offs, now_ns)
        return [out[int(o[i]):int(o[i + 1])] if st[i] == STATUS_OK else None for i in range(len(objs))]

    def skeleton(self, tid: int, obj) -> dict:
        """kwk_patch_skeleton: the template's skeleton over obj's class (see kwok_patch.h)."""
        b = obj if isinstance(obj, (bytes, bytearray)) else json.dumps(obj, separators=(",", ":")).encode()
        data, n = C.c_void_p(), C.c_uint64()
        _check(lib().kwk_patch_skeleton(self.h, int(tid), bytes(b), len(b), C.byref(data), C.byref(n)),
               "kwk_patch_skeleton", self.h)
        return json.loads(C.string_at(data, n.value).decode())

    def object_values(self, tid: int, objs: Sequence, skeleton_text: str, n_calls: int, stride: int):
        """kwk_patch_object_values -> (values uint8 [n, n_calls, stride], ok uint8 [n])."""
        from .encoder import pack_json
        buf, offs = pack_json(objs) if not isinstance(objs, tuple) else objs
        offs = np.ascontiguousarray(offs, dtype=np.uint64)
        n = len(offs) - 1
        vals = np.zeros((n, max(n_calls, 0), stride), dtype=np.uint8)
        ok = np.zeros(n, dtype=np.uint8)
        sk = skeleton_text.encode()
        _check(lib().kwk_patch_object_values(self.h, int(tid), n, buf, abi.ptr(offs), sk, len(sk), self._fn, None,
                                             self.n_threads, n_calls, stride, abi.ptr(vals) if n_calls else None,
                                             abi.ptr(ok)), "kwk_patch_object_values", self.h)
        return vals, ok
