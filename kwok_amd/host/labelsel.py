"""Label selectors as the controllers' need() filters parse and match them (host side).

Reference: the disregard filters of need() — pkg/kwok/controllers/pod_controller.go:392-409,
node_controller.go:153-166, stage_controller.go:380-392 — built by labelsParse
(controllers/utils.go:116-121: "" -> no selector, else k8s.io/apimachinery v0.30.2
labels.Parse) from the kwok configuration (controller.go:114-115,424-425,453-454,513-514), and
applied as ``selector.Matches(labels.Set(obj.Annotations))`` / ``...(obj.Labels)`` only when the
map is non-empty.

apimachinery is not vendored in the reference, so the grammar and matching are restated from
its published selector.go: requirements joined by ``,`` (AND); ``key`` (Exists), ``!key``
(DoesNotExist), ``key=v`` / ``key==v`` / ``key!=v``, ``key in (a,b)`` / ``key notin (a,b)``,
``key>n`` / ``key<n`` (integers, strconv.ParseInt base 10); NotIn / != also match objects without
the key; an empty value list ``()`` means {""}; keys are qualified names, values label values.
Parity is pinned only by pod_controller_test.go:195-345 ("fake=custom"); the rest is unpinned
(tests/test_disregard.py holds known-answer cases from the grammar).

The device never sees selectors: the compiler folds need()'s result into one feature bit
(``disregard``) that the encoder computes per object and the exploration tracks through deltas.
"""
from __future__ import annotations

import re
from dataclasses import dataclass
from typing import Dict, List, Optional, Tuple


class SelectorError(ValueError):
    pass


_SPECIAL = "=!(),><"
_WS = " \t\r\n"
_QNAME = re.compile(r"^([A-Za-z0-9][-A-Za-z0-9_.]*)?[A-Za-z0-9]$")
_DNS1123 = re.compile(r"^[a-z0-9]([-a-z0-9]*[a-z0-9])?(\.[a-z0-9]([-a-z0-9]*[a-z0-9])?)*$")
_LVALUE = re.compile(r"^(([A-Za-z0-9][-A-Za-z0-9_.]*)?[A-Za-z0-9])?$")

# tokens
ID, IN, NOTIN, NOT, NEQ, EQ, DEQ, GT, LT, OPEN, CLOSE, COMMA, END = range(13)
_SYMBOLS = {"!": NOT, "!=": NEQ, "(": OPEN, ")": CLOSE, ",": COMMA, "=": EQ, "==": DEQ, ">": GT, "<": LT}


def _lex(s: str) -> List[Tuple[int, str]]:
    out, i = [], 0
    while i < len(s):
        c = s[i]
        if c in _WS:
            i += 1
            continue
        if c in _SPECIAL:
            two = s[i:i + 2]
            if two in _SYMBOLS:
                out.append((_SYMBOLS[two], two))
                i += 2
            else:
                out.append((_SYMBOLS[c], c))
                i += 1
            continue
        j = i
        while j < len(s) and s[j] not in _WS and s[j] not in _SPECIAL:
            j += 1
        lit = s[i:j]
        out.append(({"in": IN, "notin": NOTIN}.get(lit, ID), lit))
        i = j
    out.append((END, ""))
    return out


def parse_int10(s: str) -> Optional[int]:
    """strconv.ParseInt(s, 10, 64)."""
    if not re.fullmatch(r"[+-]?[0-9]+", s):
        return None
    v = int(s)
    return v if -(1 << 63) <= v < (1 << 63) else None


def _check_key(k: str):
    parts = k.split("/")
    if len(parts) == 1:
        name = parts[0]
    elif len(parts) == 2:
        prefix, name = parts
        if not prefix or len(prefix) > 253 or not _DNS1123.match(prefix):
            raise SelectorError(f"invalid label key {k!r}: bad prefix")
    else:
        raise SelectorError(f"invalid label key {k!r}")
    if not name or len(name) > 63 or not _QNAME.match(name):
        raise SelectorError(f"invalid label key {k!r}")


def _check_value(v: str):
    if len(v) > 63 or not _LVALUE.match(v):
        raise SelectorError(f"invalid label value {v!r}")


@dataclass
class Requirement:
    key: str
    op: str          # in notin = == != exists !  gt lt
    values: Tuple[str, ...]

    def matches(self, ls: Dict[str, str]) -> bool:
        has = self.key in ls
        if self.op in ("in", "=", "=="):
            return has and ls[self.key] in self.values
        if self.op in ("notin", "!="):
            return not has or ls[self.key] not in self.values
        if self.op == "exists":
            return has
        if self.op == "!":
            return not has
        if not has:  # gt / lt
            return False
        v = parse_int10(ls[self.key])
        if v is None or len(self.values) != 1:
            return False
        r = parse_int10(self.values[0])
        if r is None:
            return False
        return v > r if self.op == "gt" else v < r


class Selector:
    """labels.Parse(text): a conjunction of requirements (no requirements: everything)."""

    def __init__(self, text: str):
        self.text = text
        self.reqs: List[Requirement] = []
        t = _lex(text)
        p = 0

        def look(values=True):
            k, lit = t[p]
            if values and k in (IN, NOTIN):
                k = ID
            return k, lit

        def take(values=True):
            nonlocal p
            r = look(values)
            p += 1
            return r

        while True:
            k, lit = look()
            if k in (ID, NOT):
                self.reqs.append(self._requirement(look, take))
                k2, lit2 = take()
                if k2 == END:
                    break
                if k2 == COMMA:
                    k3, lit3 = look()
                    if k3 not in (ID, NOT):
                        raise SelectorError(f"found '{lit3}', expected: identifier after ','")
                    continue
                raise SelectorError(f"found '{lit2}', expected: ',' or 'end of string'")
            if k == END:
                break
            raise SelectorError(f"found '{lit}', expected: !, identifier, or 'end of string'")

    @staticmethod
    def _requirement(look, take) -> Requirement:
        op = None
        k, lit = take()
        if k == NOT:
            op = "!"
            k, lit = take()
        if k != ID:
            raise SelectorError(f"found '{lit}', expected: identifier")
        key = lit
        _check_key(key)
        if look()[0] in (END, COMMA):
            return Requirement(key, op or "exists", ())
        if op == "!":
            return Requirement(key, "!", ())
        k, lit = take(values=False)
        ops = {IN: "in", NOTIN: "notin", EQ: "=", DEQ: "==", NEQ: "!=", GT: "gt", LT: "lt"}
        if k not in ops:
            raise SelectorError(f"found '{lit}', expected: one of in, notin, =, ==, !=, gt, lt")
        op = ops[k]
        vals: List[str] = []
        if op in ("in", "notin"):
            k, lit = take()
            if k != OPEN:
                raise SelectorError(f"found '{lit}' expected: '('")
            k, lit = look()
            if k == CLOSE:
                take()
                vals = [""]
            elif k in (ID, COMMA):
                s: List[str] = []
                while True:
                    k, lit = take()
                    if k == ID:
                        s.append(lit)
                        k2, lit2 = look()
                        if k2 == COMMA:
                            continue
                        if k2 == CLOSE:
                            break
                        raise SelectorError(f"found '{lit2}', expected: ',' or ')'")
                    elif k == COMMA:
                        if not s:
                            s.append("")
                        k2, _ = look()
                        if k2 == CLOSE:
                            s.append("")
                            break
                        if k2 == COMMA:
                            take()
                            s.append("")
                    else:
                        raise SelectorError(f"found '{lit}', expected: ',', or identifier")
                if take()[0] != CLOSE:
                    raise SelectorError("expected: ')'")
                vals = s
            else:
                raise SelectorError(f"found '{lit}', expected: ',', ')' or identifier")
        else:
            k, lit = look()
            if k in (END, COMMA):
                vals = [""]
            else:
                k, lit = take()
                if k != ID:
                    raise SelectorError(f"found '{lit}', expected: identifier")
                vals = [lit]
        vals = sorted(set(vals))
        if op in ("in", "notin") and not vals:
            raise SelectorError("for 'in', 'notin' operators, values set can't be empty")
        if op in ("=", "==", "!=") and len(vals) != 1:
            raise SelectorError("exact-match compatibility requires one single value")
        if op in ("gt", "lt"):
            if len(vals) != 1 or parse_int10(vals[0]) is None:
                raise SelectorError("for 'Gt', 'Lt' operators, the value must be an integer")
        for v in vals:
            _check_value(v)
        return Requirement(key, op, tuple(vals))

    def matches(self, ls: Dict[str, str]) -> bool:
        return all(r.matches(ls) for r in self.reqs)


def labels_parse(text: str) -> Optional[Selector]:
    """controllers/utils.go:116-121 labelsParse: "" -> nil (no filter)."""
    return None if text == "" else Selector(text)


@dataclass
class DisregardSpec:
    """The kwok configuration's disregardStatusWith{Annotation,Label}Selector (controller.go:114-115)."""
    annotation_selector: str = ""
    label_selector: str = ""

    def __post_init__(self):
        self._ann = labels_parse(self.annotation_selector)
        self._lab = labels_parse(self.label_selector)

    @property
    def active(self) -> bool:
        return self._ann is not None or self._lab is not None

    def disregarded(self, obj: dict) -> bool:
        """not need(obj), the selector part (pod_controller.go:397-407): a selector applies only
        to a non-empty map."""
        md = (obj or {}).get("metadata") or {}
        ann = md.get("annotations") or {}
        lab = md.get("labels") or {}
        if self._ann is not None and len(ann) and self._ann.matches({str(k): str(v) for k, v in ann.items()}):
            return True
        if self._lab is not None and len(lab) and self._lab.matches({str(k): str(v) for k, v in lab.items()}):
            return True
        return False
