"""ORACLE / TEST INFRASTRUCTURE — not product code.

Independent restatement of k8s.io/apimachinery v0.30.2 labels.Parse + Selector.Matches (not
vendored in the reference; pkg/labels/selector.go as published) as need()'s disregard filters use
them: pkg/kwok/controllers/pod_controller.go:392-409, node_controller.go:153-166 (a selector
applies only to a non-empty annotation / label map), controllers/utils.go:116-121 ("" -> nil).

Written as a token stream from one regular expression and a small state machine, separately
from the product's kwok_amd/host/labelsel.py; only tests/ import it.  Parity for the grammar is
unpinned beyond pod_controller_test.go:195-345 ("fake=custom").
"""
from __future__ import annotations

import re

_TOK = re.compile(r"\s*(?:(!=|==|=|!|\(|\)|,|>|<)|([^\s=!(),<>]+))")
_KEYNAME = r"(?:[A-Za-z0-9](?:[-A-Za-z0-9_.]{0,61}[A-Za-z0-9])?)"
_PREFIX = r"(?:[a-z0-9](?:[-a-z0-9]*[a-z0-9])?(?:\.[a-z0-9](?:[-a-z0-9]*[a-z0-9])?)*)"
_VALUE = re.compile(r"(?:[A-Za-z0-9](?:[-A-Za-z0-9_.]{0,61}[A-Za-z0-9])?)?")


class BadSelector(ValueError):
    pass


def _key_ok(k):
    if "/" in k:
        pre, _, name = k.partition("/")
        if "/" in name or not pre or len(pre) > 253 or not re.fullmatch(_PREFIX, pre):
            return False
    else:
        name = k
    return bool(re.fullmatch(_KEYNAME, name))


def _int(s):
    return int(s) if re.fullmatch(r"[+-]?\d+", s) and -(2 ** 63) <= int(s) < 2 ** 63 else None


def tokens(text):
    pos, out = 0, []
    text = text.rstrip(" \t\r\n")
    while pos < len(text):
        m = _TOK.match(text, pos)
        if not m or m.end() == pos:
            raise BadSelector(text)
        out.append(("sym", m.group(1)) if m.group(1) else ("word", m.group(2)))
        pos = m.end()
    return out


def parse(text):
    """-> list of (key, op, frozenset(values)); op in {"in", "notin", "exists", "!", "gt", "lt"}."""
    toks = tokens(text) + [("end", None)]
    i = 0
    reqs = []
    if toks[0][0] == "end":
        return reqs
    while True:
        neg = toks[i] == ("sym", "!")
        if neg:
            i += 1
        kind, key = toks[i]
        if kind != "word" or not _key_ok(key):
            raise BadSelector(f"key at {i}")
        i += 1
        nxt = toks[i]
        if nxt[0] == "end" or nxt == ("sym", ","):
            reqs.append((key, "!" if neg else "exists", frozenset()))
        elif neg:
            raise BadSelector("'!key' takes no operator")
        else:
            opk, op = toks[i]
            i += 1
            if opk == "word" and op in ("in", "notin"):
                if toks[i] != ("sym", "("):
                    raise BadSelector("( expected")
                i += 1
                vals, expect_item = set(), True
                while True:
                    k, v = toks[i]
                    i += 1
                    if k == "word":
                        if not expect_item:
                            raise BadSelector("',' or ')' expected")
                        vals.add(v)
                        expect_item = False
                    elif (k, v) == ("sym", ","):
                        if expect_item:  # an empty item: "(,", ",,"
                            vals.add("")
                        expect_item = True
                    elif (k, v) == ("sym", ")"):
                        if expect_item:  # "()" or ",)"
                            vals.add("")
                        break
                    else:
                        raise BadSelector("bad value list")
                op = "in" if op == "in" else "notin"
            elif opk == "sym" and op in ("=", "==", "!=", ">", "<"):
                k, v = toks[i]
                if k == "word":
                    vals = {v}
                    i += 1
                elif k == "end" or (k, v) == ("sym", ","):
                    vals = {""}
                else:
                    raise BadSelector("value expected")
                op = {"=": "in", "==": "in", "!=": "notin", ">": "gt", "<": "lt"}[op]
                if op in ("gt", "lt") and _int(next(iter(vals))) is None:
                    raise BadSelector("Gt / Lt need an integer")
            else:
                raise BadSelector("operator expected")
            if any(len(v) > 63 or not _VALUE.fullmatch(v) for v in vals):
                raise BadSelector("bad label value")
            reqs.append((key, op, frozenset(vals)))
        k, v = toks[i]
        i += 1
        if k == "end":
            return reqs
        if (k, v) != ("sym", ","):
            raise BadSelector("',' or end expected")
        if toks[i][0] == "end":
            raise BadSelector("identifier expected after ','")


def matches(reqs, labels) -> bool:
    for key, op, vals in reqs:
        v = labels.get(key)
        has = key in labels
        if op == "in" and not (has and v in vals):
            return False
        if op == "notin" and has and v in vals:
            return False
        if op == "exists" and not has:
            return False
        if op == "!" and has:
            return False
        if op in ("gt", "lt"):
            a, b = (_int(v) if has else None), _int(next(iter(vals)))
            if a is None or b is None or not (a > b if op == "gt" else a < b):
                return False
    return True


def disregarded(annotation_selector: str, label_selector: str, obj) -> bool:
    """not need(obj), the selector part."""
    md = (obj or {}).get("metadata") or {}
    for sel, m in ((annotation_selector, md.get("annotations") or {}), (label_selector, md.get("labels") or {})):
        if sel != "" and m and matches(parse(sel), {str(k): str(x) for k, x in m.items()}):
            return True
    return False
