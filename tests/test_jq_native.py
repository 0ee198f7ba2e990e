"""The native jq subset (kwok_amd/csrc/jqc.hpp, run by libkwok_encoder / libkwok_compiler) against the
reference's own query / selector / getter vectors and against two independent restatements: the
Python mirror (kwok_amd/host/jq.py) and the oracle's gojq restatement (oracle/refcpu/jq.hpp).

Reference: expression.NewQuery / Query.Execute (pkg/utils/expression/query.go:33-69), Requirement
(selector.go:37-120), int64From.Get (value_int_from.go:53-81); gojq v0.12.16 semantics (go.mod:17):
JSON numbers are float64, literals / length / int arithmetic are ints (hasValue matches those
through FormatInt), object keys iterate sorted."""
import ctypes as C
import json
import random

import numpy as np
import pytest

from kwok_amd.host import abi
from kwok_amd.host.encoder import EncoderUnsupported, jq_eval, lib as enc_lib
from kwok_amd.host.jq import Query, has_value

GOLD = json.load(open(__file__.replace("test_jq_native.py", "golden/reference_unit_vectors.json")))


def _obj(o):
    return GOLD["EMPTY_POD"] if o == "EMPTY_POD" else o


def _oracle_query(src, obj):
    from oracle import refcpu
    L = refcpu.lib()
    cap = 1 << 16
    buf = C.create_string_buffer(cap)
    n = L.rc_query(src.encode(), json.dumps(obj).encode(), buf, cap)
    if n == -1000000:
        raise RuntimeError(L.rc_last_error().decode())
    return json.loads(buf.value.decode())


def _num_eq(a, b):
    """JSON values equal, numbers by value (an int and the float of the same value compare equal)."""
    if isinstance(a, bool) or isinstance(b, bool):
        return a is b
    if isinstance(a, (int, float)) and isinstance(b, (int, float)):
        return a == b or (a != a and b != b)
    if isinstance(a, list) and isinstance(b, list):
        return len(a) == len(b) and all(_num_eq(x, y) for x, y in zip(a, b))
    if isinstance(a, dict) and isinstance(b, dict):
        return a.keys() == b.keys() and all(_num_eq(a[k], b[k]) for k in a)
    return a == b


@pytest.mark.parametrize("case", GOLD["query"], ids=lambda c: c["ref"].split(":")[-1])
def test_query_vectors_native(case):
    """query_test.go:39-171 — every vector, the assignment forms `.a = 1` and `.a += [{b:2}]`
    included — through kwk_jq_eval, the Python mirror and the oracle."""
    obj = _obj(case["obj"])
    assert _num_eq(jq_eval(case["src"], obj), case["want"]), case["ref"]
    assert _num_eq(Query(case["src"]).execute(obj), case["want"]), case["ref"]
    assert _num_eq(_oracle_query(case["src"], obj), case["want"]), case["ref"]


class _Enc:
    """A one-feature (and one int slot) native encoder: the pred bits and the value record of one
    object, as kwk_encode computes them for the engine."""

    def __init__(self, query, literals, slot_query=None):
        spec = {"features": [{"query": query, "present_bit": 0,
                              "literals": {v: i + 1 for i, v in enumerate(literals)}}],
                "finalizers": {}, "finalizer_other_bit": None,
                "slots": [{"type": "int", "query": slot_query}] if slot_query else [],
                "classes": {}, "identity_meta": []}
        self.h = C.c_void_p()
        st = enc_lib().kwk_encoder_create(json.dumps(spec).encode(), C.byref(self.h))
        if st == abi.KWK_EINVAL:
            raise EncoderUnsupported(enc_lib().kwk_encoder_last_error(None).decode())
        assert st == 0
        self.n_lits = len(literals)

    def encode(self, obj):
        buf = json.dumps(obj).encode()
        offs = np.array([0, len(buf)], dtype=np.uint64)
        hot = np.zeros(1, dtype=abi.HOT_DTYPE)
        dels = np.zeros(1, dtype=np.int64)
        rec = np.zeros(1, dtype=np.uint32)
        cls = np.zeros(1, dtype=np.uint16)
        nu = C.c_uint32()
        st = enc_lib().kwk_encode(self.h, 1, buf, abi.ptr(offs), 1, abi.ptr(hot), abi.ptr(dels), abi.ptr(rec),
                                  abi.ptr(cls), C.byref(nu))
        assert st == 0, enc_lib().kwk_encoder_last_error(self.h).decode()
        pred = int(hot["pred"][0])
        value = None
        if int(hot["sched"][0]) & abi.F_HASREC:
            n = C.c_uint32()
            recs = np.zeros(int(rec[0]) + 1, dtype=abi.VALUE_DTYPE)
            enc_lib().kwk_encoder_records(self.h, abi.ptr(recs), len(recs), C.byref(n))
            value = recs[int(rec[0])]
        return pred, value

    def close(self):
        enc_lib().kwk_encoder_destroy(self.h)


def _matches(pred, op, n_lits):
    """Requirement.Matches (selector.go:65-99) from the feature's bits: present (bit 0) and the
    literals' bits (1..n)."""
    present = bool(pred & 1)
    any_lit = any(pred >> (i + 1) & 1 for i in range(n_lits))
    return {"In": any_lit, "NotIn": not any_lit, "Exists": present, "DoesNotExist": not present}[op]


@pytest.mark.parametrize("case", GOLD["requirement"], ids=lambda c: c["ref"].split(":")[-1])
def test_requirement_vectors_native_encoder(case):
    """selector_test.go:44-131 through the native encoder's feature bits (what the device matches)."""
    enc = _Enc(case["key"], case["values"])
    try:
        pred, _ = enc.encode(_obj(case["obj"]))
        assert _matches(pred, case["op"], len(case["values"])) == case["want"], case["ref"]
    finally:
        enc.close()


@pytest.mark.parametrize("case", GOLD["int_from"][2:], ids=lambda c: c["ref"].split(":")[-1])
def test_int_from_vectors_native_encoder(case):
    """value_int_from_test.go:57-97 (the *From cases) through the native encoder's value record."""
    enc = _Enc(".metadata.name", [], slot_query=case["src"])
    try:
        _, v = enc.encode(_obj(case["obj"]))
        assert v is not None and int(v["kind"]) == abi.V_OK and int(v["value"]) == case["want"], case["ref"]
    finally:
        enc.close()


# ------------------------------------------------------------------ gojq value-model specifics
@pytest.mark.parametrize("query,obj,op,values,want", [
    # length is a gojq int: FormatInt "2" matches (a float64 JSON number never does)
    (".status.conditions | length", {"status": {"conditions": [{}, {}]}}, "In", ["2"], True),
    (".spec.replicas", {"spec": {"replicas": 2}}, "In", ["2"], False),
    (".spec.replicas | length", {"spec": {"replicas": 2}}, "In", ["2"], False),  # abs(float64) stays float
    (".metadata.labels | length", {"metadata": {}}, "In", ["0"], True),  # null has length 0 (an int)
    ('.status.phase != "Running"', {"status": {"phase": "Pending"}}, "In", ["true"], True),
    ('.status.phase != "Running"', {"status": {}}, "In", ["true"], True),  # null != "Running"
    ('.status.conditions | map(select(.status == "True")) | length >= 2',
     {"status": {"conditions": [{"status": "True"}, {"status": "False"}, {"status": "True"}]}}, "In", ["true"], True),
    ('.metadata.annotations | has("x")', {"metadata": {"annotations": {"x": ""}}}, "In", ["true"], True),
    ('.metadata.annotations | has("x")', {"metadata": {}}, "Exists", [], False),  # has on null: error -> nil
    ('.metadata.labels.tier // "none"', {"metadata": {"labels": {}}}, "In", ["none"], True),
    ('.metadata.labels.tier // "none"', {"metadata": {"labels": {"tier": "gold"}}}, "In", ["gold"], True),
    ('(.status.phase == "Failed") | not', {"status": {"phase": "Failed"}}, "In", ["false"], True),
    (".a.b", {"a": 3}, "NotIn", ["x"], True),  # runtime error: nil -> NotIn true
    (".a.b?", {"a": 3}, "DoesNotExist", [], True),
    ('.status.containerStatuses[0].restartCount + 1', {"status": {"containerStatuses": [{"restartCount": 1}]}},
     "In", ["2"], False),  # float64 + int = float64
    ("1 + 1", {}, "In", ["2"], True),
    ('[.spec.containers[].name] | length', {"spec": {"containers": [{"name": "a"}, {"name": "b"}]}}, "In", ["2"], True),
    ('.metadata.annotations | keys | .[0]', {"metadata": {"annotations": {"b": "1", "a": "2"}}}, "In", ["a"], True),
    ('.metadata.annotations[]', {"metadata": {"annotations": {"b": "1", "a": "2"}}}, "In", ["1"], True),
    ('if .spec.x then "y" else "n" end', {"spec": {"x": False}}, "In", ["n"], True),
])
def test_gojq_value_model_through_native_encoder(query, obj, op, values, want):
    """Selector semantics that depend on gojq's value model, through the native encoder, the Python
    mirror and the oracle (where its subset reaches)."""
    enc = _Enc(query, values)
    try:
        pred, _ = enc.encode(obj)
        assert _matches(pred, op, len(values)) == want
    finally:
        enc.close()
    out = Query(query).execute(obj)
    mirror = {"In": out is not None and any(has_value(d, values) for d in out),
              "Exists": bool(out), "DoesNotExist": not out}
    mirror["NotIn"] = not mirror["In"]
    assert mirror[op] == want


def test_int_getter_gojq_int_falls_to_default():
    """int64From.Get switches on string / float64 only: a gojq int (e.g. `length`) takes the default
    (value_int_from.go:61-80) — the encoder leaves the slot at KWK_V_DEFAULT."""
    enc = _Enc(".metadata.name", [], slot_query=".spec.containers | length")
    try:
        _, v = enc.encode({"metadata": {"name": "x"}, "spec": {"containers": [{}, {}]}})
        assert v is None  # every slot at its default: no value record
        _, v = enc.encode({"metadata": {"name": "x"}, "spec": {"containers": "ab"}})
        assert v is None
    finally:
        enc.close()
    enc = _Enc(".metadata.name", [], slot_query=".spec.n * 2")
    try:
        _, v = enc.encode({"metadata": {"name": "x"}, "spec": {"n": 3}})
        assert int(v["kind"]) == abi.V_OK and int(v["value"]) == 6  # float64 * int = float64
    finally:
        enc.close()


def test_refused_constructs_name_the_construct():
    """Outside the subset: KWK_EINVAL with the construct named (kwk_jq_eval, kwk_encoder_create and
    the mirror alike); a Go host keeps the reference lifecycle for such a resourceRef."""
    from kwok_amd.host.jq import JqError
    for q, what in (("reduce .[] as $x (0; . + $x)", "'reduce'"), (".[] as $x | $x", "'as'"), ('test("a")', "test/1"),
                    (".a[1:]", "slices"), ('"\\(.a)"', "interpolation"), ("..", "'..'"), ("@csv", "formats"),
                    ("$ENV", "variables"), ("def f: .; f", "'def'"), ("try .a catch .", "catch")):
        with pytest.raises(EncoderUnsupported, match=what):
            jq_eval(q, {})
        with pytest.raises(EncoderUnsupported, match=what):
            _Enc(q, [])
        with pytest.raises(JqError, match=what):
            Query(q)


# ------------------------------------------------------------------ differential fuzzing
_KEYS = ["a", "b", "c", "phase", "x y"]


def _rand_json(rng, depth=0):
    r = rng.random()
    if depth > 2 or r < 0.35:
        return rng.choice([None, True, False, 0, 1, 2.5, -3, "", "a", "b", "Running", "2", "true"])
    if r < 0.65:
        return [_rand_json(rng, depth + 1) for _ in range(rng.randrange(4))]
    return {rng.choice(_KEYS): _rand_json(rng, depth + 1) for _ in range(rng.randrange(4))}


def _rand_path(rng):
    p = ""
    for _ in range(rng.randrange(1, 4)):
        k = rng.choice(_KEYS)
        p += f'."{k}"' if " " in k else ("." + k if rng.random() < 0.7 else f'.["{k}"]')
        r = rng.random()
        if r < 0.15:
            p += "[]"
        elif r < 0.22:
            p += "[0]"
        elif r < 0.27:
            p += "?"
    return p


def _rand_lit(rng):
    return rng.choice(['"a"', '"Running"', "1", "2", "0", "2.5", "true", "false", "null", '""'])


def _rand_query(rng, depth=0, oracle=False):
    r = rng.random()
    if depth > 2 or r < 0.25:
        return _rand_path(rng)
    if r < 0.35:
        return f"{_rand_query(rng, depth + 1, oracle)} | length"
    if r < 0.45:
        op = rng.choice(["==", "!=", "<", "<=", ">", ">="])
        return f"({_rand_query(rng, depth + 1, oracle)}) {op} {_rand_lit(rng)}"
    if r < 0.52:
        return f"({_rand_query(rng, depth + 1, oracle)}) // {_rand_lit(rng)}"
    if r < 0.58:
        return f"({_rand_query(rng, depth + 1, oracle)}) {rng.choice(['and', 'or'])} ({_rand_query(rng, depth + 1, oracle)})"
    if r < 0.63:
        return f"{_rand_query(rng, depth + 1, oracle)} | not"
    if r < 0.70:
        return f"{_rand_path(rng)} | select({_rand_query(rng, depth + 1, oracle)})"
    if r < 0.75:
        return f'{_rand_path(rng)} | has("{rng.choice(_KEYS)}")'
    if r < 0.79:
        return f"{_rand_path(rng)} | keys"
    if r < 0.83:
        return f"[{_rand_query(rng, depth + 1, oracle)}]"
    if r < 0.87:
        return f"({_rand_query(rng, depth + 1, oracle)}) {rng.choice(['+', '-'])} {_rand_lit(rng)}"
    if r < 0.91:
        return f"if {_rand_query(rng, depth + 1, oracle)} then {_rand_lit(rng)} else {_rand_path(rng)} end"
    if r < 0.94:
        return f"{_rand_query(rng, depth + 1, oracle)}, {_rand_query(rng, depth + 1, oracle)}"
    if oracle:
        return f"{_rand_path(rng)} | type"
    return rng.choice([f"{_rand_path(rng)} | map(length)", f"{_rand_path(rng)} | tostring",
                       f"{_rand_path(rng)} | add", f"{_rand_path(rng)} | any", f"{_rand_path(rng)} * 2",
                       f'{_rand_path(rng)} | contains("a")', f"{_rand_path(rng)} | first",
                       f'{_rand_path(rng)} |= . // "d"', f"{_rand_path(rng)} = 1", f"{_rand_path(rng)} += 1",
                       f"{_rand_path(rng)} | tonumber?", f'{_rand_path(rng)} | startswith("a")?'])


@pytest.mark.parametrize("seed", range(4))
def test_differential_native_mirror_oracle(seed):
    """Random queries over the subset on random documents: kwk_jq_eval = the Python mirror (output
    values) on every query, = the oracle on the oracle's subset; and the native encoder's feature
    bits = the mirror's Requirement.Matches for literals drawn from the outputs (ints, strings,
    bools: the FormatInt / FormatBool cases)."""
    rng = random.Random(1000 + seed)
    n_checked = n_oracle = n_nil = 0
    for _ in range(300):
        oracle = rng.random() < 0.5
        q = _rand_query(rng, oracle=oracle)
        doc = {k: _rand_json(rng) for k in rng.sample(_KEYS, rng.randrange(1, 5))}
        mir = Query(q).execute(doc)
        nat = jq_eval(q, doc)
        assert (mir is None) == (nat is None), (q, doc, mir, nat)
        if mir is None:
            n_nil += 1
        else:
            assert _num_eq(nat, mir), (q, doc, mir, nat)
        if oracle:
            orc = _oracle_query(q, doc)
            assert (orc is None) == (mir is None) and (mir is None or _num_eq(orc, mir)), (q, doc, mir, orc)
            n_oracle += 1
        lits = sorted({("true" if d else "false") if isinstance(d, bool) else str(d) for d in (mir or [])
                       if isinstance(d, (str, bool, int))} | {"2", "true"})[:12]
        enc = _Enc(q, lits)
        try:
            pred, _ = enc.encode(doc)
        finally:
            enc.close()
        assert bool(pred & 1) == bool(mir), (q, doc)
        for i, v in enumerate(lits):
            assert bool(pred >> (i + 1) & 1) == (mir is not None and any(has_value(d, (v,)) for d in mir)), (q, doc, v)
        n_checked += 1
    assert n_checked == 300 and n_oracle > 100 and 10 < n_nil < 250
