"""Native ingestion encoder (kwok_amd/csrc/encoder.cpp) against the Python Ingest (which the
oracle pins through the GPU parity tests) on every object the workloads produce: the C1 / C2
pods (initial objects and the states the compiler explores: status, finalizers, deletion
timestamps, override annotations incl. invalid ints / durations / RFC3339), nodes and the
edge cases of the Go parsers; plus its throughput (objects/s, reported, not asserted)."""
import copy
import json
import time

import numpy as np
import pytest

from kwok_amd import workload as W
from kwok_amd.host.compiler import HarnessSpec, KindProgram
from kwok_amd.host.encoder import EncoderUnsupported, NativeIngest, check_query, pack_json
from kwok_amd.host.engine import Ingest
from kwok_amd.host.stages import load_stage_files


def _rows_equal(prog, objs, n_threads=1):
    py = Ingest(prog)
    want = py.columns(objs)
    nat = NativeIngest(prog, n_threads=n_threads)
    got = nat.columns(objs)
    for col, a, b in zip(("hot", "deletion", "rec", "cls"), want, got):
        if col == "rec":
            continue
        assert np.array_equal(a, b), col
    # records: same content per object (ids are both in object order)
    ra, rb = py.record_array(), nat.record_array()
    has = (want[0]["sched"] & 0x800) != 0
    assert np.array_equal(ra[want[2][has]], rb[got[2][has]])
    assert np.array_equal(want[2], got[2])
    return nat


def _states(prog, objs):
    out = list(objs)
    for reps in prog.class_reps.values():
        out += reps
    return out


@pytest.mark.parametrize("config", ["C1", "C2"])
def test_native_encoder_equals_ingest_pods(config):
    cl = W.make_cluster(config, 20, 2000, seed=61)
    objs = cl.pods.materialize()
    prog = KindProgram(load_stage_files(*cl.pod_stage_files), HarnessSpec())
    prog.explore(objs)
    states = _states(prog, objs)
    # the explored states' successors (status / finalizer / deletion variants)
    from kwok_amd.host.compiler import exploration_funcs
    from kwok_amd.host.gotpl import Renderer
    from kwok_amd.host.nextstate import apply_next
    r = Renderer(exploration_funcs(), now_ns=1_700_000_000 * 10**9)
    more = []
    for o in states[-200:]:
        for st in prog.stages:
            try:
                o2, _ = apply_next(st, copy.deepcopy(o), r)
            except Exception:
                continue
            if o2 is not None:
                more.append(o2)
    _rows_equal(prog, states + more, n_threads=4)


def test_native_encoder_equals_ingest_nodes_and_edge_values():
    cl = W.make_cluster("C1", 50, 50, seed=62)
    objs = cl.nodes.materialize()
    prog = KindProgram(load_stage_files(*W.stage_paths(W.NODE_FAST + W.NODE_CHAOS)))
    prog.explore(objs)
    edge = []
    for i, v in enumerate(["2", "0x10", "010", "1_0", "0b_1", "abc", "", "-9223372036854775808", "9223372036854775808",
                           "500ms", "1.5h", "1h2m3.5s", ".5s", "2006-01-02T15:04:05Z", "2006-01-02T15:04:05.123+07:00",
                           "2006-01-02T15:04:05,5Z", "1e3", "µs"]):
        edge.append(W.node_object(f"e{i}", labels={"node-not-ready.stage.kwok.x-k8s.io": "true"},
                                  annotations={"node-not-ready.stage.kwok.x-k8s.io/weight": v,
                                               "node-not-ready.stage.kwok.x-k8s.io/delay": v}))
    edge.append(W.node_object("num", annotations={"node-not-ready.stage.kwok.x-k8s.io/weight": 7}))
    edge.append(W.node_object("ünï", annotations={"x": "ÿ☃"}))
    _rows_equal(prog, objs + edge)


def test_unknown_class_reported():
    cl = W.make_cluster("C1", 4, 40, seed=63)
    objs = cl.pods.materialize()
    prog = KindProgram(load_stage_files(*cl.pod_stage_files))
    prog.explore([o for o in objs if not o["metadata"].get("ownerReferences")])
    nat = NativeIngest(prog)
    hot, _, _, cls = nat.columns(objs)
    job = np.array([bool(o["metadata"].get("ownerReferences")) for o in objs])
    assert np.all(cls[job] == 0xFFFF) and np.all(cls[~job] != 0xFFFF) and nat.unknown_classes == job.sum()


def test_query_forms():
    """The encoder spec carries each query's source; the native jq subset (jqc.hpp / jq.py) accepts
    the shipped forms and the gojq constructs Stage CRs may use, and refuses the rest with the
    construct named."""
    for q in ('.status.conditions.[] | select( .type == "Ready" ) | .status', '.metadata.labels["a/b"]',
              ".status.conditions | length", '.status.phase != "Running"', ".a // .b", 'has("x")',
              ".spec.containers | map(.name) | length > 1", "if .a then 1 else 2 end", ".a.b? | not"):
        assert check_query(q) == q
    for q, what in ((". as $x | $x", "'as'"), ("reduce .[] as $x (0; . + $x)", "'reduce'"), ('test("a")', "test/1"),
                    (".a[1:2]", "slices"), ('"\\(.a)"', "interpolation"), ("..", "'..'"), ("@base64", "formats")):
        with pytest.raises(EncoderUnsupported, match=what):
            check_query(q)


def test_native_encoder_throughput_report(capsys):
    """objects/s of kwk_encode on 200k C2 pod objects (JSON bytes prepared beforehand)."""
    cl = W.make_cluster("C2", 200, 20000, seed=64)
    objs = cl.pods.materialize() * 10
    prog = KindProgram(load_stage_files(*cl.pod_stage_files), HarnessSpec())
    prog.explore(cl.pods.variants)
    buf, offs = pack_json(objs)
    rates = {}
    for t in (1, 8):
        nat = NativeIngest(prog, n_threads=t)
        t0 = time.perf_counter()
        nat.encode_buffer(buf, offs)
        rates[t] = len(objs) / (time.perf_counter() - t0)
    with capsys.disabled():
        print(f"\nnative encoder: {rates[1]:.0f} objects/s (1 thread), {rates[8]:.0f} objects/s (8 threads)")
    assert rates[1] > 0
