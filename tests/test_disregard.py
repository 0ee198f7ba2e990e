"""need()'s disregard selectors.

Reference: pkg/kwok/controllers/pod_controller.go:392-409 and node_controller.go:153-166 — a pod
whose node kwok does not manage, or an object whose non-empty annotation / label map matches the
configured disregardStatusWith{Annotation,Label}Selector (controller.go:114-115, parsed by
labelsParse, controllers/utils.go:116-121 = apimachinery labels.Parse), is skipped by
watchResources: it is never preprocessed (matched), while a job already queued for it still plays.

* CPU: the label-selector grammar and matching — product (kwok_amd/host/labelsel.py), native
  (kwok_amd/csrc/labelsel.hpp, through libkwok_compiler + libkwok_encoder) and the oracle's own
  restatement (oracle/labels_ref.py) — agree on known-answer cases (parity pinned only by
  pod_controller_test.go:195-345, "fake=custom"; the other cases come from the grammar and are
  parity unpinned); the compilers agree byte for byte with a disregard bit configured.
* GPU: disregarded pods and nodes, and pods on unknown nodes, never fire, and the engine stays
  bit-exact with the oracle extended with the same filter."""
import json

import numpy as np
import pytest

from kwok_amd import workload as W
from kwok_amd.host import abi
from kwok_amd.host.labelsel import DisregardSpec, SelectorError, Selector, labels_parse
from oracle import labels_ref

T, F, E = True, False, "error"
CASES = [
    # pod_controller_test.go:195,345: labels.Parse("fake=custom") on the pod's annotations
    ("fake=custom", {"fake": "custom"}, T), ("fake=custom", {"fake": "x"}, F), ("fake=custom", {"other": "custom"}, F),
    ("a", {"a": ""}, T), ("a", {"b": "1"}, F),
    ("!a", {"b": "1"}, T), ("!a", {"a": "1"}, F),
    ("a!=1", {"b": "1"}, T), ("a!=1", {"a": "1"}, F), ("a!=1", {"a": "2"}, T),
    ("a in (1,2)", {"a": "2"}, T), ("a in (1,2)", {"a": "3"}, F), ("a in (1,2)", {"b": "1"}, F),
    ("a notin (1,2)", {"b": "1"}, T), ("a notin (1,2)", {"a": "1"}, F), ("a notin(1,2)", {"a": "3"}, T),
    ("a in ()", {"a": ""}, T), ("a in ()", {"a": "x"}, F), ("a in (,x)", {"a": ""}, T), ("a in (x,)", {"a": ""}, T),
    ("a in (x,,y)", {"a": ""}, T), ("a in (x,,y)", {"a": "y"}, T),
    ("a>5", {"a": "6"}, T), ("a>5", {"a": "5"}, F), ("a>5", {"a": "x"}, F), ("a>5", {"b": "9"}, F),
    ("a<5", {"a": "-1"}, T), ("a<5", {"a": "+4"}, T), ("a < 5", {"a": "5"}, F),
    ("a==b", {"a": "b"}, T), ("a=", {"a": ""}, T), ("a==", {"a": ""}, T), ("a=", {"a": "x"}, F),
    ("a=b,c", {"a": "b", "c": "1"}, T), ("a=b,c", {"a": "b"}, F), ("  a = b , !c ", {"a": "b"}, T),
    ("x.io/y=1", {"x.io/y": "1"}, T), ("example.com/k in (v)", {"example.com/k": "v"}, T),
    ("in in (in)", {"in": "in"}, T), ("   ", {"z": "1"}, T),
    ("a in", {}, E), ("a in (b", {}, E), ("=b", {}, E), ("a b", {}, E), ("!a=b", {}, E), ("a,", {}, E), (",a", {}, E),
    ("a>b", {}, E), ("a>-5", {}, E), ("A_/b=1", {}, E), ("-a=1", {}, E), ("a=-b", {}, E), ("a in (b c)", {}, E),
    ("a=b=c", {}, E), ("a!", {}, E), ("a/b/c=1", {}, E), ("a=" + "x" * 64, {}, E),
]


@pytest.mark.parametrize("sel,labels,want", CASES)
def test_selector_product_and_oracle(sel, labels, want):
    if want == E:
        with pytest.raises(SelectorError):
            Selector(sel)
        with pytest.raises(labels_ref.BadSelector):
            labels_ref.parse(sel)
        return
    assert Selector(sel).matches(labels) is want
    assert labels_ref.matches(labels_ref.parse(sel), labels) is want


def test_labels_parse_empty_is_no_selector():
    assert labels_parse("") is None and not DisregardSpec().active
    d = DisregardSpec(annotation_selector="fake=custom")
    pod = W.pod_object("p", "n")
    assert not d.disregarded(pod)
    pod["metadata"]["annotations"] = {"fake": "custom"}
    assert d.disregarded(pod)
    # a selector applies only to a non-empty map: "!x" disregards a labelled object, never an unlabelled one
    d2 = DisregardSpec(label_selector="!x")
    assert not d2.disregarded(W.pod_object("p", "n")) and d2.disregarded(W.pod_object("p", "n", labels={"y": "1"}))
    assert labels_ref.disregarded("", "!x", W.pod_object("p", "n", labels={"y": "1"}))
    assert not labels_ref.disregarded("", "!x", W.pod_object("p", "n"))


def test_selector_native_via_encoder():
    """The native selector (labelsel.hpp) — compiled by libkwok_compiler, evaluated per object by
    libkwok_encoder into the disregard feature bit — on the same cases (the label map as the pods'
    labels; invalid selectors are compile errors)."""
    from kwok_amd.host.encoder import NativeIngest
    from kwok_amd.host.native_compiler import CompileError, NativeProgram, stage_docs_from_files
    docs = stage_docs_from_files(*W.stage_paths(W.POD_FAST))
    for sel, labels, want in CASES:
        spec = DisregardSpec(label_selector=sel) if want != E else None
        if want == E:
            with pytest.raises(CompileError):
                NativeProgram(docs, disregard=type("D", (), {"active": True, "annotation_selector": "",
                                                             "label_selector": sel})())
            continue
        nat = NativeProgram(docs, disregard=spec)
        bit = nat.describe()["disregard"]["bit"]
        ing = NativeIngest(nat)
        hot = ing.columns([W.pod_object("p", "n", labels=labels or None)], register=True)[0]
        assert bool(int(hot["pred"][0]) >> bit & 1) is (want and bool(labels)), (sel, labels)
        assert nat.table().disregard_mask == 1 << bit
        ing.close()
        nat.close()


@pytest.mark.parametrize("harness", [False, True])
def test_compilers_agree_with_disregard(harness):
    from kwok_amd.host.compiler import HarnessSpec, KindProgram
    from kwok_amd.host.encoder import encoder_spec
    from kwok_amd.host.native_compiler import NativeProgram, stage_docs_from_files
    from kwok_amd.host.stages import load_stage_files
    paths = W.stage_paths(W.POD_GENERAL + W.POD_CHAOS)
    d = DisregardSpec(annotation_selector="fake=custom", label_selector="tier in (batch),!keep")
    roots = [W.pod_object("p", "n"), W.pod_object("p", "n", annotations={"fake": "custom"}),
             W.pod_object("p", "n", labels={"tier": "batch"}), W.pod_object("p", "n", init=1, labels={"tier": "web"})]
    kp = KindProgram(load_stage_files(*paths), HarnessSpec() if harness else None, disregard=d)
    nat = NativeProgram(stage_docs_from_files(*paths), HarnessSpec() if harness else None, disregard=d)
    kp.explore(roots)
    nat.explore(roots)
    assert bytes(nat.table(3)) == bytes(kp.table(3)) and kp.table(3).disregard_mask
    assert np.array_equal(nat.delta_array(), kp.delta_array())
    assert bytes(nat.harness_struct()) == bytes(kp.harness_struct())
    assert nat.describe() == kp.describe()
    assert nat.encoder_spec() == encoder_spec(kp)
    if harness:  # labels / annotations survive the harness re-creation
        assert kp.harness_struct().keep_mask & kp.table().disregard_mask
    nat.close()


def _disregard_cluster(seed):
    cl = W.make_cluster("C2", 30, 360, seed=seed)
    objs = cl.pods.materialize()
    for i, o in enumerate(objs):
        md = o["metadata"]
        if i % 5 == 1:
            md.setdefault("annotations", {})["fake"] = "custom"      # disregarded (annotation selector)
        elif i % 5 == 2:
            md.setdefault("labels", {})["tier"] = "batch"            # disregarded (label selector)
        elif i % 5 == 3:
            md.setdefault("labels", {})["tier"] = "web"              # needed: selector does not match
    return cl, objs


@pytest.mark.gpu
@pytest.mark.parametrize("compiler", ["python", "native"])
def test_gpu_disregarded_pods_never_fire(compiler):
    """C2 pods with need()'s selectors configured — a fifth annotated fake=custom, a fifth labelled
    tier=batch (both disregarded) — plus pods on a node kwok does not manage (need() false until
    the node is known, then synced): disregarded pods never fire, every other pod runs its stages,
    bit-exact against the oracle with the same filter at every step (fired sets, states, feature
    bits incl. the disregard bit, dirty flags)."""
    from tests.parity_util import NOW0, build, compare_state
    cl, objs = _disregard_cluster(81)
    d = DisregardSpec(annotation_selector="fake=custom", label_selector="tier in (batch)")
    prog, eng, sim = build(cl.pod_stage_files, objs, harness=True, compiler=compiler, disregard=d)
    try:
        # pods of "node-0" are on a node kwok does not know (pod_controller.go:393-395): not managed
        unknown = [i for i, o in enumerate(objs) if o["spec"]["nodeName"] == "node-0"]
        hot, dels = eng.read()
        hot["sched"][unknown] &= ~np.uint32(abi.F_MANAGED)
        eng.upsert(np.asarray(unknown), hot[unknown], dels[unknown], np.zeros(len(unknown), np.uint32),
                   (hot["sched"][unknown] >> 16).astype(np.uint16))
        for i in unknown:
            sim.managed[i] = False
        disregarded = {i for i in range(len(objs)) if i % 5 in (1, 2)}
        fired_slots = set()
        for k in range(36):
            now = NOW0 + k * 500 * 10**6
            if k == 12:  # the node becomes known: ManageNode -> podsOnNodeSync re-sends its pods
                hot, dels = eng.read()
                hot["sched"][unknown] |= np.uint32(abi.F_MANAGED | abi.F_DIRTY)
                eng.upsert(np.asarray(unknown), hot[unknown], dels[unknown], np.zeros(len(unknown), np.uint32),
                           (hot["sched"][unknown] >> 16).astype(np.uint16))
                for i in unknown:
                    sim.set_managed(i, True, True)
            eng.step(now, 0x81, k)
            got = sorted((int(r["slot"]), int(r["stage"]), int(r["flags"])) for r in eng.fired())
            assert got == sorted(sim.step(now, 0x81, k)), f"step {k}"
            compare_state(prog, eng, sim, k)
            fired_slots |= {g[0] for g in got}
            if k < 12:
                assert not fired_slots & set(unknown), k
        assert not fired_slots & disregarded
        needed = set(range(len(objs))) - disregarded
        assert len(fired_slots & needed) > 0.9 * len(needed)
        assert fired_slots & set(unknown) - disregarded  # they run once their node is known
    finally:
        eng.close()


@pytest.mark.gpu
def test_gpu_disregarded_nodes_never_fire():
    """node-fast + node-heartbeat with a label selector disregarding a third of the nodes."""
    from tests.parity_util import run
    objs = [W.node_object(f"node-{i}", labels={"pool": "frozen"} if i % 3 == 0 else None) for i in range(60)]
    total, per = run(W.stage_paths(W.NODE_FAST + W.NODE_HEARTBEAT), objs, steps=20, dt_ns=2 * 10**9, kind_salt=1,
                     compiler="native", disregard=DisregardSpec(label_selector="pool=frozen"))
    assert per["node-initialize"] == 40 and per["node-heartbeat"] > 0


@pytest.mark.gpu
def test_gpu_queued_pod_relabelled_disregarded_and_back():
    """pods with a queued stage whose labels change to match the disregard selector (a
    Modified event need() skips, pod_controller.go:397-407) still fire the queued stage and are
    not re-matched while disregarded; when the label is removed again, re-matching resumes.  The
    host re-encodes the changed objects and upserts them with the device's queued stage and due
    time kept (the informer's event); the oracle gets the same label edits.  Fired sets and
    states against the oracle every step."""
    from kwok_amd.host.engine import Ingest
    from tests.parity_util import NOW0, build, compare_state
    cl, objs = _disregard_cluster(83)
    d = DisregardSpec(annotation_selector="fake=custom", label_selector="tier in (batch)")
    prog, eng, sim = build(cl.pod_stage_files, objs, harness=True, disregard=d)
    try:
        _, _, rec0, _ = Ingest(prog).columns(objs)  # the record index each slot was loaded with
        ing = Ingest(prog)
        moved, fired_moved = [], {"off": set(), "on": set()}

        def relabel(on):
            for i in moved:
                for o in (sim.objs[i], sim.orig[i]):  # the re-created object keeps its labels too
                    if o is None:
                        continue
                    labels = o.setdefault("metadata", {}).setdefault("labels", {})
                    if on:
                        labels["tier"] = "batch"
                    else:
                        labels.pop("tier", None)
                if sim.objs[i] is not None:
                    sim.dirty[i] = True
            hot, dels = eng.read()
            cur = [sim.objs[i] if sim.objs[i] is not None else sim.orig[i] for i in moved]
            nh, _, _, nc = ing.columns(cur)
            rows = hot[moved].copy()
            rows["pred"] = nh["pred"]
            alive = (rows["sched"] & np.uint32(abi.F_ALIVE)) != 0
            rows["sched"] = np.where(alive, rows["sched"] | np.uint32(abi.F_DIRTY), rows["sched"])
            eng.replace(np.asarray(moved), rows, dels[moved], rec0[moved], nc)

        for k in range(40):
            now = NOW0 + k * 500 * 10**6
            if k == 8:  # needed pods with a queued stage not yet due
                moved = [i for i in range(len(objs)) if i % 5 in (0, 3, 4) and sim.objs[i] is not None
                         and sim.pending[i] is not None and sim.due[i] > now][:24]
                assert len(moved) >= 8
                relabel(True)
            if k == 24:
                relabel(False)
            eng.step(now, 0x83, k)
            got = sorted((int(r["slot"]), int(r["stage"]), int(r["flags"])) for r in eng.fired())
            assert got == sorted(sim.step(now, 0x83, k)), f"step {k}"
            compare_state(prog, eng, sim, k)
            mv = {g[0] for g in got} & set(moved)
            if 8 <= k < 24:
                fired_moved["off"] |= mv
            elif k >= 24:
                fired_moved["on"] |= mv
        assert fired_moved["off"], "queued stages of relabelled pods fire"
        assert fired_moved["on"], "re-matching resumes once the label is gone"
    finally:
        eng.close()
