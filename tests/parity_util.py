"""Shared driver for the GPU parity tests: run the HIP engine and the oracle simulation
side by side on the same seeded cluster and compare every step bit for bit."""
from __future__ import annotations

import numpy as np

from kwok_amd.host import abi
from kwok_amd.host.compiler import HarnessSpec, KindProgram
from kwok_amd.host.engine import Engine, Ingest
from kwok_amd.host.stages import load_stage_files
from oracle.next_ref import load_stage_docs
from oracle.sim import OracleSim, oracle_pred

NOW0 = 1_700_000_000 * 10**9


def expected_state_bytes(prog, state="auto"):
    """Mirror of make_fmt (engine.hip): packed word = pred | class | stage code | 5 flags; the set
    of sizes the engine may pick ("auto" on a 16-bit program: the 1-byte dictionary ids when the
    program is table-only and its words close within 255 ids, else the 2-byte words; a word of
    at most 28 bits not held in 2 bytes: the 8-byte fused record unless "u32")."""
    if state == "wide":
        return {8}
    t = prog.table()
    pb = t.pred_bits or 32
    bits = pb + max(0, t.n_classes - 1).bit_length() + t.n_stages.bit_length() + 5
    if bits <= 16 and state == "auto":
        return {1, 2}
    if bits <= 16 and state == "u16":
        return {2}
    if bits <= 28 and state != "u32":
        return {8}
    return {4} if bits <= 32 else {8}


def build(stage_files, objs, harness=False, kind_salt=0, slot_base=0, wide_state=False, state="auto", tuning=None,
          compiler="python", disregard=None):
    """compiler: "python" (KindProgram + the Python Ingest) or "native" (libkwok_compiler's
    kwk_compile_stages / kwk_program_explore, rows from libkwok_encoder built from its spec: the
    Go host's path, no Python compiler involved)."""
    if compiler == "native":
        from kwok_amd.host.encoder import NativeIngest
        from kwok_amd.host.native_compiler import NativeProgram, stage_docs_from_files
        prog = NativeProgram(stage_docs_from_files(*stage_files), HarnessSpec() if harness else None, disregard=disregard)
        prog.explore(objs)
        ing = NativeIngest(prog)
        hot, dels, rec, cls = ing.columns(objs, register=True)
        records = ing.record_array()
        ing.close()
    else:
        stages = load_stage_files(*stage_files)
        prog = KindProgram(stages, HarnessSpec() if harness else None, disregard=disregard)
        prog.explore(objs)
        assert not prog.delta_conflicts, prog.delta_conflicts
        ing = Ingest(prog)
        hot, dels, rec, cls = ing.columns(objs)
        records = ing.record_array()
    eng = Engine(prog, capacity=max(1, len(objs)), kind_salt=kind_salt, slot_base=slot_base, wide_state=wide_state,
                 state=state, max_records=max(1 << 16, len(records) + 16))
    for k, v in (tuning or {}).items():
        eng.set_tuning(k, v)
    eng.load_stages()
    eng.set_harness(harness)
    eng.load(hot, dels, rec, cls, records)
    sim = OracleSim(load_stage_docs(*stage_files), objs, harness=harness, kind_salt=kind_salt, slot_base=slot_base,
                    disregard=None if disregard is None else (disregard.annotation_selector, disregard.label_selector))
    return prog, eng, sim


def compare_state(prog, eng, sim, step, rows=None):
    """Every simulated object's device row against the oracle: alive, pending stage, due,
    feature bits (recomputed by the oracle's jq), deletion column, dirty flag.  rows: the
    device rows (hot, deletion_s) at sim.slots, when the caller has read them already."""
    if rows is None:
        hot, dels = eng.read()
        if sim.slots != list(range(len(sim.objs))):
            idx = np.asarray(sim.slots, dtype=np.int64)
            hot, dels = hot[idx], dels[idx]
    else:
        hot, dels = rows
    desc = prog.describe()
    bad = []
    for i, o in enumerate(sim.objs):
        sched = int(hot["sched"][i])
        alive = bool(sched & abi.F_ALIVE)
        if alive != (o is not None):
            bad.append((i, "alive", alive))
            continue
        if o is None:
            continue
        st = sched & 0xFF
        exp_st = 0xFF if sim.pending[i] is None else sim.pending[i]
        if st != exp_st:
            bad.append((i, "stage", st, exp_st))
        elif st != 0xFF and int(hot["due"][i]) != sim.due[i]:
            bad.append((i, "due", int(hot["due"][i]), sim.due[i]))
        p = oracle_pred(desc, o)
        applied = sum(1 << b for b in desc["applied_bits"].values())  # checked through the REMATCH flag
        if int(hot["pred"][i]) & ~applied != p:
            bad.append((i, "pred", hex(int(hot["pred"][i])), hex(p)))
        if desc["uses_deletion_column"] and int(dels[i]) != sim.deletion_s(i):
            bad.append((i, "deletion", int(dels[i]), sim.deletion_s(i)))
        if bool(sched & abi.F_DIRTY) != sim.dirty[i]:
            bad.append((i, "dirty", bool(sched & abi.F_DIRTY), sim.dirty[i]))
    assert not bad, f"step {step}: {len(bad)} mismatches, first: {bad[:8]}"


def run(stage_files, objs, steps, dt_ns, harness=False, seed=0x5EED, kind_salt=0, check_state=True, wide_state=False,
        state="auto", tuning=None, expect_kernel=None, nows=None, compiler="python", disregard=None):
    """expect_kernel: the abi.SWEEP_* every step must launch (the shape under test); nows: the
    clock of each step (default NOW0 + k * dt_ns)."""
    if wide_state:
        state = "wide"
    prog, eng, sim = build(stage_files, objs, harness=harness, kind_salt=kind_salt, state=state, tuning=tuning,
                           compiler=compiler, disregard=disregard)
    total = 0
    per_stage = np.zeros(len(prog.names), dtype=np.int64)
    try:
        for k in range(steps):
            now = NOW0 + k * dt_ns if nows is None else nows[k]
            eng.step(now, seed, k)
            if expect_kernel is not None:
                assert eng.last_sweep()["kernel"] == expect_kernel, (k, eng.last_sweep())
            got = eng.fired()
            exp = sim.step(now, seed, k)
            g = sorted((int(r["slot"]), int(r["stage"]), int(r["flags"])) for r in got)
            assert g == sorted(exp), f"step {k}: fired differ: device-only {sorted(set(g) - set(exp))[:8]} " \
                                     f"oracle-only {sorted(set(exp) - set(g))[:8]}"
            total += len(exp)
            for _, s, _ in exp:
                per_stage[s] += 1
            if check_state:
                compare_state(prog, eng, sim, k)
        st = eng.stats()
        assert st["state_bytes"] in expected_state_bytes(prog, state)
        assert st["fired"] == total
        assert [st["fired_per_stage"][n] for n in prog.names] == list(per_stage)
    finally:
        eng.close()
    return total, dict(zip(prog.names, per_stage.tolist()))
