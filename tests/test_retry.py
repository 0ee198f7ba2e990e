"""playStage retry / backoff (kwk_retry): oracle/retry_ref.py restates backoffDelayByStep
(pkg/kwok/controllers/utils.go:138-143) and the retry branch of playStageWorker
(pod_controller.go:273-284); the GPU test fails some fired jobs and checks the device and the
oracle stay bit-exact through the retries."""
import copy
import math

import numpy as np
import pytest

from kwok_amd import workload as W
from kwok_amd.host import abi
from kwok_amd.host.engine import Ingest
from oracle import retry_ref

B = abi.DEFAULT_BACKOFF


def test_go_pow_int_exact_powers():
    for k in range(0, 80):
        assert retry_ref.go_pow_int(2.0, k) == 2.0 ** k
    assert retry_ref.go_pow_int(2.0, 5000) == math.inf
    assert retry_ref.go_pow_int(0.5, 3) == 0.125
    assert retry_ref.go_pow_int(3.0, 4) == 81.0


def test_default_backoff_without_jitter_draw():
    """u = 0: 1 s * 2^steps, capped at 32 min (defaultBackoff, utils.go:133-135)."""
    for steps in range(0, 40):
        want = min(10**9 * 2**steps, 32 * 60 * 10**9)
        assert retry_ref.backoff_delay(steps, B["duration_ns"], B["factor"], B["jitter"], B["cap_ns"], 0.0) == want


def test_backoff_jitter_bounds_and_nonpositive_factor():
    d = retry_ref.backoff_delay(3, 10**9, 2.0, 0.2, 10**12, 0.5)
    assert d == 8 * 10**9 + int(0.5 * 0.2 * 8e9)
    # wait.Jitter: maxFactor <= 0 means 1.0
    assert retry_ref.backoff_delay(0, 10**9, 2.0, 0.0, 10**12, 0.25) == 10**9 + 250_000_000


@pytest.mark.gpu
def test_retry_parity_pod_fast():
    from tests.parity_util import NOW0, build, compare_state
    cl = W.make_cluster("C1", 10, 200, seed=21)
    objs = cl.pods.materialize()
    prog, eng, sim = build(cl.pod_stage_files, objs)
    ing = Ingest(prog)
    seed = 0x5EED
    try:
        rc = {}
        for k in range(14):
            now = NOW0 + k * 10**9
            pre = [copy.deepcopy(o) for o in sim.objs]
            eng.step(now, seed, k)
            got = sorted((int(r["slot"]), int(r["stage"]), int(r["flags"])) for r in eng.fired())
            exp = sorted(sim.step(now, seed, k))
            assert got == exp, f"step {k}"
            # the apiserver rejects every third fired job of this step (retryable error)
            failed = [(i, s) for (i, s, _) in exp[::3] if pre[i] is not None]
            if k < 10 and failed:
                slots = np.array([i for i, _ in failed], dtype=np.uint32)
                stages = np.array([s for _, s in failed], dtype=np.uint16)
                counts = np.array([rc.get(i, 0) for i, _ in failed], dtype=np.uint32)
                hot = np.zeros(len(failed), dtype=abi.HOT_DTYPE)
                cls = np.zeros(len(failed), dtype=np.uint16)
                for j, (i, s) in enumerate(failed):
                    pred, flags, _, _, c = ing.encode(pre[i])
                    hot[j] = (pred, flags | abi.STAGE_NONE, 0)
                    cls[j] = c
                eng.retry(now, seed, k, slots, hot, cls, stages, counts)
                for j, (i, s) in enumerate(failed):
                    sim.objs[i] = pre[i]
                    sim.pending[i] = s
                    sim.dirty[i] = False
                    sim.matcherr[i] = False
                    sim.due[i] = retry_ref.retry_due(now, seed, 0, i, k, int(counts[j]), B)
                    rc[i] = rc.get(i, 0) + 1
            compare_state(prog, eng, sim, k)
    finally:
        eng.close()


@pytest.mark.gpu
def test_retry_backoff_reaches_the_cap():
    """Retry counts far past the doubling range: the device's due times equal the oracle's
    backoffDelayByStep through the 32-minute cap (utils.go:133-143), Philox jitter included,
    and the pending stage is re-queued."""
    from tests.parity_util import NOW0, build
    cl = W.make_cluster("C1", 4, 64, seed=5)
    objs = cl.pods.materialize()
    prog, eng, sim = build(cl.pod_stage_files, objs)
    ing = Ingest(prog)
    seed = 0xBAC0
    try:
        now = NOW0
        pre = [copy.deepcopy(o) for o in sim.objs]
        eng.step(now, seed, 0)
        fired = sorted((int(r["slot"]), int(r["stage"])) for r in eng.fired())
        assert len(fired) >= 20
        fired = fired[:20]
        counts = np.array([0, 1, 5, 10, 11, 12, 13, 20, 31, 40, 63, 64, 100, 1000, 10**5, 2**31, 2**32 - 1, 3, 7, 9],
                          dtype=np.uint32)
        slots = np.array([i for i, _ in fired], dtype=np.uint32)
        stages = np.array([s for _, s in fired], dtype=np.uint16)
        hot = np.zeros(len(fired), dtype=abi.HOT_DTYPE)
        cls = np.zeros(len(fired), dtype=np.uint16)
        for j, (i, _) in enumerate(fired):
            pred, flags, _, _, c = ing.encode(pre[i])
            hot[j] = (pred, flags | abi.STAGE_NONE, 0)
            cls[j] = c
        eng.retry(now, seed, 0, slots, hot, cls, stages, counts)
        got, _ = eng.read()
        cap = B["cap_ns"]
        for j, (i, s) in enumerate(fired):
            want = retry_ref.retry_due(now, seed, 0, i, 0, int(counts[j]), B)
            assert int(got["due"][i]) == want, (j, int(counts[j]))
            assert int(got["sched"][i]) & 0xFF == s
            if counts[j] >= 12:  # 2^11 s > 32 min: capped, then jittered by up to 20 %
                assert cap <= want - now <= cap * 1.2 + 1
    finally:
        eng.close()
