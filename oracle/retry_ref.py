"""ORACLE / TEST INFRASTRUCTURE — not product code.

CPU restatement of KWOK's playStage retry branch, the checker for kwk_retry.  Only tests/
import it.

  playStageWorker retry  pkg/kwok/controllers/pod_controller.go:273-284
                         (needRetry -> retryCount = RetryCount++ ; addStageJob(job, delay, 1))
  backoffDelayByStep     pkg/kwok/controllers/utils.go:138-143
                         min(float64(Duration) * math.Pow(Factor, steps), float64(Cap)),
                         time.Duration(...) then wait.Jitter(d, Jitter)
  defaultBackoff         utils.go:133-135 (1 s, x2, jitter 0.2, cap 32 min)
  math.Pow               Go 1.22 src/math/pow.go, integer exponent branch (frexp, repeated
                         squaring of the mantissa with a separate exponent, Ldexp)

rand.Float64 inside wait.Jitter is replaced by the Philox hook, site 4.
The reference has no unit test for backoffDelayByStep; the restatement is pinned by the
exact powers of two of the default backoff (1 s, 2 s, 4 s, ... capped at 32 min) in
tests/test_retry.py and by the device parity test.
"""
from __future__ import annotations

import math

from . import refcpu
from .lease_ref import sat_add

SITE_RETRY_JITTER = 4
INT64_MIN = -(1 << 63)


def go_pow_int(x: float, n: int) -> float:
    """math.Pow(x, float64(n)) for an integer n >= 0 (pow.go's yi loop; yf = 0)."""
    if n == 0 or x == 1.0:
        return 1.0
    if n == 1:
        return x
    if x == 0.0 or math.isinf(x) or math.isnan(x):
        return math.pow(x, n)
    a1, ae = 1.0, 0
    x1, xe = math.frexp(x)
    i = n
    while i != 0:
        if xe < -(1 << 12) or (1 << 12) < xe:
            ae += xe
            break
        if i & 1:
            a1 *= x1
            ae += xe
        x1 *= x1
        xe <<= 1
        if x1 < 0.5:
            x1 += x1
            xe -= 1
        i >>= 1
    try:
        return math.ldexp(a1, ae)
    except OverflowError:
        return math.inf


def go_duration(d: float) -> int:
    """time.Duration(float64) on amd64: truncation; out of range -> math.MinInt64."""
    if not (-9223372036854775808.0 < d < 9223372036854775808.0):
        return INT64_MIN
    return int(d)


def backoff_delay(steps: int, duration_ns: int, factor: float, jitter_f: float, cap_ns: int, u: float) -> int:
    d = min(float(duration_ns) * go_pow_int(factor, steps), float(cap_ns))
    base = go_duration(d)
    mf = 1.0 if jitter_f <= 0.0 else jitter_f
    return base + go_duration(u * mf * float(base))


def float64_hook(key: int, slot: int, step: int) -> float:
    return float(refcpu.philox_u64(key, slot, step, SITE_RETRY_JITTER) >> 11) / 9007199254740992.0


def retry_due(now_ns: int, seed: int, kind_salt: int, gslot: int, step: int, steps: int, backoff: dict) -> int:
    u = float64_hook(seed ^ (kind_salt << 32), gslot, step)
    return sat_add(now_ns, backoff_delay(steps, backoff["duration_ns"], backoff["factor"], backoff["jitter"],
                                         backoff["cap_ns"], u))
