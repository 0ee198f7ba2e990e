"""ORACLE / TEST INFRASTRUCTURE — not product code.

CPU restatement of KWOK's node-lease controller, the checker for the device's lease step
(kwk_lease_step).  Pure Python over plain records; only tests/ import it.

  tryAcquireOrRenew      pkg/kwok/controllers/node_lease_controller.go:293-306
  expireTime             node_lease_controller.go:309-319
  nextTryDuration        node_lease_controller.go:322-338
  syncWorker + sync      node_lease_controller.go:108-143, 174-275 (ensureLease / renewLease)
  interval / wait.Jitter node_lease_controller.go:145-147; k8s apimachinery wait.Jitter:
                         d + time.Duration(rand.Float64() * maxFactor * float64(d)), maxFactor <= 0 -> 1
  Held / readOnlyFunc    node_lease_controller.go:164-171, controller.go:285-288

rand.Float64 is replaced by the same Philox hook as the device (site 3, (u64 >> 11) * 2^-53).
The apiserver round trip returns renewTime as a metav1.MicroTime, i.e. truncated to
microseconds.  A rejected write (LeaseSim.fail) is syncWorker's err branch (:121-128):
the informer keeps the old lease and the sync is retried after the same interval() draw.
"""
from __future__ import annotations

from dataclasses import dataclass, replace
from typing import List, Optional, Tuple

from . import refcpu

EXISTS, HOLDER, DURATION, RENEW, HOLD, QUEUED = 1, 2, 4, 8, 16, 32
OP_CREATE, OP_RENEW, OP_ACQUIRE, OP_BUSY, OP_FAILED = 1, 2, 3, 4, 5
SITE_LEASE_JITTER = 3
SEC = 10**9
INT64_MAX = (1 << 63) - 1
INT64_MIN = -(1 << 63)


def sat_add(a: int, b: int) -> int:
    return max(INT64_MIN, min(INT64_MAX, a + b))


@dataclass
class Lease:
    renew_ns: int = 0
    next_try_ns: int = 0
    holder: int = 0
    duration_s: int = 0
    transitions: int = 0
    flags: int = 0


def try_acquire_or_renew(lease: Lease, holder: int, now_ns: int) -> bool:
    """node_lease_controller.go:293-306."""
    if not (lease.flags & HOLDER) or lease.holder == holder:
        return True
    if not (lease.flags & RENEW) or not (lease.flags & DURATION):
        return True
    return sat_add(lease.renew_ns, lease.duration_s * SEC) < now_ns  # expireTime.Before(now)


def expire_time(lease: Optional[Lease]) -> Tuple[int, bool]:
    """node_lease_controller.go:309-319: (renewTime + leaseDurationSeconds, ok)."""
    if lease is None or not (lease.flags & HOLDER) or not (lease.flags & DURATION) or not (lease.flags & RENEW):
        return 0, False
    return sat_add(lease.renew_ns, lease.duration_s * SEC), True


def next_try_duration(renew_interval: int, expire: int, hold: bool) -> int:
    """node_lease_controller.go:322-338."""
    if not hold:
        return renew_interval
    if renew_interval < expire:
        return renew_interval
    if expire < SEC:
        return SEC
    return expire


def jitter(duration: int, max_factor: float, u: float) -> int:
    """wait.Jitter with rand.Float64() = u; time.Duration(float64) truncates toward zero."""
    if max_factor <= 0.0:
        max_factor = 1.0
    return duration + int(u * max_factor * float(duration))


def float64_hook(key: int, slot: int, step: int) -> float:
    return float(refcpu.philox_u64(key, slot, step, SITE_LEASE_JITTER) >> 11) / 9007199254740992.0


def held(lease: Lease, holder: int) -> bool:
    """NodeLeaseController.Held (:164-171) on the cached lease."""
    return bool(lease.flags & EXISTS) and bool(lease.flags & HOLDER) and lease.holder == holder


class LeaseSim:
    """syncWorker over all held nodes whose queued sync is due, in slot order (the device runs
    them in parallel; they are independent)."""

    def __init__(self, leases: List[Lease], holder_id: int, lease_duration_s: int, renew_interval_ns: int,
                 renew_jitter: float = 0.04, slot_base: int = 0, kind_salt: int = 1, slots=None):
        """slots: the engine slot of each lease (default leases[i] is slot i): a deterministic
        sample of a large engine's nodes is simulated exactly (leases are independent, the Philox
        counter is the global slot)."""
        self.leases = [replace(l) for l in leases]
        self.slots = list(range(len(leases))) if slots is None else [int(x) for x in slots]
        assert len(self.slots) == len(self.leases)
        self.me = holder_id
        self.duration_s = lease_duration_s
        self.renew_interval = renew_interval_ns
        self.jitter = renew_jitter
        self.slot_base = slot_base
        self.kind_salt = kind_salt

    def step(self, now_ns: int, seed: int, step: int):
        """-> [(slot, op)] for the syncs that ran (op = OP_*)."""
        key = seed ^ (self.kind_salt << 32)
        out = []
        for i, L in enumerate(self.leases):
            if (L.flags & (HOLD | QUEUED)) != (HOLD | QUEUED) or L.next_try_ns > now_ns:
                continue
            dur = jitter(self.renew_interval, self.jitter, float64_hook(key, self.slot_base + self.slots[i], step))
            now_us = now_ns - now_ns % 1000
            ok = False
            if L.flags & EXISTS:
                if try_acquire_or_renew(L, self.me, now_ns):  # renewLease (:252-275)
                    op = OP_RENEW
                    if not (L.flags & HOLDER) or L.holder != self.me:
                        L.holder = self.me
                        L.duration_s = self.duration_s
                        L.transitions += 1
                        L.flags |= HOLDER | DURATION
                        op = OP_ACQUIRE
                    L.renew_ns = now_us
                    L.flags |= RENEW
                    ok = True
                else:
                    op = OP_BUSY
            else:  # ensureLease (:225-249)
                L.flags |= EXISTS | HOLDER | DURATION | RENEW
                L.holder = self.me
                L.duration_s = self.duration_s
                L.renew_ns = now_us
                L.transitions = 0
                op = OP_CREATE
                ok = True
            if ok:
                exp, _ = expire_time(L)
                nxt = next_try_duration(dur, exp - now_ns, try_acquire_or_renew(L, self.me, now_ns))
            else:
                nxt = dur
            L.next_try_ns = now_ns if nxt <= 0 else sat_add(now_ns, nxt)
            out.append((i, op))
        return out

    def fail(self, i: int, old: Lease, now_ns: int, seed: int, step: int):
        """syncWorker's err branch (node_lease_controller.go:121-128): the write of the sync
        that ran at (now_ns, step) was rejected; the cached lease stays `old`, the controller's
        hold / queue flags stay, AddWeightAfter(node, 1, dur) with the same dur."""
        key = seed ^ (self.kind_salt << 32)
        dur = jitter(self.renew_interval, self.jitter, float64_hook(key, self.slot_base + self.slots[i], step))
        ctl = self.leases[i].flags & (HOLD | QUEUED)
        L = replace(old)
        L.flags = (L.flags & ~(HOLD | QUEUED)) | ctl
        L.next_try_ns = sat_add(now_ns, dur)
        self.leases[i] = L
