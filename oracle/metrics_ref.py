"""ORACLE / TEST INFRASTRUCTURE — not product code.

The values of kwok's shipped Metric CR (kustomize/metrics/resource/metrics-resource.yaml,
shipped as kwok_amd/metrics/metrics-resource.yaml) restated per metric name for one node
scrape (pkg/kwok/metrics/metrics.go:168-354: node series, one per pod of the node, one per
container of those pods), with the usage callbacks of pkg/kwok/server/metrics_resource_usage.go
answered by oracle/usage_ref.py.  The CEL is not interpreted here: each value below is the
restatement of its expression, cited by line.
"""
from __future__ import annotations

from . import usage_ref

MAX_SECONDS = 9223372036.854775807  # time.Duration(math.MaxInt64).Seconds(): time.Since saturates


def _since(now_ns: int, created_ns) -> float:
    """pod.SinceSecond() = time.Since(creationTimestamp).Seconds() (pkg/utils/cel/funcs.go:41-43),
    against the scrape's clock; an unset creationTimestamp is the zero time."""
    if created_ns is None:
        return MAX_SECONDS
    d = max(-(1 << 63), min((1 << 63) - 1, now_ns - created_ns))
    return usage_ref.seconds(d)


class MetricsOracle:
    def __init__(self, docs):
        self.docs = docs
        self.cum = usage_ref.Cumulative()

    def scrape(self, now_ns, node, pods, created_ns):
        """node: JSON; pods: the node's alive pods (JSON) in slot order; created_ns(pod) -> ns or None.
        -> {metric name: [(labels, value)]}"""
        D = self.docs
        name = node["metadata"]["name"]
        out = {k: [] for k in ("scrape_error", "container_start_time_seconds", "container_cpu_usage_seconds_total",
                               "container_memory_working_set_bytes", "pod_cpu_usage_seconds_total",
                               "pod_memory_working_set_bytes", "node_cpu_usage_seconds_total",
                               "node_memory_working_set_bytes")}
        out["scrape_error"].append(((), 0.0))  # metrics-resource.yaml:8-13  value: '0'
        node_cpu = node_mem = 0.0
        for pod in pods:
            md = pod["metadata"]
            pl = (("namespace", md.get("namespace", "")), ("pod", md.get("name", "")))
            pc = pm = 0.0
            pcum = 0.0
            for c in pod["spec"].get("containers") or []:
                cn = c.get("name", "")
                cl = (("container", cn),) + pl
                cpu = usage_ref.container_usage(D, pod, cn, "cpu")
                mem = usage_ref.container_usage(D, pod, cn, "memory")
                pc += cpu
                pm += mem
                c_cum = self.cum.advance((md.get("namespace"), md.get("name"), cn, "cpu"), cpu, now_ns)
                pcum += c_cum
                # :14-26 pod.SinceSecond(); :27-39 pod.CumulativeUsage("cpu", container.name);
                # :40-52 pod.Usage("memory", container.name)
                out["container_start_time_seconds"].append((cl, _since(now_ns, created_ns(pod))))
                out["container_cpu_usage_seconds_total"].append((cl, c_cum))
                out["container_memory_working_set_bytes"].append((cl, mem))
            # :53-63 pod.CumulativeUsage("cpu") (the containers' integrators); :64-74 pod.Usage("memory")
            out["pod_cpu_usage_seconds_total"].append((pl, pcum))
            out["pod_memory_working_set_bytes"].append((pl, pm))
            node_cpu += pc
            node_mem += pm
        # :75-81 node.CumulativeUsage("cpu") (one integrator keyed by the node, :67-109); :82-88 node.Usage("memory")
        out["node_cpu_usage_seconds_total"].append(((), self.cum.advance(("node", name), node_cpu, now_ns)))
        out["node_memory_working_set_bytes"].append(((), node_mem))
        return out


def go_float64_to_uint64(x: float) -> int:
    """uint64(x) for a float64 x as Go compiles it for amd64 (cmd/compile ssagen
    float64ToUint64: `if x < 2^63 { r = CVTTSD2SQ(x) } else { r = CVTTSD2SQ(x - 2^63) | 1<<63 }`;
    CVTTSD2SQ of a NaN or of a value outside the int64 range is 0x8000000000000000)."""
    two63 = float(1 << 63)

    def cvttsd2sq(v: float) -> int:
        if v != v or v >= two63 or v < -two63:
            return 1 << 63
        return int(v) % (1 << 64)  # truncation toward zero, two's complement bits

    if x < two63:
        return cvttsd2sq(x)
    return cvttsd2sq(x - two63) | (1 << 63)


def histogram_series(buckets, values):
    """One histogram series as the reference builds and writes it: updateHistogram calls
    histogram.Set(b.Le, uint64(value)) for every bucket in CR order (metrics.go:380-390; a
    later equal le overwrites: SyncMap.Store, histogram.go:161-164); getOrRegisterHistogram
    passes the non-hidden le's as Buckets (metrics.go:143-149), NewHistogram sorts them
    (histogram.go:88); Write (histogram.go:107-148) walks the stored keys in ascending order.
    buckets: [(le, hidden)], values: float64 bucket values -> (bounds, counts incl. +Inf,
    sample count, sample sum)."""
    stored = {}
    for (le, _), v in zip(buckets, values):
        stored[le] = go_float64_to_uint64(v)
    upper = sorted(le for le, hidden in buckets if not hidden) + [float("inf")]
    cum = [0] * len(upper)
    idx = 0
    count = 0
    total = 0.0
    for le in sorted(stored):
        while idx < len(upper) and le > upper[idx]:
            idx += 1
            cum[idx] = (cum[idx] + count) % (1 << 64)
        cum[idx] = (cum[idx] + stored[le]) % (1 << 64)
        count = (count + stored[le]) % (1 << 64)
        total += le * float(stored[le])
    return upper[:-1], cum, count, total
