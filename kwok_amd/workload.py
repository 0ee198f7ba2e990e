"""Synthetic clusters for the BASELINE.json configurations.

Objects follow kwokctl's resource templates (kustomize/kwokctl/resource/{node,pod}.yaml:
nodes with the 8 standard labels and 3 annotations and no status, pods with one
``container-0`` busybox container in namespace ``default``).  A cluster is stored as a
small list of *variants* plus a per-object variant index, which is how the host interns
100M-pod clusters; ``materialize`` expands a small cluster into full objects for the
oracle.  Everything is seeded (default cluster seed 0x6b776f6b = "kwok").
"""
from __future__ import annotations

import copy
import os
from dataclasses import dataclass, field
from typing import Dict, List, Optional, Tuple

import numpy as np

CLUSTER_SEED = 0x6B776F6B
# the default Stage CRs kwok ships (kustomize/stage/**, byte-identical copies; the reference embeds
# them, kustomize/stage/*/embed.go)
STAGE_DIR = os.path.join(os.path.dirname(os.path.abspath(__file__)), "stages")
# the default usage / Metric CRs (kustomize/metrics/**)
METRICS_DIR = os.path.join(os.path.dirname(os.path.abspath(__file__)), "metrics")

POD_FAST = ["pod/fast/pod-ready.yaml", "pod/fast/pod-complete.yaml", "pod/fast/pod-delete.yaml"]
POD_GENERAL = ["pod/general/pod-create.yaml", "pod/general/pod-init-container-running.yaml",
               "pod/general/pod-init-container-completed.yaml", "pod/general/pod-ready.yaml",
               "pod/general/pod-complete.yaml", "pod/general/pod-remove-finalizer.yaml",
               "pod/general/pod-delete.yaml"]
POD_CHAOS = ["pod/chaos/pod-container-running-failed.yaml", "pod/chaos/pod-init-container-running-failed.yaml"]
NODE_FAST = ["node/fast/node-initialize.yaml"]
NODE_HEARTBEAT = ["node/heartbeat/node-heartbeat.yaml"]
NODE_HEARTBEAT_LEASE = ["node/heartbeat-with-lease/node-heartbeat-with-lease.yaml"]
NODE_CHAOS = ["node/chaos/node-not-ready.yaml"]

# override annotation values drawn by C2
OVERRIDE_VALUES = ["2", "0x10", "010", "1_0", "abc", "", "500ms", "1s", "2006-01-02T15:04:05Z"]
GENERAL_NAMES = ["pod-create", "pod-init-container-running", "pod-init-container-completed", "pod-ready",
                 "pod-complete", "pod-remove-finalizer", "pod-delete"]


def stage_paths(names: List[str]) -> List[str]:
    return [os.path.join(STAGE_DIR, n) for n in names]


def node_object(name: str, labels: Optional[dict] = None, annotations: Optional[dict] = None) -> dict:
    lab = {"beta.kubernetes.io/arch": "amd64", "beta.kubernetes.io/os": "linux", "kubernetes.io/arch": "amd64",
           "kubernetes.io/hostname": name, "kubernetes.io/os": "linux", "kubernetes.io/role": "agent",
           "node-role.kubernetes.io/agent": "", "type": "kwok"}
    lab.update(labels or {})
    ann = {"kwok.x-k8s.io/node": "fake", "node.alpha.kubernetes.io/ttl": "0",
           "metrics.k8s.io/resource-metrics-path": f"/metrics/nodes/{name}/metrics/resource"}
    ann.update(annotations or {})
    return {"apiVersion": "v1", "kind": "Node", "metadata": {"name": name, "annotations": ann, "labels": lab},
            "spec": {"podCIDR": "10.0.0.1/24"},
            "status": {"allocatable": {"cpu": "32", "memory": "256Gi", "pods": "110"},
                       "capacity": {"cpu": "32", "memory": "256Gi", "pods": "110"},
                       "nodeInfo": {"architecture": "amd64", "operatingSystem": "linux"}}}


def pod_object(name: str, node: str, job: bool = False, init: int = 0, containers: int = 1,
               labels: Optional[dict] = None, annotations: Optional[dict] = None,
               deletion: Optional[str] = None) -> dict:
    md: dict = {"name": name, "namespace": "default"}
    if job:
        md["ownerReferences"] = [{"apiVersion": "batch/v1", "kind": "Job", "name": f"job-{name}", "uid": f"uid-{name}"}]
    if labels:
        md["labels"] = dict(labels)
    if annotations:
        md["annotations"] = dict(annotations)
    if deletion:
        md["deletionTimestamp"] = deletion
    spec: dict = {"containers": [{"name": f"container-{i}", "image": "busybox"} for i in range(containers)],
                  "hostNetwork": False, "nodeName": node}
    if init:
        spec["initContainers"] = [{"name": f"init-{i}", "image": "busybox"} for i in range(init)]
    return {"apiVersion": "v1", "kind": "Pod", "metadata": md, "spec": spec}


@dataclass
class KindSet:
    """Objects of one kind as variants + per-object variant index."""
    variants: List[dict]
    index: np.ndarray                       # int32 [n]
    name_fmt: str = "obj-{i}"
    node_of: Optional[np.ndarray] = None    # pods: owning node id [n]

    def __len__(self):
        return len(self.index)

    def materialize(self, lo: int = 0, hi: Optional[int] = None, node_name_fmt: str = "node-{i}") -> List[dict]:
        hi = len(self.index) if hi is None else hi
        out = []
        for i in range(lo, hi):
            o = copy.deepcopy(self.variants[int(self.index[i])])
            name = self.name_fmt.format(i=i)
            o["metadata"]["name"] = name
            if self.node_of is not None:
                o["spec"]["nodeName"] = node_name_fmt.format(i=int(self.node_of[i]))
            if o["metadata"].get("ownerReferences"):
                for r in o["metadata"]["ownerReferences"]:
                    r["name"], r["uid"] = f"job-{name}", f"uid-{name}"
            out.append(o)
        return out


@dataclass
class Cluster:
    config: str
    nodes: KindSet
    pods: KindSet
    node_ptr: np.ndarray                    # pods are node-sorted: node j owns [node_ptr[j], node_ptr[j+1])
    pod_stage_files: List[str]
    node_stage_files: List[str]
    usage_keys: Optional[np.ndarray] = None
    usage_cpu: Optional[np.ndarray] = None
    usage_mem: Optional[np.ndarray] = None
    meta: Dict[str, object] = field(default_factory=dict)


def _pods_per_node(n_nodes: int, n_pods: int) -> np.ndarray:
    base = np.full(n_nodes, n_pods // n_nodes, dtype=np.int64)
    base[: n_pods % n_nodes] += 1
    return base


def _c2_override_sets(rng, n_over: int = 32) -> List[dict]:
    """C2's override-annotation sets: 3 stages x {weight, delay, jitter-delay} per set."""
    out = []
    for _ in range(n_over):
        ann = {}
        for st in rng.choice(GENERAL_NAMES, size=3, replace=False):
            kind = rng.choice(["weight", "delay", "jitter-delay"])
            ann[f"{st}.stage.kwok.x-k8s.io/{kind}"] = str(rng.choice(OVERRIDE_VALUES))
        out.append(ann)
    return out


def _splitmix64(x: np.ndarray) -> np.ndarray:
    x = (x + np.uint64(0x9E3779B97F4A7C15)).astype(np.uint64)
    x = ((x ^ (x >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)).astype(np.uint64)
    x = ((x ^ (x >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)).astype(np.uint64)
    return x ^ (x >> np.uint64(31))


def _unit(ids: np.ndarray, seed: int, salt: int) -> np.ndarray:
    h = _splitmix64(ids ^ np.uint64((seed ^ (salt * 0x2545F4914F6CDD1D)) & 0xFFFFFFFFFFFFFFFF))
    return (h >> np.uint64(11)).astype(np.float64) * (1.0 / (1 << 53)), h


def c2_pod_variants(pod_lo: int, pod_hi: int, seed: int = CLUSTER_SEED, now_s: int = 1_700_000_000,
                    job_frac: float = 0.1) -> Tuple[List[dict], np.ndarray]:
    """The C2 pod mix (pod-general + chaos: 20 % with 1-2 init containers, 10 % override
    annotations, 5 % chaos label, 10 % deletionTimestamp, job_frac Job-owned) for global pods
    [pod_lo, pod_hi) at any scale: every attribute is a hash of the GLOBAL pod id, so every
    sharding of the cluster sees the same objects (vectorised; make_cluster's per-pod draw is
    the small-cluster form of the same mix)."""
    over_sets = _c2_override_sets(np.random.default_rng(seed))
    del_ts = np.datetime_as_string(np.datetime64(now_s + 30, "s")) + "Z"
    n = pod_hi - pod_lo
    code = np.empty(n, dtype=np.int32)
    chunk = 1 << 24
    for a in range(pod_lo, pod_hi, chunk):
        b = min(pod_hi, a + chunk)
        ids = np.arange(a, b, dtype=np.uint64)
        job = _unit(ids, seed, 1)[0] < job_frac
        u2, h2 = _unit(ids, seed, 2)
        init = np.where(u2 < 0.2, 1 + (h2 & np.uint64(1)).astype(np.int64), 0)
        u4, h4 = _unit(ids, seed, 4)
        over = np.where(u4 < 0.1, (h4 % np.uint64(len(over_sets))).astype(np.int64), -1)
        chaos = np.where(_unit(ids, seed, 6)[0] < 0.05, np.where(init > 0, 2, 1), 0)
        dele = _unit(ids, seed, 7)[0] < 0.1
        code[a - pod_lo:b - pod_lo] = job + 2 * (init + 3 * ((over + 1) + 33 * (chaos + 3 * dele)))
    present = np.zeros(2 * 3 * 33 * 3 * 2, dtype=bool)
    present[code] = True
    ids_of = np.cumsum(present) - 1
    variants = []
    for c in np.flatnonzero(present):
        c = int(c)
        job, r = c % 2, c // 2
        init, r = r % 3, r // 3
        over, r = r % 33 - 1, r // 33
        chaos, dele = r % 3, r // 3
        labels = None
        if chaos == 1:
            labels = {"pod-container-running-failed.stage.kwok.x-k8s.io": "true"}
        elif chaos == 2:
            labels = {"pod-init-container-running-failed.stage.kwok.x-k8s.io": "true"}
        variants.append(pod_object("p", "n", job=bool(job), init=init, labels=labels,
                                   annotations=over_sets[over] if over >= 0 else None,
                                   deletion=del_ts if dele else None))
    return variants, ids_of[code].astype(np.int32)


def make_cluster(config: str, n_nodes: int, n_pods: int, seed: int = CLUSTER_SEED, now_s: int = 1_700_000_000,
                 job_frac: float = 0.1) -> Cluster:
    """Configs C1..C5 (BASELINE.json `configs`)."""
    rng = np.random.default_rng(seed)
    ppn = _pods_per_node(n_nodes, n_pods)
    node_ptr = np.zeros(n_nodes + 1, dtype=np.int64)
    np.cumsum(ppn, out=node_ptr[1:])
    node_of = np.repeat(np.arange(n_nodes, dtype=np.int64), ppn)

    nodes = KindSet(variants=[node_object("node")], index=np.zeros(n_nodes, dtype=np.int32), name_fmt="node-{i}")
    if config in ("C1", "C5", "C3"):
        pod_vars = [pod_object("p", "n"), pod_object("p", "n", job=True)]
        pidx = (rng.random(n_pods) < job_frac).astype(np.int32)
        pod_files, node_files = POD_FAST, NODE_FAST + NODE_HEARTBEAT
        if config == "C3":
            pod_files = []
    elif config == "C2":
        # pod-general 7 + pod-chaos 2: 20% with 1-2 init containers, 10% override annotations,
        # 5% chaos label, 10% deletionTimestamp = now + 30 s (second precision)
        del_ts = np.datetime_as_string(np.datetime64(now_s + 30, "s")) + "Z"
        n_over = 32
        over_sets = _c2_override_sets(rng, n_over)
        key_to_var: Dict[Tuple, int] = {}
        pod_vars = []
        job = rng.random(n_pods) < job_frac
        init = np.where(rng.random(n_pods) < 0.2, rng.integers(1, 3, n_pods), 0)
        over = np.where(rng.random(n_pods) < 0.1, rng.integers(0, n_over, n_pods), -1)
        chaos_r = rng.random(n_pods)
        chaos = np.where(chaos_r < 0.05, np.where(init > 0, 2, 1), 0)
        dele = rng.random(n_pods) < 0.1
        pidx = np.zeros(n_pods, dtype=np.int32)
        for i in range(n_pods):
            k = (bool(job[i]), int(init[i]), int(over[i]), int(chaos[i]), bool(dele[i]))
            v = key_to_var.get(k)
            if v is None:
                labels = None
                if k[3] == 1:
                    labels = {"pod-container-running-failed.stage.kwok.x-k8s.io": "true"}
                elif k[3] == 2:
                    labels = {"pod-init-container-running-failed.stage.kwok.x-k8s.io": "true"}
                v = key_to_var[k] = len(pod_vars)
                pod_vars.append(pod_object("p", "n", job=k[0], init=k[1], labels=labels,
                                           annotations=over_sets[k[2]] if k[2] >= 0 else None,
                                           deletion=del_ts if k[4] else None))
            pidx[i] = v
        pod_files, node_files = POD_GENERAL + POD_CHAOS, NODE_FAST + NODE_HEARTBEAT
    elif config == "C4":
        pod_vars = []
        pidx = np.zeros(n_pods, dtype=np.int32)
        pod_files, node_files = POD_FAST, NODE_FAST
    else:
        raise ValueError(config)
    pods = KindSet(variants=pod_vars, index=pidx, name_fmt="pod-{i}", node_of=node_of)
    cl = Cluster(config=config, nodes=nodes, pods=pods, node_ptr=node_ptr, pod_stage_files=stage_paths(pod_files),
                 node_stage_files=stage_paths(node_files), meta={"seed": seed, "now_s": now_s})
    if config == "C4":
        _usage_workload(cl, rng)
    return cl


CPU_VALUES = [f"{m}m" for m in (1, 2, 5, 10, 20, 50, 100, 200, 250, 500, 750)] + ["1", "1.5", "2", "3", "4"]
MEM_VALUES = [f"{x}Mi" for x in (1, 2, 4, 8, 16, 32, 64, 100, 128, 256, 512)] + ["1Gi", "1.5Gi", "2Gi", "3Gi", "4Gi"]


def _usage_workload(cl: Cluster, rng):
    """C4: containers/pod in {1..4}; 50% of pods annotated kwok.x-k8s.io/usage-cpu / -memory."""
    n = len(cl.pods.index)
    ncont = rng.integers(1, 5, n)
    annotated = rng.random(n) < 0.5
    cpu_i = rng.integers(0, len(CPU_VALUES), n)
    mem_i = rng.integers(0, len(MEM_VALUES), n)
    key_to_var: Dict[Tuple, int] = {}
    variants = []
    idx = np.zeros(n, dtype=np.int32)
    for i in range(n):
        k = (int(ncont[i]), int(cpu_i[i]) if annotated[i] else -1, int(mem_i[i]) if annotated[i] else -1)
        v = key_to_var.get(k)
        if v is None:
            ann = None
            if k[1] >= 0:
                ann = {"kwok.x-k8s.io/usage-cpu": CPU_VALUES[k[1]], "kwok.x-k8s.io/usage-memory": MEM_VALUES[k[2]]}
            v = key_to_var[k] = len(variants)
            variants.append(pod_object("p", "n", containers=k[0], annotations=ann))
        idx[i] = v
    cl.pods.variants = variants
    cl.pods.index = idx
