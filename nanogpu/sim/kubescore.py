"""How kube-scheduler turns extender priorities into a node choice (the stand-ins model it).

kube-scheduler (v1.18, the reference's k8s.io/kube-scheduler v0.18.0, /root/reference/go.mod:19;
extender configured with `"weight": 1`, /root/reference/README.md:43-58) scores every feasible
node as

    total = sum over score plugins (weight x 0..100)
          + sum over extenders (weight x priority x MaxNodeScore / MaxExtenderPriority)   [x 10]

and `selectHost` picks uniformly among the nodes with the highest total. The default plugins
whose scores differ between otherwise identical GPU nodes are NodeResourcesLeastAllocated
(prefers the emptiest node by CPU / memory requests) and NodeResourcesBalancedAllocation
(prefers CPU and memory used in the same proportion), weight 1 each. So an extender top score
is not always the node kube-scheduler binds: a one-point lead (x 10) loses to a node that is
more than 10 points emptier. This is what makes a priorities-time nomination wrong sometimes.

Pods here carry CPU / memory requests proportional to their GPU share (a GPU pod brings its
host threads and staging memory): `cpu_per_gpu` cores and `mem_per_gpu` bytes per whole
device, plus the HBM the pod requests mirrored in host memory.

Two more parts of kube-scheduler decide which nodes an extender sees and which it gets:
  * node sampling (generic_scheduler.go numFeasibleNodesToFind): with 100 nodes or more the
    in-tree filters stop after an adaptive share of feasible nodes (50 % - nodes/125, at
    least 5 % and 100 nodes; 42 % of 1,000), starting where the last cycle stopped, and only
    those are sent to the extender's filter;
  * PodTopologySpread's system default constraints for pods a ReplicaSet / StatefulSet /
    ReplicationController / Service selects: hostname maxSkew 3 and zone maxSkew 5, both
    ScheduleAnyway, plugin weight 2. Nodes without zone labels skip the zone term.
The native stand-in (native/src/schedsim.cpp) implements the same three models.
"""
from __future__ import annotations

import math
import random
from dataclasses import dataclass, field

MAX_NODE_SCORE = 100
MAX_EXTENDER_PRIORITY = 10
MIN_FEASIBLE_NODES = 100
MIN_FEASIBLE_PERCENT = 5
BASE_PERCENT = 50


def num_feasible_nodes_to_find(all_nodes: int, percentage: int = 0) -> int:
    """kube-scheduler's numFeasibleNodesToFind (percentageOfNodesToScore 0 = adaptive)."""
    if all_nodes < MIN_FEASIBLE_NODES:
        return all_nodes
    pct = percentage if percentage > 0 else max(MIN_FEASIBLE_PERCENT, BASE_PERCENT - all_nodes // 125)
    if pct >= 100:
        return all_nodes
    return max(MIN_FEASIBLE_NODES, all_nodes * pct // 100)


def spread_scores(counts: list[int], max_skew: int = 3) -> list[int]:
    """PodTopologySpread Score + NormalizeScore for the hostname constraint over the nodes
    being scored: raw = int(matching pods on the node x log(nodes + 2) + maxSkew - 1), then
    100 x (max + min - raw) / max (100 for every node when max is 0)."""
    w = math.log(len(counts) + 2)
    raw = [int(c * w + (max_skew - 1)) for c in counts]
    lo, hi = min(raw, default=0), max(raw, default=0)
    if hi == 0:
        return [MAX_NODE_SCORE] * len(raw)
    return [MAX_NODE_SCORE * (hi + lo - r) // hi for r in raw]


@dataclass
class KubeScoring:
    extender_weight: int = 1
    node_cpu_m: int = 256_000                 # 2 x 64-core EPYC, SMT: 256 threads
    node_mem: int = 3 << 40                   # 3 TiB host memory
    cpu_per_gpu_m: int = 24_000               # 24 threads per whole MI355X
    mem_per_gpu: int = 96 << 30
    least_weight: int = 1
    balanced_weight: int = 1
    spread_weight: int = 2                    # PodTopologySpread (system default constraints)
    spread_max_skew: int = 3
    sample_nodes: bool = True                 # numFeasibleNodesToFind
    percentage_of_nodes_to_score: int = 0
    rng: random.Random = field(default_factory=lambda: random.Random(0))
    next_start: int = 0                       # nextStartNodeIndex

    def feasible(self, n_nodes: int, fits) -> list[int]:
        """Indices of the nodes the in-tree filters pass to the extender: from nextStartNodeIndex,
        node by node, until numFeasibleNodesToFind have passed `fits(i)`."""
        if not n_nodes:
            return []
        want = num_feasible_nodes_to_find(n_nodes, self.percentage_of_nodes_to_score) if self.sample_nodes \
            else n_nodes
        out, processed = [], 0
        for k in range(n_nodes):
            if len(out) >= want:
                break
            i = (self.next_start + k) % n_nodes
            processed += 1
            if fits(i):
                out.append(i)
        self.next_start = (self.next_start + processed) % n_nodes
        return out

    def pod_requests(self, demand) -> tuple[int, int]:
        """(cpu millicores, memory bytes) of a pod whose containers request `demand`
        [(gpu-percent, hbm-mib), ...]."""
        cpu = mem = 0
        for d in demand:
            pct, mib = d[0], d[1]
            cpu += self.cpu_per_gpu_m * pct // 100
            mem += self.mem_per_gpu * pct // 100 + (mib << 20)
        return max(cpu, 100), max(mem, 64 << 20)

    def plugin_score(self, used: tuple[int, int], pod: tuple[int, int]) -> int:
        cpu, mem = used[0] + pod[0], used[1] + pod[1]
        cf, mf = min(1.0, cpu / self.node_cpu_m), min(1.0, mem / self.node_mem)
        least = int(((1 - cf) * MAX_NODE_SCORE + (1 - mf) * MAX_NODE_SCORE) / 2)
        balanced = int((1 - abs(cf - mf)) * MAX_NODE_SCORE)
        return self.least_weight * least + self.balanced_weight * balanced

    def total(self, ext_score: int, used: tuple[int, int], pod: tuple[int, int], spread: int = 0) -> int:
        """`spread`: the node's normalised PodTopologySpread score (spread_scores), or 0."""
        return (self.plugin_score(used, pod) + self.spread_weight * spread +
                self.extender_weight * ext_score * (MAX_NODE_SCORE // MAX_EXTENDER_PRIORITY))

    def select(self, totals: list[int]) -> int:
        """selectHost: uniformly random among the maxima (index into `totals`)."""
        best = max(totals)
        return self.rng.choice([i for i, t in enumerate(totals) if t == best])
