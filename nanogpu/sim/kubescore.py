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
"""
from __future__ import annotations

import random
from dataclasses import dataclass, field

MAX_NODE_SCORE = 100
MAX_EXTENDER_PRIORITY = 10


@dataclass
class KubeScoring:
    extender_weight: int = 1
    node_cpu_m: int = 256_000                 # 2 x 64-core EPYC, SMT: 256 threads
    node_mem: int = 3 << 40                   # 3 TiB host memory
    cpu_per_gpu_m: int = 24_000               # 24 threads per whole MI355X
    mem_per_gpu: int = 96 << 30
    least_weight: int = 1
    balanced_weight: int = 1
    rng: random.Random = field(default_factory=lambda: random.Random(0))

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

    def total(self, ext_score: int, used: tuple[int, int], pod: tuple[int, int]) -> int:
        return (self.plugin_score(used, pod) +
                self.extender_weight * ext_score * (MAX_NODE_SCORE // MAX_EXTENDER_PRIORITY))

    def select(self, totals: list[int]) -> int:
        """selectHost: uniformly random among the maxima (index into `totals`)."""
        best = max(totals)
        return self.rng.choice([i for i, t in enumerate(totals) if t == best])
