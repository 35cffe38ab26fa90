"""CPU placement of the control plane: one L3 domain (a Zen 5 CCD) per process group.

On the MI355X host (2 x EPYC 9575F, 16 CCDs of 8 cores, 32 MiB L3 each) the extender's
front-door threads, its Python loop and a co-located client exchange every request over
loopback TCP. Kept inside one CCD those hand-offs stay in one L3; spread by the kernel across
CCDs and sockets every wake-up pulls the request, the ledger lines and the socket buffers
across Infinity Fabric. Measured on the box (`bench.py`, 1k-pod bursts): unpinned 21.7k
pods/s, two CCDs 23.1k, one CCD 25.3k.

`pick_cpus()` returns the physical cores (first SMT sibling) of one L3 domain:
  * on the NUMA node of the GPU this process is paired with (the node agent / bench rank),
  * distinct per local rank when several ranks share a node,
  * otherwise the least busy domain (a shared host), counting the SMT siblings' load with the
    cores' own (another tenant on a sibling slows the core), skipping the one serving CPU 0.
Everything is read from sysfs / procfs; nothing here touches the GPU, so it can run before
worker processes are spawned.
"""
from __future__ import annotations

import os
import time
from pathlib import Path

SYS_CPU = Path("/sys/devices/system/cpu")


def _parse_list(text: str) -> list[int]:
    out: list[int] = []
    for part in text.strip().split(","):
        if not part:
            continue
        if "-" in part:
            a, b = part.split("-", 1)
            out.extend(range(int(a), int(b) + 1))
        else:
            out.append(int(part))
    return out


def _read(p: Path) -> str:
    try:
        return p.read_text()
    except OSError:
        return ""


def l3_domains(allowed: set[int] | None = None, root: Path = SYS_CPU) -> list[list[int]]:
    """Physical cores (lowest SMT sibling) grouped by shared L3, restricted to `allowed`."""
    allowed = allowed if allowed is not None else set(os.sched_getaffinity(0))
    seen: dict[tuple[int, ...], list[int]] = {}
    for cpu in sorted(allowed):
        base = root / f"cpu{cpu}"
        sib = _parse_list(_read(base / "topology" / "thread_siblings_list")) or [cpu]
        if min(sib) != cpu:
            continue                       # an SMT sibling: its core is counted once
        l3 = None
        for idx in sorted((base / "cache").glob("index*")):
            if _read(idx / "level").strip() == "3":
                l3 = tuple(_parse_list(_read(idx / "shared_cpu_list")))
                break
        key = l3 or (cpu,)
        seen.setdefault(key, []).append(cpu)
    return sorted(seen.values(), key=lambda cs: cs[0])


def numa_of_cpu(cpu: int, root: Path = SYS_CPU) -> int:
    for p in (root / f"cpu{cpu}").glob("node*"):
        try:
            return int(p.name[4:])
        except ValueError:
            pass
    return -1


def cpu_snapshot(stat: Path = Path("/proc/stat")) -> dict[int, tuple[int, int]]:
    """Per CPU (total, idle) jiffies since boot."""
    out = {}
    for line in _read(stat).splitlines():
        if line.startswith("cpu") and line[3:4].isdigit():
            f = line.split()
            v = [int(x) for x in f[1:]]
            idle = v[3] + (v[4] if len(v) > 4 else 0)
            out[int(f[0][3:])] = (sum(v), idle)
    return out


def busy_between(a: dict, b: dict, cpus) -> dict[int, float]:
    """Busy fraction of each CPU between two cpu_snapshot()s."""
    res = {}
    for c in cpus:
        if c in a and c in b:
            tot = b[c][0] - a[c][0]
            res[c] = 1.0 - (b[c][1] - a[c][1]) / tot if tot > 0 else 0.0
    return res


def _busy(cpus: list[int], window_s: float) -> dict[int, float]:
    a = cpu_snapshot()
    time.sleep(window_s)
    return busy_between(a, cpu_snapshot(), cpus)


def smt_siblings(cpus: list[int], root: Path | None = None) -> list[int]:
    """The other hardware threads of the cores `cpus` sit on (not in `cpus` themselves)."""
    root = root or SYS_CPU
    mine = set(cpus)
    out: set[int] = set()
    for c in cpus:
        out.update(_parse_list(_read(root / f"cpu{c}" / "topology" / "thread_siblings_list")))
    return sorted(out - mine)


def cpu_layout(cpus: list[int], root: Path | None = None) -> dict | None:
    """Physical-core / SMT layout of a pinned CPU set: the cores, their sibling threads,
    the L3 domains and NUMA nodes they span."""
    if not cpus:
        return None
    root = root or SYS_CPU
    cores = {tuple(_parse_list(_read(root / f"cpu{c}" / "topology" / "thread_siblings_list")) or [c])
             for c in cpus}
    return {"cpus": len(cpus), "physical_cores": len(cores), "smt_siblings": smt_siblings(cpus, root),
            "whole_cores": all(set(core) <= set(cpus) for core in cores),
            "numa": sorted({numa_of_cpu(c, root) for c in cpus})}


def busy_report(a: dict, b: dict, groups: dict[str, list[int]]) -> dict[str, float | None]:
    """Mean busy % of each named CPU group between two snapshots, plus the whole host."""
    out: dict[str, float | None] = {}
    for name, cs in groups.items():
        v = busy_between(a, b, cs)
        out[name] = round(100.0 * sum(v.values()) / len(v), 1) if v else None
    v = busy_between(a, b, list(b))
    out["host"] = round(100.0 * sum(v.values()) / len(v), 1) if v else None
    return out


def _domain_busy(dom: list[int], load: dict[int, float]) -> float:
    """A domain's load for placement: its cores and their SMT siblings alike. Another tenant
    on a sibling takes half of the core's issue slots; on the MI355X box runs whose siblings
    were 25-40 % busy lost 20-35 % of their pods/s (profiles/variance_r04.md)."""
    cpus = list(dom) + smt_siblings(dom)
    return sum(load.get(c, 0.0) for c in cpus) / len(cpus)


def pick_cpus(numa: int = -1, local_rank: int = 0, local_ranks_numa: list[int] | None = None,
              window_s: float = 0.25) -> list[int]:
    """Cores of one L3 domain for this process (see module docstring); [] when the host gives
    no usable topology (then leave the affinity alone)."""
    doms = l3_domains()
    if not doms:
        return []
    if numa >= 0:
        local = [d for d in doms if numa_of_cpu(d[0]) == numa]
        doms = local or doms
    if len(doms) > 1:
        doms = [d for d in doms if 0 not in d] or doms   # CPU 0 carries housekeeping work
    if local_ranks_numa and len(local_ranks_numa) > 1:
        # several ranks on this node: the k-th rank of a NUMA node takes its k-th domain
        k = sum(1 for r in range(local_rank) if local_ranks_numa[r] == numa)
        return doms[k % len(doms)]
    load = _busy([c for d in doms for c in list(d) + smt_siblings(d)], window_s)
    return min(doms, key=lambda d: (round(_domain_busy(d, load), 3), d[0]))


def pick_cpus_avoiding(taken: list[int], near: int = -1, window_s: float = 0.25) -> list[int]:
    """An L3 domain for a helper process (the bench's shared API server) that shares no core
    with `taken` (the ranks' domains, which may not be busy yet when the helper starts):
    a domain on NUMA node `near` that is less than half busy (every request and watch event
    crosses the socket otherwise: the box measured 28.7k pods/s with the API server on the far
    socket, 34.9k on the near one), else the least busy such domain; any domain if all are
    taken."""
    doms = l3_domains()
    if not doms:
        return []
    avoid = set(taken)
    free = [d for d in doms if not avoid.intersection(d)]
    if len(free) > 1:
        free = [d for d in free if 0 not in d] or free   # CPU 0 carries housekeeping work
    if not free:
        return pick_cpus()
    load = _busy([c for d in free for c in list(d) + smt_siblings(d)], window_s)

    def key(d):
        busy = _domain_busy(d, load)
        far = near >= 0 and numa_of_cpu(d[0]) != near
        return (busy >= 0.5, far, round(busy, 1), d[0])

    return min(free, key=key)


def domain_of(cpus: list[int]) -> list[int] | None:
    """The L3 domain (physical cores) `cpus` belong to, when they are one domain's cores."""
    for d in l3_domains():
        if set(cpus) <= set(d):
            return d
    return None


def quieter_domain(current: list[int], numa: int = -1, exclude: list[int] | None = None,
                   window_s: float = 0.3, threshold_cpus: float = 0.5) -> list[int] | None:
    """While this process group is idle (all of its CPU load is someone else's): when other
    tenants keep at least `threshold_cpus` CPUs' worth of the domain `current` sits on busy
    (its cores and their SMT siblings), the least busy other domain on NUMA node `numa` (none
    of `exclude`) with under half that load; else None. Moving away from contention, never
    holding CPUs. On the MI355X box one CPU of foreign work on the rank's cores cost 11 % of
    pods/s (profiles/variance_r04.md)."""
    doms = l3_domains()
    if numa >= 0:
        doms = [d for d in doms if numa_of_cpu(d[0]) == numa] or doms
    cur = next((d for d in doms if set(current) <= set(d)), None)
    if cur is None:
        return None
    avoid = set(exclude or [])
    others = [d for d in doms if d is not cur and 0 not in d and not avoid.intersection(d)]
    load = _busy([c for d in [cur] + others for c in list(d) + smt_siblings(d)], window_s)

    def cpus_busy(d: list[int]) -> float:   # CPUs' worth of work on the domain's hw threads
        return sum(load.get(c, 0.0) for c in list(d) + smt_siblings(d))

    here = cpus_busy(cur)
    if here < threshold_cpus or not others:
        return None
    best = min(others, key=lambda d: (cpus_busy(d), d[0]))
    return best if cpus_busy(best) < here / 2 else None


def proc_cpu_ns(pid: int) -> int:
    """CPU time of every thread of process `pid`, ns (/proc/<pid>/task/*/schedstat)."""
    total = 0
    try:
        tids = os.listdir(f"/proc/{pid}/task")
    except OSError:
        return 0
    for tid in tids:
        try:
            with open(f"/proc/{pid}/task/{tid}/schedstat") as f:
                total += int(f.read().split()[0])
        except (OSError, ValueError, IndexError):
            pass
    return total


class ContentionWatch:
    """Other tenants' load on a process group's L3 domain while the group is busy: the
    domain's hardware threads' busy time minus the group's own CPU time, between two calls
    of `check()`. When it reaches `threshold_cpus`, `check()` returns the quietest other domain
    on the same NUMA node (all of whose load is someone else's) if it carries under half as
    much; the caller moves there (`relocate`). Cooperative: it never holds CPUs."""

    def __init__(self, cpus: list[int], pids: list[int], numa: int = -1, exclude: list[int] | None = None,
                 threshold_cpus: float = 0.5):
        self.cpus, self.pids, self.numa = list(cpus), list(pids), numa
        self.exclude = list(exclude or [])
        self.threshold = threshold_cpus
        self.last = None
        self.hot = 0        # consecutive windows at or over the threshold (two are needed to move)
        self.moves = 0      # at most two moves per run: no chasing a tenant around the node

    def _sample(self):
        return cpu_snapshot(), sum(proc_cpu_ns(p) for p in self.pids), time.perf_counter()

    def check(self) -> tuple[float, list[int] | None]:
        """(other tenants' CPUs on our domain since the last call, a domain to move to or None)."""
        now = self._sample()
        prev, self.last = self.last, now
        if prev is None:
            return 0.0, None
        (a, own_a, t_a), (b, own_b, t_b) = prev, now
        wall = t_b - t_a
        if wall <= 0:
            return 0.0, None
        cur = domain_of(self.cpus) or list(self.cpus)
        hw = list(cur) + smt_siblings(cur)
        busy = busy_between(a, b, hw)
        foreign = max(0.0, sum(busy.values()) - (own_b - own_a) / 1e9 / wall)
        self.hot = self.hot + 1 if foreign >= self.threshold else 0
        if self.hot < 2 or self.moves >= 2:
            return foreign, None
        doms = l3_domains()
        if self.numa >= 0:
            doms = [d for d in doms if numa_of_cpu(d[0]) == self.numa] or doms
        avoid = set(self.exclude) | set(cur)
        others = [d for d in doms if 0 not in d and not avoid.intersection(d)]
        if not others:
            return foreign, None
        load = busy_between(a, b, [c for d in others for c in list(d) + smt_siblings(d)])
        best = min(others, key=lambda d: (sum(load.get(c, 0.0) for c in list(d) + smt_siblings(d)), d[0]))
        if sum(load.get(c, 0.0) for c in list(best) + smt_siblings(best)) >= foreign / 2:
            return foreign, None
        self.hot, self.moves = 0, self.moves + 1
        return foreign, best


def relocate(pids: list[int], cpus: list[int]) -> int:
    """Pins every thread of the processes `pids` to `cpus` (threads of a running process keep
    their own masks: each is set). Returns the threads moved."""
    n = 0
    for pid in pids:
        try:
            tids = os.listdir(f"/proc/{pid}/task")
        except OSError:
            continue
        for tid in tids:
            try:
                os.sched_setaffinity(int(tid), cpus)
                n += 1
            except OSError:
                pass
    return n


def apply(cpus: list[int]) -> bool:
    """Pins this process (and the threads and children it creates later) to `cpus`."""
    if not cpus:
        return False
    try:
        os.sched_setaffinity(0, cpus)
        return True
    except OSError:
        return False


def gpu_numa_nodes() -> list[int]:
    """NUMA node of each GPU in HIP enumeration order, from KFD sysfs only (no GPU init)."""
    try:
        from .native import core

        import json

        host = json.loads(core().discover_topology("", False))
        return [int(g.get("numa", -1)) for g in host.get("gpus", [])]
    except Exception:
        return []


def available_cores(cgroup_root: Path = Path("/sys/fs/cgroup")) -> float:
    """CPUs this process may actually use: its affinity mask, capped by a cgroup v2 CPU quota
    (`cpu.max`, what a pod's `limits.cpu` becomes) or a v1 CFS quota."""
    n = float(len(os.sched_getaffinity(0)))
    quota = _read(cgroup_root / "cpu.max").split()
    if len(quota) == 2 and quota[0] != "max":
        try:
            n = min(n, int(quota[0]) / max(1, int(quota[1])))
        except ValueError:
            pass
    else:
        q, p = _read(cgroup_root / "cpu" / "cpu.cfs_quota_us").strip(), _read(cgroup_root / "cpu" / "cpu.cfs_period_us").strip()
        if q.lstrip("-").isdigit() and p.isdigit() and int(q) > 0 and int(p) > 0:
            n = min(n, int(q) / int(p))
    return n


def busy_poll_fits(workers: int, frontend_threads: int, cores: float) -> bool:
    """Busy-polling front-door threads only pay off while each has a core of its own: every
    worker keeps its epoll threads plus its Python loop runnable (the same budget bench.py
    checks per rank). With fewer cores the spinning threads would steal them."""
    return cores >= workers * (frontend_threads + 1)
