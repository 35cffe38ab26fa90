"""Observability: Prometheus metrics, per-request trace ring, sampling profiler.

Reference: logging only — klog on every verb incl. full JSON results (routes.go:70-116),
`PrintStatus` dumps of every node (dealer.go:303-309), Go pprof routes (pprof.go:10-21),
no /metrics. Here the hot path records numbers, not log lines.
"""
from __future__ import annotations

import collections
import sys
import threading
import time
import traceback
from contextlib import contextmanager
from dataclasses import dataclass, field

import bisect

from prometheus_client import CollectorRegistry, Gauge, generate_latest
from prometheus_client.core import CounterMetricFamily, HistogramMetricFamily

_BUCKETS = (5e-5, 1e-4, 2.5e-4, 5e-4, 1e-3, 2.5e-3, 5e-3, 1e-2, 2.5e-2, 5e-2, 0.1, 0.25, 0.5, 1.0, 2.5)


# Counters and histograms of the request path. prometheus_client takes a lock and walks a
# value object per increment (9 increments per scheduled pod, about a fifth of the extender's
# Python time in the bench profile); these are plain numbers updated on the event-loop thread
# (every writer runs there) and turned into metric families only when /metrics is scraped.
class _CounterChild:
    __slots__ = ("v",)

    def __init__(self):
        self.v = 0.0

    def inc(self, n: float = 1.0) -> None:
        self.v += n


class _HistChild:
    __slots__ = ("counts", "sum", "n")

    def __init__(self, nb: int):
        self.counts = [0] * (nb + 1)     # last slot: +Inf
        self.sum = 0.0
        self.n = 0

    def observe(self, v: float) -> None:
        self.counts[bisect.bisect_left(_BUCKETS, v)] += 1
        self.sum += v
        self.n += 1


class LoopCounter:
    def __init__(self, name: str, doc: str, labelnames=(), registry: CollectorRegistry | None = None):
        self.name, self.doc, self.labelnames = name, doc, tuple(labelnames)
        self.children: dict[tuple, _CounterChild] = {}
        if not self.labelnames:
            self.children[()] = _CounterChild()
        if registry is not None:
            registry.register(self)

    def labels(self, *values) -> _CounterChild:
        key = tuple(str(v) for v in values)
        c = self.children.get(key)
        if c is None:
            c = self.children[key] = _CounterChild()
        return c

    def inc(self, n: float = 1.0) -> None:
        self.children[()].v += n

    def collect(self):
        base = self.name[:-6] if self.name.endswith("_total") else self.name
        fam = CounterMetricFamily(base, self.doc, labels=list(self.labelnames))
        for key, c in self.children.items():
            fam.add_metric(list(key), c.v)
        yield fam


class LoopHistogram:
    def __init__(self, name: str, doc: str, labelnames=(), registry: CollectorRegistry | None = None):
        self.name, self.doc, self.labelnames = name, doc, tuple(labelnames)
        self.children: dict[tuple, _HistChild] = {}
        if registry is not None:
            registry.register(self)

    def labels(self, *values) -> _HistChild:
        key = tuple(str(v) for v in values)
        c = self.children.get(key)
        if c is None:
            c = self.children[key] = _HistChild(len(_BUCKETS))
        return c

    def collect(self):
        fam = HistogramMetricFamily(self.name, self.doc, labels=list(self.labelnames))
        for key, c in self.children.items():
            acc, buckets = 0, []
            for le, k in zip([*map(str, _BUCKETS), "+Inf"], c.counts):
                acc += k
                buckets.append((le, acc))
            fam.add_metric(list(key), buckets, c.sum)
        yield fam


class Metrics:
    def __init__(self, registry: CollectorRegistry | None = None):
        self.registry = registry or CollectorRegistry()
        r = self.registry
        self.verb_latency = LoopHistogram("nanogpu_verb_latency_seconds", "extender verb latency", ["verb"], r)
        self.verb_total = LoopCounter("nanogpu_verb_total", "extender verb calls", ["verb", "result"], r)
        self.bind_phase = LoopHistogram("nanogpu_bind_phase_seconds", "bind phases", ["phase"], r)
        self.api_errors = LoopCounter("nanogpu_api_errors_total", "API server errors", ["op", "code"], r)
        self.pods_bound = LoopCounter("nanogpu_pods_bound_total", "pods bound by this extender", registry=r)
        self.pods_released = LoopCounter("nanogpu_pods_released_total", "pods released", registry=r)
        self.pods_reaccounted = LoopCounter("nanogpu_pods_reaccounted_total",
                                            "bound pods moved to the devices kubelet ran them on (agent reconciliation)",
                                            registry=r)
        self.rollbacks = LoopCounter("nanogpu_rollbacks_total", "reservations rolled back", registry=r)
        self.frag_pct = Gauge("nanogpu_frag_percent", "free gpu-percent on partially used devices / free",
                              registry=r)
        self.frag_mib = Gauge("nanogpu_frag_hbm_percent", "free HBM on partially used devices / free HBM",
                              registry=r)
        self.free_pct = Gauge("nanogpu_free_gpu_percent", "cluster free gpu-percent", registry=r)
        self.nodes = Gauge("nanogpu_nodes", "nodes in the ledger", registry=r)
        self.pods = Gauge("nanogpu_pods", "pods in the ledger", registry=r)
        self.workqueue_depth = Gauge("nanogpu_workqueue_depth", "controller queue depth", ["queue"], registry=r)
        self.stream_owners = LoopCounter("nanogpu_stream_owners_total",
                                         "owners learned / forgotten as HBM-streaming (telemetry)", ["event"], r)
        self.metric_polls = LoopCounter("nanogpu_metric_queries_total", "PromQL queries of the load poller",
                                        ["result"], r)

        self._children: dict = {}

    def child(self, metric, *labels):
        """Cached labelled child (prometheus_client's .labels() costs a lock + dict walk)."""
        key = (id(metric), labels)
        c = self._children.get(key)
        if c is None:
            c = self._children[key] = metric.labels(*labels)
        return c

    def render(self) -> bytes:
        return generate_latest(self.registry)


@dataclass
class Span:
    verb: str
    pod: str
    start: float
    dur: float = 0.0
    ok: bool = True
    note: str = ""
    phases: dict = field(default_factory=dict)

    def as_dict(self) -> dict:
        return {"verb": self.verb, "pod": self.pod, "start": self.start, "dur_ms": round(self.dur * 1e3, 4),
                "ok": self.ok, "note": self.note,
                "phases_ms": {k: round(v * 1e3, 4) for k, v in self.phases.items()}}


class Tracer:
    """Ring buffer of the last N request spans (GET /debug/trace)."""

    def __init__(self, capacity: int = 4096):
        self.buf: collections.deque[Span] = collections.deque(maxlen=capacity)

    @contextmanager
    def span(self, verb: str, pod: str = ""):
        s = Span(verb, pod, time.time())
        t0 = time.perf_counter()
        try:
            yield s
        except Exception as e:
            s.ok = False
            s.note = repr(e)
            raise
        finally:
            s.dur = time.perf_counter() - t0
            self.buf.append(s)

    def dump(self, limit: int = 512, verb: str | None = None) -> list[dict]:
        out = [s.as_dict() for s in list(self.buf) if verb is None or s.verb == verb]
        return out[-limit:]


def thread_stacks() -> str:
    """Goroutine-dump equivalent (reference /debug/pprof/goroutine)."""
    frames = sys._current_frames()
    names = {t.ident: t.name for t in threading.enumerate()}
    out = []
    for tid, fr in frames.items():
        out.append(f"--- thread {names.get(tid, tid)} ({tid})\n" + "".join(traceback.format_stack(fr)))
    return "\n".join(out)


def sample_profile(seconds: float = 5.0, interval: float = 0.005, top: int = 40) -> str:
    """Statistical profiler over all threads (reference /debug/pprof/profile)."""
    counts: collections.Counter = collections.Counter()
    me = threading.get_ident()
    deadline = time.monotonic() + seconds
    samples = 0
    while time.monotonic() < deadline:
        for tid, fr in sys._current_frames().items():
            if tid == me:
                continue
            stack = []
            f = fr
            while f is not None and len(stack) < 12:
                stack.append(f"{f.f_code.co_filename.rsplit('/', 1)[-1]}:{f.f_code.co_name}:{f.f_lineno}")
                f = f.f_back
            counts[" <- ".join(stack[:6])] += 1
        samples += 1
        time.sleep(interval)
    lines = [f"samples={samples} interval={interval}s"]
    for stack, n in counts.most_common(top):
        lines.append(f"{n:6d} {stack}")
    return "\n".join(lines)


def _maps() -> list[tuple[int, int, int, str]]:
    """(start, end, file offset, path) of this process's file-backed executable mappings."""
    out = []
    with open("/proc/self/maps") as f:
        for ln in f:
            parts = ln.split(None, 5)
            if len(parts) < 6 or "x" not in parts[1]:
                continue
            a, b = (int(x, 16) for x in parts[0].split("-"))
            out.append((a, b, int(parts[2], 16), parts[5].strip()))
    out.sort()
    return out


def _symbolize(pcs: set[int]) -> dict[int, str]:
    """pc -> "function (object)" through /proc/self/maps and addr2line (llvm-symbolizer when
    binutils is missing); unmapped or anonymous code keeps its address."""
    import os
    import shutil
    import subprocess

    maps = _maps()
    starts = [m[0] for m in maps]
    by_obj: dict[str, list[tuple[int, int]]] = collections.defaultdict(list)
    names: dict[int, str] = {}
    for pc in pcs:
        i = bisect.bisect_right(starts, pc) - 1
        if i < 0 or pc >= maps[i][1]:
            names[pc] = hex(pc)               # anonymous code (a JIT, a trampoline)
            continue
        if not maps[i][3].startswith("/"):
            names[pc] = maps[i][3]            # [vdso]: a clock read or its syscall fallback
            continue
        a, _b, off, path = maps[i]
        by_obj[path].append((pc, pc - a + off))
    tool = shutil.which("addr2line") or shutil.which("llvm-addr2line") or "/opt/rocm/lib/llvm/bin/llvm-addr2line"
    for path, items in by_obj.items():
        obj = os.path.basename(path)
        fns = []
        if os.path.exists(tool):
            try:
                r = subprocess.run([tool, "-f", "-C", "-e", path] + [hex(o) for _pc, o in items],
                                   capture_output=True, text=True, timeout=60)
                lines = r.stdout.splitlines()
                fns = lines[0::2] if len(lines) == 2 * len(items) else []
            except (OSError, subprocess.SubprocessError):
                fns = []
        for k, (pc, o) in enumerate(items):
            fn = fns[k] if k < len(fns) and fns[k] != "??" else f"+{o:#x}"
            names[pc] = f"{fn.split('(')[0][:90]} ({obj})"
    return names


def cpu_profile(samples: list[tuple[int, int, int]], top: int = 25) -> dict:
    """Per thread group (the bench's groups: main, ngpu-fe, ngpu-wr-io, ...), the share of
    samples in each function, from the native sampler (nanogpu._native.sampler_stop). A leaf in
    a libc system-call stub (send, recv, epoll_wait, ...) is the kernel time of that call. libc's
    internal routines (memcpy, memchr, malloc's) have no exported symbol: addr2line names them
    after the nearest exported one (e.g. __nss_database_lookup)."""
    import os

    comm: dict[int, str] = {}
    pid = os.getpid()
    for tid in {s[2] for s in samples}:
        try:
            with open(f"/proc/{pid}/task/{tid}/comm") as f:
                c = f.read().strip()
        except OSError:
            c = "exited"
        comm[tid] = "main" if tid == pid else (c.rstrip("0123456789") if c.startswith("ngpu-") else "other")
    names = _symbolize({s[0] for s in samples})
    groups: dict[str, collections.Counter] = collections.defaultdict(collections.Counter)
    for pc, _caller, tid in samples:
        groups[comm[tid]][names[pc]] += 1
    out = {"samples": len(samples)}
    for g, cnt in sorted(groups.items(), key=lambda kv: -sum(kv[1].values())):
        n = sum(cnt.values())
        out[g] = {"samples": n, "top": [[name, round(100.0 * k / n, 1)] for name, k in cnt.most_common(top)]}
    return out
