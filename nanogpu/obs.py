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

from prometheus_client import CollectorRegistry, Counter, Gauge, Histogram, generate_latest

_BUCKETS = (5e-5, 1e-4, 2.5e-4, 5e-4, 1e-3, 2.5e-3, 5e-3, 1e-2, 2.5e-2, 5e-2, 0.1, 0.25, 0.5, 1.0, 2.5)


class Metrics:
    def __init__(self, registry: CollectorRegistry | None = None):
        self.registry = registry or CollectorRegistry()
        r = self.registry
        self.verb_latency = Histogram("nanogpu_verb_latency_seconds", "extender verb latency",
                                      ["verb"], buckets=_BUCKETS, registry=r)
        self.verb_total = Counter("nanogpu_verb_total", "extender verb calls", ["verb", "result"], registry=r)
        self.bind_phase = Histogram("nanogpu_bind_phase_seconds", "bind phases", ["phase"],
                                    buckets=_BUCKETS, registry=r)
        self.api_errors = Counter("nanogpu_api_errors_total", "API server errors", ["op", "code"], registry=r)
        self.pods_bound = Counter("nanogpu_pods_bound_total", "pods bound by this extender", registry=r)
        self.pods_released = Counter("nanogpu_pods_released_total", "pods released", registry=r)
        self.rollbacks = Counter("nanogpu_rollbacks_total", "reservations rolled back", registry=r)
        self.frag_pct = Gauge("nanogpu_frag_percent", "free gpu-percent on partially used devices / free",
                              registry=r)
        self.frag_mib = Gauge("nanogpu_frag_hbm_percent", "free HBM on partially used devices / free HBM",
                              registry=r)
        self.free_pct = Gauge("nanogpu_free_gpu_percent", "cluster free gpu-percent", registry=r)
        self.nodes = Gauge("nanogpu_nodes", "nodes in the ledger", registry=r)
        self.pods = Gauge("nanogpu_pods", "pods in the ledger", registry=r)
        self.workqueue_depth = Gauge("nanogpu_workqueue_depth", "controller queue depth", ["queue"], registry=r)

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
