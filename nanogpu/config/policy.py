"""policy.yaml schema + hot reload that actually reaches the scheduler.

Reference: pkg/dealer/type.go:16-33 (Policy/PolicySpec/Period/PriorityPolicy),
stats.go:13-28 (GetPolicyFromFile panics on unreadable file), context.go:19-59 (3 s mtime
poll). The reference reloads into a DSContext that nothing reads after startup:
main.go:118 copies the spec by value into the verb closures. Here the
watcher publishes an immutable snapshot and calls subscribers (cluster policy, telemetry
poller periods) on every change; a bad file keeps the last good snapshot instead of
panicking.

Schema (reference keys kept; MI355X additions are optional):
  apiVersion: v1
  kind: public-dynamic-scheduler
  spec:
    syncPeriod: [{name: gpu_core_usage_avg, period: 15s}, ...]
    priority:   [{name: ..., weight: ...}]          # parsed, informational (as reference)
    scheduling: {policy: binpack, compat: false, topologyWeight: 1.0, scoreNormalize: false}
    metrics:    {gpu_core_usage_avg: {query: '<PromQL with {node} {card}>', fallback: '...',
                                      batch: '<PromQL with {node}: all cards>', cardLabel: card}}
"""
from __future__ import annotations

import asyncio
import logging
import os
import re
from dataclasses import dataclass
from typing import Callable

import yaml

from .. import types as T

log = logging.getLogger(__name__)

_DUR = re.compile(r"(\d+(?:\.\d+)?)(ns|us|µs|ms|s|m|h)")
_UNIT = {"ns": 1e-9, "us": 1e-6, "µs": 1e-6, "ms": 1e-3, "s": 1.0, "m": 60.0, "h": 3600.0}


def parse_duration(v) -> float:
    """Go time.ParseDuration subset ("15s", "1m30s", "500ms"); bare numbers are seconds."""
    if isinstance(v, (int, float)):
        return float(v)
    s = str(v).strip()
    if not s:
        raise ValueError("empty duration")
    if re.fullmatch(r"\d+(\.\d+)?", s):
        return float(s)
    pos, total = 0, 0.0
    for m in _DUR.finditer(s):
        if m.start() != pos:
            raise ValueError(f"bad duration {v!r}")
        total += float(m.group(1)) * _UNIT[m.group(2)]
        pos = m.end()
    if pos != len(s):
        raise ValueError(f"bad duration {v!r}")
    return total


@dataclass(frozen=True)
class Period:
    name: str
    period_s: float


@dataclass(frozen=True)
class MetricQuery:
    query: str
    fallback: str | None = None
    # One query for every card of a node ({metric} {node}, no {card}); each series names its
    # card in the first of `card_labels` it carries. None: one query per card (the reference).
    batch: str | None = None
    card_labels: tuple[str, ...] = ("card",)
    # One query for every node and card ({metric} only); each series names its node in the
    # first of `node_labels` it carries. Used when the policy sets `metricsScope: cluster`.
    cluster: str | None = None
    node_labels: tuple[str, ...] = ("node",)

    def window_s(self) -> float:
        """The longest range selector in the query (`avg_over_time(...[1m])` -> 60 s): how far
        back the samples behind one answer reach. 0 for an instant query."""
        best = 0.0
        for q in (self.query, self.batch, self.cluster):
            for n, unit in re.findall(r"\[(\d+(?:\.\d+)?)(ms|s|m|h)\]", q or ""):
                best = max(best, float(n) * {"ms": 1e-3, "s": 1.0, "m": 60.0, "h": 3600.0}[unit])
        return best


# Reference query shapes (prometheus.go:70-76) as the default templates.
REFERENCE_QUERY = '{metric}{{node=~"{node}",card="{card}"}} /100'
REFERENCE_FALLBACK = '{metric}{{node="{node}",cardNode="{card}"}} /100'
# every card of the node in one query: series labelled `card` (the primary template) win
# over `cardNode` ones (the fallback's label)
REFERENCE_BATCH = '{metric}{{node=~"{node}"}} /100'
REFERENCE_CARD_LABELS = ("card", "cardNode")
REFERENCE_CLUSTER = '{metric} /100'
# AMD device-metrics-exporter shaped templates (gfx / memory-controller activity in %).
AMD_QUERIES = {
    T.GPU_CORE_USAGE_METRIC: MetricQuery(
        'avg_over_time(gpu_gfx_activity{{hostname="{node}",gpu_id="{card}"}}[1m]) / 100',
        batch='avg_over_time(gpu_gfx_activity{{hostname="{node}"}}[1m]) / 100', card_labels=("gpu_id",),
        cluster='avg_over_time(gpu_gfx_activity[1m]) / 100', node_labels=("hostname",)),
    T.GPU_MEMORY_USAGE_METRIC: MetricQuery(
        'gpu_used_vram{{hostname="{node}",gpu_id="{card}"}} / gpu_total_vram{{hostname="{node}",gpu_id="{card}"}}',
        batch='gpu_used_vram{{hostname="{node}"}} / gpu_total_vram{{hostname="{node}"}}', card_labels=("gpu_id",),
        cluster='gpu_used_vram / gpu_total_vram', node_labels=("hostname",)),
    T.GPU_HBM_ACTIVITY_METRIC: MetricQuery(
        'avg_over_time(gpu_umc_activity{{hostname="{node}",gpu_id="{card}"}}[1m]) / 100',
        batch='avg_over_time(gpu_umc_activity{{hostname="{node}"}}[1m]) / 100', card_labels=("gpu_id",),
        cluster='avg_over_time(gpu_umc_activity[1m]) / 100', node_labels=("hostname",)),
}

# The node agent's own exporter (nanogpu/agent/metrics.py); assumes the scrape config puts
# the node name in a `node` label (kubernetes_sd relabeling of __meta_kubernetes_pod_node_name).
AGENT_QUERIES = {
    T.GPU_CORE_USAGE_METRIC: MetricQuery(
        'avg_over_time(nanogpu_device_busy_percent{{node="{node}",device="{card}"}}[1m]) / 100',
        batch='avg_over_time(nanogpu_device_busy_percent{{node="{node}"}}[1m]) / 100', card_labels=("device",),
        cluster='avg_over_time(nanogpu_device_busy_percent[1m]) / 100'),
    T.GPU_MEMORY_USAGE_METRIC: MetricQuery(
        'nanogpu_device_vram_used_bytes{{node="{node}",device="{card}"}} / '
        'nanogpu_device_vram_total_bytes{{node="{node}",device="{card}"}}',
        batch='nanogpu_device_vram_used_bytes{{node="{node}"}} / nanogpu_device_vram_total_bytes{{node="{node}"}}',
        card_labels=("device",), cluster='nanogpu_device_vram_used_bytes / nanogpu_device_vram_total_bytes'),
    T.GPU_HBM_ACTIVITY_METRIC: MetricQuery(
        'avg_over_time(nanogpu_device_mem_busy_percent{{node="{node}",device="{card}"}}[1m]) / 100',
        batch='avg_over_time(nanogpu_device_mem_busy_percent{{node="{node}"}}[1m]) / 100', card_labels=("device",),
        cluster='avg_over_time(nanogpu_device_mem_busy_percent[1m]) / 100'),
}
PRESETS = {"amd": AMD_QUERIES, "nanogpu-agent": AGENT_QUERIES}


@dataclass(frozen=True)
class PolicySpec:
    sync_period: tuple[Period, ...] = ()
    priority: tuple[tuple[str, float], ...] = ()
    policy: str | None = None
    compat: bool | None = None
    topology_weight: float | None = None
    score_normalize: bool | None = None
    metrics: tuple[tuple[str, MetricQuery], ...] = ()
    # "node": one query per GPU node and metric each period, failures backed off per node (the
    # reference's node/metric keys). "cluster": one query per metric for the whole cluster.
    metrics_scope: str = "node"
    # HBM activity at or above which a device is marked streaming (types.HBM_HOT_THRESHOLD)
    hbm_hot_threshold: float | None = None
    # (share %, mem_busy %) of a lone streaming tenant on this fleet's GPUs (types.HBM_STREAMING_CURVE)
    hbm_streaming_curve: tuple[tuple[float, float], ...] | None = None

    def learn_curve(self) -> list[tuple[float, float]]:
        """The learner's per-share threshold (percent): HBM_LEARN_FRACTION of the streaming
        curve, never above the device threshold."""
        cap = 100.0 * (self.hbm_hot_threshold or T.HBM_HOT_THRESHOLD)
        return [(s, min(cap, T.HBM_LEARN_FRACTION * b)) for s, b in (self.hbm_streaming_curve or T.HBM_STREAMING_CURVE)]

    def period_of(self, name: str) -> float:
        for p in self.sync_period:
            if p.name == name and p.period_s > 0:
                return p.period_s
        return 0.0

    def active_duration(self, name: str) -> float:
        """stats.go:57-66: period + ExtenderActivePeriod (5 min); 0 when unknown."""
        p = self.period_of(name)
        return p + T.EXTENDER_ACTIVE_PERIOD_S if p > 0 else 0.0

    def query_for(self, name: str) -> MetricQuery:
        for k, q in self.metrics:
            if k == name:
                return q
        return MetricQuery(REFERENCE_QUERY, REFERENCE_FALLBACK, REFERENCE_BATCH, REFERENCE_CARD_LABELS,
                           REFERENCE_CLUSTER)


def parse_policy(text: str) -> PolicySpec:
    doc = yaml.safe_load(text) or {}
    spec = doc.get("spec") or {}
    periods = []
    for item in spec.get("syncPeriod") or []:
        periods.append(Period(str(item["name"]), parse_duration(item.get("period", 0))))
    prio = tuple((str(p.get("name", "")), float(p.get("weight", 0))) for p in spec.get("priority") or [])
    sch = spec.get("scheduling") or {}
    pol = sch.get("policy")
    if pol is not None and pol not in T.POLICIES:
        raise ValueError(f"unknown policy {pol!r}")
    metrics = []
    preset = spec.get("metricsPreset")
    if preset is not None:
        if preset not in PRESETS:
            raise ValueError(f"unknown metricsPreset {preset!r} (one of {sorted(PRESETS)})")
        metrics.extend(PRESETS[preset].items())
    for name, q in (spec.get("metrics") or {}).items():
        labels = q.get("cardLabel") or ["card"]
        nlabels = q.get("nodeLabel") or ["node"]
        metrics.append((name, MetricQuery(q["query"], q.get("fallback"), q.get("batch"),
                                          tuple([labels] if isinstance(labels, str) else labels),
                                          q.get("cluster"),
                                          tuple([nlabels] if isinstance(nlabels, str) else nlabels))))
    hot = spec.get("hbmHotThreshold")
    if hot is not None and not 0.0 < float(hot) <= 1.0:
        raise ValueError(f"hbmHotThreshold {hot!r} outside (0, 1]")
    curve = spec.get("hbmStreamingCurve")
    if curve is not None:
        curve = tuple(sorted((float(s), float(b)) for s, b in curve))
        if not curve or any(not (0 < s <= 100 and 0 <= b <= 100) for s, b in curve):
            raise ValueError(f"hbmStreamingCurve {spec.get('hbmStreamingCurve')!r}: [[share %, busy %], ...]")
    scope = spec.get("metricsScope", "node")
    if scope not in ("node", "cluster"):
        raise ValueError(f"unknown metricsScope {scope!r} (node or cluster)")
    return PolicySpec(
        sync_period=tuple(periods), priority=prio, policy=pol,
        compat=sch.get("compat"), topology_weight=sch.get("topologyWeight"),
        score_normalize=sch.get("scoreNormalize"), metrics=tuple(metrics), metrics_scope=scope,
        hbm_hot_threshold=None if hot is None else float(hot), hbm_streaming_curve=curve)


def load_policy(path: str) -> PolicySpec:
    with open(path) as f:
        return parse_policy(f.read())


class PolicyWatcher:
    """mtime poller (reference context.go:44-59 used 3 s); publishes snapshots to subscribers."""

    def __init__(self, path: str, interval_s: float = 3.0):
        self.path = path
        self.interval_s = interval_s
        self.spec = PolicySpec()
        self.mtime = 0.0
        self.subscribers: list[Callable[[PolicySpec], None]] = []
        self.reloads = 0
        self.errors = 0
        self._task: asyncio.Task | None = None

    def subscribe(self, fn: Callable[[PolicySpec], None]) -> None:
        self.subscribers.append(fn)

    def load_now(self) -> bool:
        try:
            st = os.stat(self.path)
        except OSError:
            return False
        if st.st_mtime <= self.mtime:
            return False
        try:
            spec = load_policy(self.path)
        except (OSError, ValueError, KeyError, TypeError, yaml.YAMLError) as e:
            self.errors += 1
            log.error("policy %s invalid, keeping previous: %s", self.path, e)
            self.mtime = st.st_mtime
            return False
        self.spec, self.mtime = spec, st.st_mtime
        self.reloads += 1
        for fn in self.subscribers:
            try:
                fn(spec)
            except Exception:
                log.exception("policy subscriber failed")
        return True

    async def run(self) -> None:
        while True:
            self.load_now()
            await asyncio.sleep(self.interval_s)

    def start(self) -> asyncio.Task:
        self._task = asyncio.ensure_future(self.run())
        return self._task
