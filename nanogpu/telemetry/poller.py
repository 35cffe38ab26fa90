"""Load-aware scheduling inputs: per-metric periodic polls -> store -> ledger.

Reference: pkg/controller/node.go (syncMetricLoop :31-43 one goroutine per metric that
enqueues `node/metric` for every node each period, nodeWorker -> syncNode :85-109 with one
query per card, failures re-queued per key with rate limiting 10 s..360 s x5 :57-83 and
controller.go:35-36,126; node label `nvidia-device-enable=enable` :153-158). Here: one
cancellable ticker per metric (periods follow policy reloads), the same per-key queue (a
failing node/metric key backs off on its own while every other key keeps its period), one
PromQL query per node and metric for all its cards instead of one per card (MetricQuery.batch),
the AMD node selector by default (legacy label accepted), and the derived device load written
to the native ledger so filter/score never parse strings or load tzdata.
"""
from __future__ import annotations

import asyncio
import logging
import time

from .. import types as T
from ..config.policy import PolicySpec
from ..k8s import podutil as pu
from ..k8s.informer import WorkQueue
from .store import TelemetryStore, normalize_hbm_activity

log = logging.getLogger(__name__)
CLUSTER_KEY = "*"          # queue key prefix of a cluster-scoped metric (never a node name)


def is_gpu_node(node: dict, selectors: list[tuple[str, str]]) -> bool:
    labels = pu.node_labels(node)
    return any(labels.get(k) == v for k, v in selectors)


class LoadPoller:
    def __init__(self, state, prom, list_nodes, spec: PolicySpec | None = None,
                 selectors: list[tuple[str, str]] | None = None, concurrency: int = 32,
                 max_retries: int = 5, base_backoff_s: float = 10.0, max_backoff_s: float = 360.0,
                 metrics=None, get_node=None, forget_after: int = 3):
        self.state = state
        self.prom = prom
        self.list_nodes = list_nodes          # () -> list[node dict]
        # name -> node dict (the node informer's store lookup). Without it, a name index is
        # rebuilt once per period tick: never a scan of every node per node/metric key.
        self.get_node = get_node
        self._by_name: dict[str, dict] = {}
        # a learned streaming owner is forgotten only after this many passes in a row in which
        # every lone replica of it was measured cool
        self.forget_after = max(1, int(forget_after))
        self.spec = spec or PolicySpec()
        self.selectors = selectors or [T.AMD_GPU_NODE_LABEL, T.LEGACY_GPU_NODE_LABEL]
        self.store = TelemetryStore()
        # `node/metric` keys, rate-limited per key (the reference's nodeQueue)
        self.queue = WorkQueue("metrics", max_retries=max_retries, base_backoff=base_backoff_s,
                               max_backoff=max_backoff_s)
        self.concurrency = concurrency
        self.tasks: dict[str, asyncio.Task] = {}
        self.workers: list[asyncio.Task] = []
        self.errors = 0
        self.polls = 0        # successful node/metric syncs
        self.queries = 0
        self.hbm_threshold = self.spec.hbm_hot_threshold or T.HBM_HOT_THRESHOLD
        self.owners_learned = 0
        self.owners_forgotten = 0
        self.metrics = metrics      # obs.Metrics (stream_owners counter), optional

    # -------------------------------------------------------------- policy changes
    def on_policy(self, spec: PolicySpec) -> None:
        self.spec = spec
        self.hbm_threshold = spec.hbm_hot_threshold or T.HBM_HOT_THRESHOLD
        self.restart()

    def restart(self) -> None:
        for t in self.tasks.values():
            t.cancel()
        self.tasks.clear()
        if not self.workers:
            self.workers = [asyncio.ensure_future(self.queue.worker(self._sync_key))
                            for _ in range(self.concurrency)]
        for p in self.spec.sync_period:
            if p.period_s > 0:
                self.tasks[p.name] = asyncio.ensure_future(self._loop(p.name, p.period_s))

    async def stop(self) -> None:
        tasks = list(self.tasks.values()) + self.workers
        for t in tasks:
            t.cancel()
        for t in tasks:
            try:
                await t
            except (asyncio.CancelledError, Exception):
                pass
        self.tasks.clear()
        self.workers = []

    # -------------------------------------------------------------- polling
    async def _loop(self, metric: str, period: float) -> None:
        while True:
            if metric == T.GPU_HBM_ACTIVITY_METRIC:
                # a pass over the whole pod table (milliseconds at 100k pods): off the loop
                self.learn_owners(await asyncio.get_running_loop().run_in_executor(None, self._learn_pass))
            self.enqueue(metric)
            await asyncio.sleep(period)

    def _count(self, result: str) -> None:
        if self.metrics is not None:
            self.metrics.child(self.metrics.metric_polls, result).inc()

    def attribution_cutoff(self, now: float | None = None) -> float:
        """Pods recorded after this (time.monotonic) may postdate the samples behind the
        current HBM-hot marks: the marks come from the previous tick's query (one period ago),
        which averages `window` seconds before that. Such a pod is not blamed for a mark
        measured on the tenant it replaced."""
        q = self.spec.query_for(T.GPU_HBM_ACTIVITY_METRIC)
        period = self.spec.period_of(T.GPU_HBM_ACTIVITY_METRIC)
        return (time.monotonic() if now is None else now) - (q.window_s() + period)

    def _learn_pass(self, now: float | None = None) -> tuple[int, int]:
        return self.state.ledger.learn_stream_owners(True, self.attribution_cutoff(now), self.forget_after,
                                                     self.spec.learn_curve())

    def learn_owners(self, counts: tuple[int, int] | None = None, now: float | None = None) -> tuple[int, int]:
        """Streaming owners from the last period's marks (Ledger::learn_stream_owners): a
        device measured HBM-hot while it held one pod alone makes that pod's controlling owner
        (ReplicaSet, Job, ...) streaming, so the owner's next unannotated pods are placed as
        memory-bound; an owner alone on a device that is no longer hot is forgotten. One pass
        over the ledger per HBM-activity period, off the GIL."""
        learned, forgotten = counts if counts is not None else self._learn_pass(now)
        self.owners_learned += learned
        self.owners_forgotten += forgotten
        if self.metrics is not None:
            self.metrics.child(self.metrics.stream_owners, "learned").inc(learned)
            self.metrics.child(self.metrics.stream_owners, "forgotten").inc(forgotten)
        return learned, forgotten

    def cluster_scoped(self, metric: str) -> bool:
        return self.spec.metrics_scope == "cluster" and self.spec.query_for(metric).cluster is not None

    def enqueue(self, metric: str) -> int:
        """One period tick (reference syncMetric, node.go:45-55): every GPU node's key, or the
        one cluster-wide key `*/metric` under `metricsScope: cluster`."""
        if self.cluster_scoped(metric):
            self.queue.add(f"{CLUSTER_KEY}/{metric}")
            return 1
        n = 0
        by_name = {}
        for node in self.list_nodes():
            name = pu.meta(node).get("name", "")
            by_name[name] = node
            if is_gpu_node(node, self.selectors):
                self.queue.add(f"{name}/{metric}")
                n += 1
        self._by_name = by_name
        return n

    def _node(self, name: str) -> dict | None:
        if self.get_node is not None:
            return self.get_node(name)
        return self._by_name.get(name)

    async def sync_metric(self, metric: str) -> None:
        """Polls `metric` on every GPU node now (no retries): tests and one-shot use."""
        if self.cluster_scoped(metric):
            await self.sync_cluster(metric)
            return
        await asyncio.gather(*(self.sync_node(n, metric) for n in self.list_nodes()
                               if is_gpu_node(n, self.selectors)), return_exceptions=True)

    async def _sync_key(self, key: str) -> None:
        name, _, metric = key.rpartition("/")
        if name == CLUSTER_KEY:
            await self.sync_cluster(metric)
            return
        node = self._node(name)
        if node is None or not is_gpu_node(node, self.selectors):
            return                                   # node gone or no longer a GPU node
        await self.sync_node(node, metric)

    async def sync_node(self, node: dict, metric: str) -> None:
        """All cards of one node for one metric; raises on a failed query (the queue backs
        the key off; nothing else waits for it)."""
        name = pu.meta(node).get("name", "")
        entry = self.state.node_entry(name)
        n_dev = len(entry.topology.devices) if entry else pu.node_gpu_count(node)
        q = self.spec.query_for(metric)
        try:
            if q.batch:
                self.queries += 1
                for card, v in (await self.prom.query_node(name, metric, q)).items():
                    if 0 <= card < n_dev:
                        self.store.update(name, metric, card, v)
            else:
                for card in range(n_dev):
                    self.queries += 1
                    v = await self.prom.query_latest(name, metric, card, q)
                    if v is not None:
                        self.store.update(name, metric, card, v)
        except asyncio.CancelledError:
            raise
        except Exception as e:
            self.errors += 1
            self._count("error")
            log.debug("metric %s node %s: %s", metric, name, e)
            raise
        self.polls += 1
        self._count("ok")
        self.refresh_node(name, n_dev)

    async def sync_cluster(self, metric: str) -> None:
        """Every GPU node's cards for one metric from one query; raises on a failed query (the
        one key backs off). A node absent from the answer keeps its samples until they age out,
        as a node whose per-node query returned no series would."""
        q = self.spec.query_for(metric)
        try:
            self.queries += 1
            res = await self.prom.query_cluster(metric, q)
        except asyncio.CancelledError:
            raise
        except Exception as e:
            self.errors += 1
            self._count("error")
            log.debug("metric %s (cluster): %s", metric, e)
            raise
        self._count("ok")
        for node in self.list_nodes():
            if not is_gpu_node(node, self.selectors):
                continue
            name = pu.meta(node).get("name", "")
            entry = self.state.node_entry(name)
            n_dev = len(entry.topology.devices) if entry else pu.node_gpu_count(node)
            for card, v in res.get(name, {}).items():
                if 0 <= card < n_dev:
                    self.store.update(name, metric, card, v)
            self.polls += 1
            self.refresh_node(name, n_dev)

    def refresh_node(self, name: str, n_dev: int, now: float | None = None) -> None:
        # HBM activity marks streaming devices (Device::mem_hot); it is not part of the
        # reference's load sum
        periods = [(p.name, self.spec.active_duration(p.name)) for p in self.spec.sync_period
                   if p.name != T.GPU_HBM_ACTIVITY_METRIC]
        hbm_active = self.spec.active_duration(T.GPU_HBM_ACTIVITY_METRIC)
        cal = self._hbm_cal(name)
        for card in range(n_dev):
            self.state.set_load(name, card, self.store.device_usage(name, card, periods, now))
            # unpolled (or no longer polled) metric: the mark clears. The reading is put on the
            # classifier's scale through the device's own calibration (its agent's probe)
            busy = normalize_hbm_activity(self.store.hbm_activity(name, card, hbm_active, now), cal.get(card))
            self.state.set_mem_hot(name, card, busy >= self.hbm_threshold)
            self.state.set_mem_busy(name, card, busy)

    def _hbm_cal(self, name: str) -> dict[int, list]:
        """card -> its physical GPU's mem_busy calibration (GpuSpec.hbm_busy_cal), from the
        node's published topology; a partition shares its GPU's."""
        e = self.state.node_entry(name)
        if e is None or e.topology is None:
            return {}
        by_gpu = {g.index: g.hbm_busy_cal for g in e.topology.gpus if g.hbm_busy_cal}
        return {k: by_gpu[d.gpu] for k, d in enumerate(e.topology.devices) if d.gpu in by_gpu}

    def sweep_stale(self) -> None:
        """Re-derives loads so samples that aged out stop counting (called periodically)."""
        for name in self.store.nodes():
            e = self.state.node_entry(name)
            if e:
                self.refresh_node(name, len(e.topology.devices))
