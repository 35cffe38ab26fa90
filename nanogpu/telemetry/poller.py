"""Load-aware scheduling inputs: per-metric periodic polls -> store -> ledger.

Reference: pkg/controller/node.go (syncMetricLoop :31-43 one goroutine per metric that
never stops, syncNode :85-109 one query per card, retries 10 s..360 s x5 :68-83, node
label `nvidia-device-enable=enable` :153-158). Here: one cancellable task per metric,
periods follow policy reloads, AMD node selector by default (legacy label also
accepted), bounded query concurrency, and the derived device load is written to the
native ledger so filter/score never parse strings or load tzdata.
"""
from __future__ import annotations

import asyncio
import logging
import time

from .. import types as T
from ..config.policy import PolicySpec
from ..k8s import podutil as pu
from .store import TelemetryStore

log = logging.getLogger(__name__)


def is_gpu_node(node: dict, selectors: list[tuple[str, str]]) -> bool:
    labels = pu.node_labels(node)
    return any(labels.get(k) == v for k, v in selectors)


class LoadPoller:
    def __init__(self, state, prom, list_nodes, spec: PolicySpec | None = None,
                 selectors: list[tuple[str, str]] | None = None, concurrency: int = 32,
                 max_retries: int = 5, base_backoff_s: float = 10.0, max_backoff_s: float = 360.0):
        self.state = state
        self.prom = prom
        self.list_nodes = list_nodes          # () -> list[node dict]
        self.spec = spec or PolicySpec()
        self.selectors = selectors or [T.AMD_GPU_NODE_LABEL, T.LEGACY_GPU_NODE_LABEL]
        self.store = TelemetryStore()
        self.sem = asyncio.Semaphore(concurrency)
        self.max_retries = max_retries
        self.base_backoff_s = base_backoff_s
        self.max_backoff_s = max_backoff_s
        self.tasks: dict[str, asyncio.Task] = {}
        self.errors = 0
        self.polls = 0

    # -------------------------------------------------------------- policy changes
    def on_policy(self, spec: PolicySpec) -> None:
        self.spec = spec
        self.restart()

    def restart(self) -> None:
        for t in self.tasks.values():
            t.cancel()
        self.tasks.clear()
        for p in self.spec.sync_period:
            if p.period_s > 0:
                self.tasks[p.name] = asyncio.ensure_future(self._loop(p.name, p.period_s))

    async def stop(self) -> None:
        for t in self.tasks.values():
            t.cancel()
        for t in self.tasks.values():
            try:
                await t
            except (asyncio.CancelledError, Exception):
                pass
        self.tasks.clear()

    # -------------------------------------------------------------- polling
    async def _loop(self, metric: str, period: float) -> None:
        while True:
            t0 = time.monotonic()
            await self.sync_metric(metric)
            await asyncio.sleep(max(0.0, period - (time.monotonic() - t0)))

    async def sync_metric(self, metric: str) -> None:
        nodes = [n for n in self.list_nodes() if is_gpu_node(n, self.selectors)]
        await asyncio.gather(*(self._sync_node(n, metric) for n in nodes))

    async def _sync_node(self, node: dict, metric: str) -> None:
        name = pu.meta(node).get("name", "")
        entry = self.state.node_entry(name)
        n_dev = len(entry.topology.devices) if entry else pu.node_gpu_count(node)
        q = self.spec.query_for(metric)
        for card in range(n_dev):
            for attempt in range(self.max_retries + 1):
                try:
                    async with self.sem:
                        v = await self.prom.query_latest(name, metric, card, q)
                    self.polls += 1
                    if v is not None:
                        self.store.update(name, metric, card, v)
                    break
                except asyncio.CancelledError:
                    raise
                except Exception as e:
                    self.errors += 1
                    if attempt == self.max_retries:
                        log.warning("metric %s node %s card %d dropped: %s", metric, name, card, e)
                        break
                    await asyncio.sleep(min(self.base_backoff_s * 2 ** attempt, self.max_backoff_s))
        self.refresh_node(name, n_dev)

    def refresh_node(self, name: str, n_dev: int, now: float | None = None) -> None:
        periods = [(p.name, self.spec.active_duration(p.name)) for p in self.spec.sync_period]
        for card in range(n_dev):
            self.state.set_load(name, card, self.store.device_usage(name, card, periods, now))

    def sweep_stale(self) -> None:
        """Re-derives loads so samples that aged out stop counting (called periodically)."""
        for name in self.store.nodes():
            e = self.state.node_entry(name)
            if e:
                self.refresh_node(name, len(e.topology.devices))
