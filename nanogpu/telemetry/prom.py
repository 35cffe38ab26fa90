"""Prometheus instant-query client.

Reference: pkg/prometheus/prometheus.go:17-83 — query `<metric>{node=~"<n>",card="<i>"} /100`,
fall back to `{node="<n>",cardNode="<i>"}`, 10 s timeout, negative/NaN -> 0, the LAST
vector element wins, formatted "%.5f"; query errors are swallowed as ("", nil) (D12).
Here errors are raised (the poller counts and backs off) and templates are configurable
so AMD exporter metric names can be used.
"""
from __future__ import annotations

import math

import aiohttp

from ..config.policy import MetricQuery


class PromError(Exception):
    pass


class PromClient:
    def __init__(self, url: str, timeout_s: float = 10.0):
        self.url = url.rstrip("/")
        self.timeout = aiohttp.ClientTimeout(total=timeout_s)
        self._s: aiohttp.ClientSession | None = None
        self.queries = 0

    async def _session(self) -> aiohttp.ClientSession:
        if self._s is None or self._s.closed:
            self._s = aiohttp.ClientSession(timeout=self.timeout)
        return self._s

    async def close(self) -> None:
        if self._s is not None:
            await self._s.close()

    async def query(self, promql: str) -> list[tuple[dict, float]]:
        s = await self._session()
        self.queries += 1
        async with s.get(f"{self.url}/api/v1/query", params={"query": promql}) as r:
            if r.status >= 400:
                raise PromError(f"prometheus {r.status}: {await r.text()}")
            body = await r.json(content_type=None)
        if body.get("status") != "success":
            raise PromError(f"prometheus query failed: {body.get('error')}")
        data = body.get("data") or {}
        if data.get("resultType") != "vector":
            raise PromError(f"unexpected result type {data.get('resultType')}")
        out = []
        for el in data.get("result") or []:
            try:
                v = float(el["value"][1])
            except (KeyError, IndexError, ValueError, TypeError):
                continue
            if v < 0 or math.isnan(v):
                v = 0.0
            out.append((el.get("metric") or {}, v))
        return out

    @staticmethod
    def _by_card(res, q: MetricQuery, out: dict[int, float], rank: dict[int, int]) -> None:
        """A series names its card in the first of q.card_labels it carries; earlier labels win
        (the reference's primary `card` over its fallback `cardNode`, prometheus.go:70-76)."""
        for labels, v in res:
            for r, lab in enumerate(q.card_labels):
                raw = labels.get(lab)
                if raw is None:
                    continue
                try:
                    card = int(raw)
                except ValueError:
                    break
                if card not in rank or r <= rank[card]:   # later samples of equal rank win
                    out[card], rank[card] = round(v, 5), r
                break

    async def query_node(self, node: str, metric: str, q: MetricQuery) -> dict[int, float]:
        """Every card of `node` in one query (q.batch): {card: last sample}."""
        res = await self.query(q.batch.format(metric=metric, node=node))
        out: dict[int, float] = {}
        self._by_card(res, q, out, {})
        return out

    async def query_cluster(self, metric: str, q: MetricQuery) -> dict[str, dict[int, float]]:
        """Every node and card in one query (q.cluster): {node: {card: last sample}}. A series
        names its node in the first of q.node_labels it carries; series without one are skipped."""
        res = await self.query(q.cluster.format(metric=metric))
        groups: dict[str, list] = {}
        for labels, v in res:
            node = next((labels[k] for k in q.node_labels if labels.get(k)), None)
            if node is not None:
                groups.setdefault(node, []).append((labels, v))
        out: dict[str, dict[int, float]] = {}
        for node, rows in groups.items():
            self._by_card(rows, q, out.setdefault(node, {}), {})
        return out

    async def query_latest(self, node: str, metric: str, card: int, q: MetricQuery) -> float | None:
        """Last sample of the primary template, else of the fallback (prometheus.go:68-83)."""
        res = await self.query(q.query.format(metric=metric, node=node, card=card))
        if not res and q.fallback:
            res = await self.query(q.fallback.format(metric=metric, node=node, card=card))
        if not res:
            return None
        return round(res[-1][1], 5)
