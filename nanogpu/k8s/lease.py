"""Leader election on a coordination.k8s.io/v1 Lease (client-go leaderelection semantics).

The reference runs one replica and has no HA (deploy/nano-gpu-scheduler.yaml:73).
Here several extender pods can run: all keep their informers and ledgers warm (a standby's
pod controller accounts the leader's binds from their annotations, so its ledger is the
API server's truth), but only the Lease holder reports ready and serves the verbs, so the
Service routes kube-scheduler to exactly one ledger. Acquire/renew use optimistic
concurrency on the Lease's resourceVersion; a holder that cannot renew within
`renew_deadline_s` steps down before another candidate may take over (lease expiry).
"""
from __future__ import annotations

import asyncio
import logging
import time
from datetime import datetime, timezone
from typing import Callable

from .client import ApiError

log = logging.getLogger(__name__)


def _now_rfc3339() -> str:
    return datetime.now(timezone.utc).strftime("%Y-%m-%dT%H:%M:%S.%fZ")


def _parse(ts: str | None) -> float:
    if not ts:
        return 0.0
    try:
        return datetime.strptime(ts, "%Y-%m-%dT%H:%M:%S.%fZ").replace(tzinfo=timezone.utc).timestamp()
    except ValueError:
        try:
            return datetime.strptime(ts, "%Y-%m-%dT%H:%M:%SZ").replace(tzinfo=timezone.utc).timestamp()
        except ValueError:
            return 0.0


class LeaderElector:
    def __init__(self, api, identity: str, namespace: str = "kube-system", name: str = "nano-gpu-scheduler",
                 lease_duration_s: float = 15.0, renew_deadline_s: float = 10.0, retry_period_s: float = 2.0,
                 on_change: Callable[[bool], None] | None = None):
        self.api = api
        self.identity = identity
        self.ns = namespace
        self.name = name
        self.lease_duration_s = lease_duration_s
        self.renew_deadline_s = renew_deadline_s
        self.retry_period_s = retry_period_s
        self.on_change = on_change
        self.leader = False
        self.observed_holder = ""
        self.transitions = 0
        self._last_renew = 0.0
        self._task: asyncio.Task | None = None

    def _set(self, leader: bool) -> None:
        if leader != self.leader:
            self.leader = leader
            log.info("%s %s leadership of %s/%s", self.identity, "acquired" if leader else "lost", self.ns, self.name)
            if self.on_change:
                self.on_change(leader)

    def _spec(self, transitions: int, acquire: str | None = None) -> dict:
        now = _now_rfc3339()
        return {"holderIdentity": self.identity, "leaseDurationSeconds": int(max(1, round(self.lease_duration_s))),
                "acquireTime": acquire or now, "renewTime": now, "leaseTransitions": transitions}

    async def try_acquire_or_renew(self) -> bool:
        try:
            cur = await self.api.get_lease(self.ns, self.name)
        except ApiError as e:
            if not e.not_found:
                raise
            body = {"apiVersion": "coordination.k8s.io/v1", "kind": "Lease",
                    "metadata": {"name": self.name, "namespace": self.ns}, "spec": self._spec(0)}
            try:
                await self.api.create_lease(self.ns, body)
            except ApiError as e2:
                if e2.status == 409:
                    return False
                raise
            self._last_renew = time.monotonic()
            return True
        spec = cur.get("spec") or {}
        holder = spec.get("holderIdentity") or ""
        self.observed_holder = holder
        dur = float(spec.get("leaseDurationSeconds") or self.lease_duration_s)
        expired = _parse(spec.get("renewTime")) + dur < time.time()
        if holder and holder != self.identity and not expired:
            return False
        transitions = int(spec.get("leaseTransitions") or 0) + (0 if holder == self.identity else 1)
        new = dict(cur)
        new["spec"] = self._spec(transitions, spec.get("acquireTime") if holder == self.identity else None)
        try:
            await self.api.update_lease(self.ns, self.name, new)
        except ApiError as e:
            if e.status == 409:
                return False
            raise
        if holder != self.identity:
            self.transitions += 1
        self._last_renew = time.monotonic()
        return True

    async def run(self) -> None:
        while True:
            try:
                ok = await self.try_acquire_or_renew()
            except asyncio.CancelledError:
                raise
            except Exception as e:
                log.warning("lease %s/%s: %s", self.ns, self.name, e)
                ok = False
            if ok:
                self._set(True)
            elif self.leader and time.monotonic() - self._last_renew > self.renew_deadline_s:
                self._set(False)     # could not renew in time: step down before the lease expires
            elif not self.leader:
                self._set(False)
            await asyncio.sleep(self.retry_period_s)

    def start(self) -> asyncio.Task:
        self._task = asyncio.ensure_future(self.run())
        return self._task

    async def release(self) -> None:
        """Gives the lease up on shutdown so a standby takes over without waiting for expiry."""
        if self._task:
            self._task.cancel()
        if not self.leader:
            return
        try:
            cur = await self.api.get_lease(self.ns, self.name)
            if (cur.get("spec") or {}).get("holderIdentity") == self.identity:
                new = dict(cur)
                new["spec"] = dict(cur["spec"], holderIdentity="", renewTime=_now_rfc3339(), leaseDurationSeconds=1)
                await self.api.update_lease(self.ns, self.name, new)
        except Exception as e:
            log.debug("lease release: %s", e)
        self._set(False)
