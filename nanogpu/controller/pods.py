"""Pod lifecycle controller: keeps the ledger equal to what the API server says.

Reference: pkg/controller/controller.go (NewController :77-162, syncPod :210-243,
add/update/delete handlers :270-357). Semantics kept: a pod bound by someone else (or found
after a restart) with the assume annotation is allocated from its annotations; a
completed pod is released. Fixed:
  * a terminating pod (deletionTimestamp, still in its grace period) keeps its percent, HBM
    and CUs until it stops (Succeeded/Failed) or is DELETED; the reference releases at the
    deletionTimestamp (pod.go:15-24), which hands a running pod's HBM to the next one
    (compat mode keeps the reference behaviour);
  * D3 — the reference's delete handler only `Forget`s (dealer.go:311-319), leaking the
    GPU share whenever the pod disappears before the worker runs; here DELETED releases;
  * D4 — no one-second sleep between work items;
  * P5 — handlers never block on a global lock (the ledger lookup is a native shard read).
"""
from __future__ import annotations

import asyncio
import logging

from .. import types as T
from ..k8s import podutil as pu
from ..k8s.informer import Informer, WorkQueue
from ..state.cluster import ClusterState

log = logging.getLogger(__name__)


class PodController:
    def __init__(self, state: ClusterState, informer: Informer, workers: int = 1, metrics=None,
                 relabel=None):
        self.state = state
        self.informer = informer
        self.queue = WorkQueue("podQueue")
        self.workers = max(1, workers)
        self.metrics = metrics
        # async (namespace, name, node): PATCHes the assume label onto a bound pod. The bind
        # answers kube-scheduler once the binding (which carries the placement annotations)
        # landed and the label follows; a process killed in between leaves a placed pod
        # without it, which the next relist (every start begins with one) puts back
        self.relabel = relabel
        self._tasks: list[asyncio.Task] = []
        self.reconciled = 0        # shares released because a relist no longer held their pod
        self.relabeled = 0         # assume labels re-applied after a relist
        informer.add_handler(self._on_event)
        informer.add_relist_hook(self._on_relist)
        if getattr(informer, "watch_filter", None) is not None:
            state.add_listener(self._mirror_policy)
            self._mirror_policy()

    def _mirror_policy(self) -> None:
        # the native watch filter drops what this controller would ignore: it must agree on
        # when a terminating pod's share ends
        self.informer.watch_filter.release_on_terminating = bool(self.state.options.compat)

    # ---------------------------------------------------------------- handlers
    def _release(self, uid: str) -> None:
        if self.state.release_uid(uid) and self.metrics:
            self.metrics.pods_released.inc()

    async def _on_relist(self, pods: list[dict], before: float) -> None:
        """client-go's reflector turns every key missing from a relist into a delete, and the
        reference's informer handlers rely on it (controller.go:89-136, 337-357). The store's
        own diff (informer.py::_list) covers the pods Python held; pods the native watch filter
        kept away from Python (bound by this extender, held only by the ledger) are reconciled
        here: a committed share whose pod the LIST no longer returns is released. The ledger
        walk runs on an executor thread without the GIL (the UIDs cross as one string), so the
        event loop keeps serving while a 100k-pod relist is reconciled."""
        joined = "\n".join(u for u in ((p.get("metadata") or {}).get("uid", "") for p in pods) if u)
        loop = asyncio.get_running_loop()
        gone = await loop.run_in_executor(None, self.state.reconcile_native, joined, before)
        self.state.note_released(gone)
        if gone:
            self.reconciled += len(gone)
            if self.metrics:
                self.metrics.pods_released.inc(len(gone))
            log.info("relist: released %d pods deleted while the watch was down", len(gone))
        if self.relabel is not None:
            missing = [(m.get("namespace", "default"), m.get("name", ""), pu.node_name_of(p))
                       for p in pods for m in (pu.meta(p),)
                       if pu.node_name_of(p) and pu.is_assumed(p)
                       and (m.get("labels") or {}).get(T.LABEL_GPU_ASSUME) != "true"
                       and not pu.share_gone(p, self.state.options.compat)]
            if missing:
                self._tasks.append(asyncio.ensure_future(self._relabel_all(missing)))

    async def _relabel_all(self, missing: list[tuple[str, str, str]]) -> None:
        sem = asyncio.Semaphore(8)

        async def one(ns: str, name: str, node: str) -> None:
            async with sem:
                try:
                    await self.relabel(ns, name, node)
                    self.relabeled += 1
                except Exception as e:   # gone, moved, or the API down: the next relist retries
                    log.warning("relist: assume label of %s/%s not re-applied: %s", ns, name, e)

        await asyncio.gather(*(one(*m) for m in missing))
        log.info("relist: re-applied the assume label to %d of %d placed pods without it",
                 self.relabeled, len(missing))

    def _on_event(self, etype: str, pod: dict, old: dict | None) -> None:
        # hot: every pod event of the cluster passes here (four per scheduled pod), so the
        # cheap tests come first and the container limits are parsed only when they decide
        m = pod.get("metadata") or {}
        uid = m.get("uid", "")
        if old is not None:
            ouid = (old.get("metadata") or {}).get("uid", "")
            if ouid and ouid != uid:
                self._release(ouid)            # same name, new object: the previous one is gone
        if etype == "DELETED":
            # D3: release right away, the object is gone from the store (a pod that never
            # held a share is simply not in the ledger)
            self._release(uid)
            self.state.forget(uid)
            self.state.forget_reaccount(uid)
            return
        node = (pod.get("spec") or {}).get("nodeName")
        # a terminating pod (deletionTimestamp only) still runs and keeps its share until it
        # stops or is DELETED; compat releases at the deletionTimestamp, like the reference
        completed = (pod.get("status") or {}).get("phase") in ("Succeeded", "Failed") or \
            (self.state.options.compat and bool(m.get("deletionTimestamp")))
        if not node and not completed:
            return                             # pending: the extender's own business until bound
        if self.state.known(uid) or uid in self.state._reaccount_wait:
            if completed:                                                        # controller.go:303-306
                self.queue.add(f"{m.get('namespace', 'default')}/{m.get('name', '')}")
            elif T.ANNOTATION_RECONCILED in (m.get("annotations") or {}):
                # the node agent found the pod running on other devices than placed (kubelet
                # admitted same-size containers out of bind order) and rewrote its annotations
                self.queue.add(f"{m.get('namespace', 'default')}/{m.get('name', '')}")
            return
        if completed or self.state.released(uid):
            return
        # bound by someone else / found at restart (controller.go:307-310); reference
        # FilterFunc (controller.go:90-106) keeps only GPU-sharing pods
        if (m.get("annotations") or {}).get(T.ANNOTATION_GPU_ASSUME) == "true" and pu.is_gpu_sharing(pod):
            self.queue.add(f"{m.get('namespace', 'default')}/{m.get('name', '')}")

    # ---------------------------------------------------------------- worker
    async def _sync(self, key: str) -> None:
        pod = self.informer.get(key)
        if pod is None:
            return
        if pu.share_gone(pod, self.state.options.compat):
            self.state.forget_reaccount(pu.pod_uid(pod))
            if self.state.release(pod) and self.metrics:
                self.metrics.pods_released.inc()
            return
        if not pu.node_name_of(pod) or not pu.is_assumed(pod):
            return
        uid = pu.pod_uid(pod)
        if T.ANNOTATION_RECONCILED in (pu.meta(pod).get("annotations") or {}) and \
                (self.state.known(uid) or uid in self.state._reaccount_wait):
            if self.state.reaccount(pod) and self.metrics:
                self.metrics.pods_reaccounted.inc()
            return
        if not self.state.known(pu.pod_uid(pod)) and not self.state.released(pu.pod_uid(pod)):
            if not self.state.allocate_existing(pod):
                raise RuntimeError(f"allocate {key} failed")

    def start(self) -> None:
        for _ in range(self.workers):
            self._tasks.append(asyncio.ensure_future(self.queue.worker(self._sync)))

    async def stop(self) -> None:
        for t in self._tasks:
            t.cancel()
        for t in self._tasks:
            try:
                await t
            except (asyncio.CancelledError, Exception):
                pass
        self._tasks.clear()


class NodeController:
    """Node informer -> ledger: capacity / topology changes re-register the node (D20)."""

    def __init__(self, state: ClusterState, informer: Informer):
        self.state = state
        self.informer = informer
        informer.add_handler(self._on_event)

    def _on_event(self, etype: str, node: dict, old: dict | None) -> None:
        name = pu.meta(node).get("name", "")
        if etype == "DELETED":
            self.state.forget_node(name)
            return
        if pu.node_gpu_count(node) > 0 or name in self.state._nodes:
            self.state.try_register_node(node)
