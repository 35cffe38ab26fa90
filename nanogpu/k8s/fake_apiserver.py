"""In-memory Kubernetes API server (pods, nodes, bindings, events, list+watch).

The reference has no fake apiserver and no integration tests. This store
backs three things: integration tests, the simulator, and the benchmark. It offers

  * `FakeKubeStore`   — the object store (resourceVersion, selectors, watch fan-out,
                         410 Gone on stale resourceVersion, 409 on binding conflicts);
  * `InProcKube`      — the `KubeClient` interface served directly from the store (with an
                         optional modelled RTT), for in-process runs;
  * `make_app(store)` — the same store over HTTP (aiohttp), wire-compatible with the paths
                         `KubeClient` uses, so the extender talks real REST in e2e tests;
  * fault injection   — per-verb error rates (409/500), latency, and watch drops.
"""
from __future__ import annotations

import asyncio
import copy
import json
import random
import time
import uuid
from collections import deque
from dataclasses import dataclass, field
from typing import Any, AsyncIterator

from aiohttp import web

from . import podutil as pu
from .client import ApiError


def _match_labels(obj: dict, selector: str | None) -> bool:
    if not selector:
        return True
    labels = pu.meta(obj).get("labels") or {}
    for term in selector.split(","):
        term = term.strip()
        if not term:
            continue
        if "!=" in term:
            k, v = term.split("!=", 1)
            if labels.get(k.strip()) == v.strip():
                return False
        elif "=" in term:
            k, v = term.split("=", 1)
            if labels.get(k.strip().rstrip("=")) != v.strip().lstrip("="):
                return False
        elif labels.get(term) is None:
            return False
    return True


def _match_fields(obj: dict, selector: str | None) -> bool:
    """kube-apiserver's pod field selectors: `k=v` / `k==v` and `k!=v` on spec.nodeName,
    metadata.name, metadata.namespace and status.phase (`spec.nodeName!=`: assigned pods)."""
    if not selector:
        return True
    for term in selector.split(","):
        term = term.strip()
        neg = "!=" in term
        k, _, v = term.partition("!=" if neg else "=")
        v = v.lstrip("=")
        have = {"spec.nodeName": lambda: pu.node_name_of(obj) or "",
                "metadata.name": lambda: pu.meta(obj).get("name") or "",
                "metadata.namespace": lambda: pu.meta(obj).get("namespace") or "",
                "status.phase": lambda: (obj.get("status") or {}).get("phase") or ""}.get(k.strip())
        if have is not None and (have() == v) == neg:
            return False
    return True


@dataclass
class Faults:
    latency_s: float = 0.0            # added to every API call (modelled RTT)
    watch_timeout_s: float = 0.0      # >0: watch streams end cleanly after this long (timeoutSeconds)
    patch_error_rate: float = 0.0     # 500 on pod PATCH
    bind_error_rate: float = 0.0      # 500 on binding POST
    conflict_rate: float = 0.0        # 409 on binding POST
    close_after_binding: bool = False  # answer a binding with Connection: close (requests
                                       # pipelined behind it on the connection go unanswered)
    # kube-apiserver's --max-mutating-requests-inflight (0: none): a POST / PUT / PATCH / DELETE
    # over it is answered 429 TooManyRequests with `Retry-After: retry_after_s`, not handled
    max_mutating_inflight: int = 0
    retry_after_s: int = 1
    seed: int = 0
    rng: random.Random = field(default_factory=random.Random)

    def __post_init__(self):
        self.rng.seed(self.seed)

    def roll(self, p: float) -> bool:
        return p > 0 and self.rng.random() < p


class FakeKubeStore:
    """Stored objects are immutable: every write replaces the object (copying only the
    path it changes), reads and watch events share references. Callers must not mutate
    what they get back (real clients get fresh JSON anyway)."""

    def __init__(self, history: int = 100000, faults: Faults | None = None):
        self.rv = 0
        self.pods: dict[tuple[str, str], dict] = {}
        self.nodes: dict[str, dict] = {}
        self.events: list[dict] = []
        self.bindings: list[tuple[str, str, str]] = []
        self.history: dict[str, deque] = {"pods": deque(maxlen=history), "nodes": deque(maxlen=history)}
        self.watchers: dict[str, list[_WatchBuffer]] = {"pods": [], "nodes": []}
        self.faults = faults or Faults()
        self.counts: dict[str, int] = {}
        self.leases: dict[tuple[str, str], dict] = {}
        self._ts_sec, self._ts_str = -1, ""
        # watch-cache floor per kind: a watch from an older resourceVersion gets 410 Gone
        self.compacted: dict[str, int] = {"pods": 0, "nodes": 0}

    # ------------------------------------------------------------------ internals
    def _bump(self, obj: dict) -> dict:
        """Returns a new top-level object with a new metadata dict (stored objects are
        immutable: writers copy the path they change, readers share references)."""
        self.rv += 1
        obj = dict(obj)
        obj["metadata"] = dict(obj.get("metadata") or {})
        obj["metadata"]["resourceVersion"] = str(self.rv)
        return obj

    def _stamp(self, obj: dict) -> dict:
        """`_bump` for an object whose top level and metadata the caller already copied."""
        self.rv += 1
        obj["metadata"]["resourceVersion"] = str(self.rv)
        return obj

    def _emit(self, kind: str, etype: str, obj: dict) -> None:
        ev = {"type": etype, "object": obj}
        self.history[kind].append((self.rv, ev))
        for w in self.watchers[kind]:
            w.push(ev)

    def _now_rfc3339(self) -> str:
        """Second-resolution RFC 3339 time (the API server's metav1.Time), formatted once per second."""
        t = int(time.time())
        if t != self._ts_sec:
            self._ts_sec, self._ts_str = t, time.strftime("%Y-%m-%dT%H:%M:%SZ", time.gmtime(t))
        return self._ts_str

    def _count(self, verb: str) -> None:
        self.counts[verb] = self.counts.get(verb, 0) + 1

    # ------------------------------------------------------------------ pods
    def create_pod(self, pod: dict) -> dict:
        self._count("create_pod")
        # copy-on-write like every other write here: only the paths the store changes are
        # copied (metadata, status); callers must not mutate a pod after handing it over
        pod = dict(pod)
        pod["metadata"] = m = dict(pod.get("metadata") or {})
        pod["status"] = dict(pod.get("status") or {})
        m.setdefault("namespace", "default")
        if not m.get("uid"):
            m["uid"] = str(uuid.uuid4())
        if "creationTimestamp" not in m:
            m["creationTimestamp"] = self._now_rfc3339()
        key = (m["namespace"], m["name"])
        if key in self.pods:
            raise ApiError(409, f'pods "{m["name"]}" already exists', "AlreadyExists")
        pod["status"].setdefault("phase", "Pending")
        pod = self._stamp(pod)
        self.pods[key] = pod
        self._emit("pods", "ADDED", pod)
        return pod

    def get_pod(self, ns: str, name: str) -> dict:
        self._count("get_pod")
        p = self.pods.get((ns, name))
        if p is None:
            raise ApiError(404, f'pods "{name}" not found', "NotFound")
        return p

    def patch_pod(self, ns: str, name: str, patch: dict) -> dict:
        self._count("patch_pod")
        if self.faults.patch_error_rate and self.faults.roll(self.faults.patch_error_rate):
            raise ApiError(500, "injected patch failure", "InternalError")
        p = self.pods.get((ns, name))
        if p is None:
            raise ApiError(404, f'pods "{name}" not found', "NotFound")
        np_ = pu.apply_patch(p, patch)
        if "spec" in patch and (np_.get("spec") or {}) != (p.get("spec") or {}):
            # kube-apiserver's pod update validation: the spec is immutable but for a few
            # fields, spec.nodeName included (a Binding sets it); restating it is a no-op
            raise ApiError(422, f'Pod "{name}" is invalid: spec: Forbidden: pod updates may not change fields '
                                f'other than `spec.containers[*].image`, `spec.initContainers[*].image`, '
                                f'`spec.activeDeadlineSeconds`, `spec.tolerations` (only additions to existing '
                                f'tolerations) or `spec.terminationGracePeriodSeconds`', "Invalid")
        np_ = self._stamp(np_) if np_.get("metadata") is not p.get("metadata") else self._bump(np_)
        self.pods[(ns, name)] = np_
        self._emit("pods", "MODIFIED", np_)
        return np_

    def update_pod(self, ns: str, name: str, pod: dict) -> dict:
        self._count("update_pod")
        cur = self.pods.get((ns, name))
        if cur is None:
            raise ApiError(404, f'pods "{name}" not found', "NotFound")
        want = pu.meta(pod).get("resourceVersion")
        if want and want != pu.meta(cur).get("resourceVersion"):
            raise ApiError(409, f'Operation cannot be fulfilled on pods "{name}": the object has been '
                                f'modified; please apply your changes to the latest version and try again',
                           "Conflict")
        pod = self._bump(copy.deepcopy(pod))
        self.pods[(ns, name)] = pod
        self._emit("pods", "MODIFIED", pod)
        return pod

    def bind_pod(self, ns: str, name: str, uid: str, node: str, annotations: dict | None = None) -> None:
        """pods/binding. As kube-apiserver does (setPodHostAndAnnotations), the Binding's own
        metadata.annotations are set on the pod together with spec.nodeName."""
        self._count("bind_pod")
        if self.faults.bind_error_rate and self.faults.roll(self.faults.bind_error_rate):
            raise ApiError(500, "injected binding failure", "InternalError")
        if self.faults.conflict_rate and self.faults.roll(self.faults.conflict_rate):
            raise ApiError(409, f'Operation cannot be fulfilled on pods/binding "{name}": injected', "Conflict")
        p = self.pods.get((ns, name))
        if p is None:
            raise ApiError(404, f'pods "{name}" not found', "NotFound")
        if uid and pu.pod_uid(p) != uid:
            raise ApiError(409, f"pod {name} uid mismatch", "Conflict")
        if pu.node_name_of(p):
            raise ApiError(409, f'pod {name} is already assigned to node "{pu.node_name_of(p)}"', "Conflict")
        if node not in self.nodes:
            raise ApiError(404, f'nodes "{node}" not found', "NotFound")
        np_ = dict(p)
        np_["spec"] = dict(p.get("spec") or {}, nodeName=node)
        np_["status"] = dict(p.get("status") or {}, phase="Running")
        np_["metadata"] = dict(p.get("metadata") or {})
        if annotations:
            np_["metadata"]["annotations"] = dict(np_["metadata"].get("annotations") or {}, **annotations)
        np_ = self._stamp(np_)
        self.pods[(ns, name)] = np_
        self.bindings.append((ns, name, node))
        self._emit("pods", "MODIFIED", np_)

    def delete_pod(self, ns: str, name: str) -> None:
        self._count("delete_pod")
        p = self.pods.pop((ns, name), None)
        if p is None:
            raise ApiError(404, f'pods "{name}" not found', "NotFound")
        self._emit("pods", "DELETED", self._bump(p))

    def set_phase(self, ns: str, name: str, phase: str) -> dict:
        return self.patch_pod(ns, name, {"status": {"phase": phase}})

    def list_pods(self, label_selector: str | None = None, field_selector: str | None = None,
                  namespace: str | None = None) -> tuple[list[dict], str]:
        self._count("list_pods")
        items = [p for (ns, _), p in self.pods.items()
                 if (namespace is None or ns == namespace) and _match_labels(p, label_selector)
                 and _match_fields(p, field_selector)]
        return items, str(self.rv)

    # ------------------------------------------------------------------ nodes
    def add_node(self, node: dict) -> dict:
        node = copy.deepcopy(node)
        name = pu.meta(node)["name"]
        etype = "MODIFIED" if name in self.nodes else "ADDED"
        node = self._bump(node)
        self.nodes[name] = node
        self._emit("nodes", etype, node)
        return node

    def get_node(self, name: str) -> dict:
        self._count("get_node")
        n = self.nodes.get(name)
        if n is None:
            raise ApiError(404, f'nodes "{name}" not found', "NotFound")
        return n

    def patch_node(self, name: str, patch: dict) -> dict:
        n = self.nodes.get(name)
        if n is None:
            raise ApiError(404, f'nodes "{name}" not found', "NotFound")
        nn = self._bump(pu.apply_patch(n, patch))
        self.nodes[name] = nn
        self._emit("nodes", "MODIFIED", nn)
        return nn

    def delete_node(self, name: str) -> None:
        n = self.nodes.pop(name, None)
        if n is not None:
            self._emit("nodes", "DELETED", self._bump(n))

    def list_nodes(self, label_selector: str | None = None) -> tuple[list[dict], str]:
        self._count("list_nodes")
        return [n for n in self.nodes.values() if _match_labels(n, label_selector)], str(self.rv)

    def add_event(self, ev: dict) -> None:
        self.events.append(ev)

    # ------------------------------------------------------------------ leases (coordination.k8s.io/v1)
    def get_lease(self, ns: str, name: str) -> dict:
        le = self.leases.get((ns, name))
        if le is None:
            raise ApiError(404, f'leases.coordination.k8s.io "{name}" not found', "NotFound")
        return le

    def create_lease(self, ns: str, lease: dict) -> dict:
        name = pu.meta(lease).get("name", "")
        if (ns, name) in self.leases:
            raise ApiError(409, f'leases.coordination.k8s.io "{name}" already exists', "AlreadyExists")
        le = self._bump(copy.deepcopy(lease))
        le["metadata"]["namespace"] = ns
        self.leases[(ns, name)] = le
        return le

    def update_lease(self, ns: str, name: str, lease: dict) -> dict:
        cur = self.get_lease(ns, name)
        if pu.meta(lease).get("resourceVersion") != pu.meta(cur).get("resourceVersion"):
            raise ApiError(409, f'Operation cannot be fulfilled on leases.coordination.k8s.io "{name}": '
                                "the object has been modified", "Conflict")
        le = self._bump(copy.deepcopy(lease))
        self.leases[(ns, name)] = le
        return le

    # ------------------------------------------------------------------ watch
    async def watch_batches(self, kind: str, resource_version: str, label_selector: str | None = None,
                            field_selector: str | None = None) -> AsyncIterator[list[dict]]:
        """Watch stream delivered as batches: everything emitted since the consumer last ran
        arrives as one list (one wake-up per burst instead of one queue hop per event)."""
        try:
            rv = int(resource_version or 0)
        except ValueError:
            rv = 0
        buf = _WatchBuffer()
        hist = self.history[kind]
        if rv and ((hist and hist[0][0] > rv + 1 and len(hist) == hist.maxlen) or rv < self.compacted[kind]):
            raise ApiError(410, f"too old resource version: {rv} ({self.compacted[kind] or hist[0][0]})", "Expired")
        timer = None
        if self.faults.watch_timeout_s > 0:
            timer = asyncio.get_running_loop().call_later(self.faults.watch_timeout_s, buf.push, None)
        for ev_rv, ev in list(hist):
            if ev_rv > rv:
                buf.evs.append(ev)
        self.watchers[kind].append(buf)
        try:
            while True:
                if not buf.evs:
                    buf.waiter = asyncio.get_running_loop().create_future()
                    try:
                        await buf.waiter
                    finally:
                        buf.waiter = None
                batch = list(buf.evs)
                buf.evs.clear()
                end = None in batch
                if end:
                    batch = batch[:batch.index(None)]
                if label_selector or field_selector:
                    batch = [ev for ev in batch if ev["type"] == "ERROR" or
                             (_match_labels(ev["object"], label_selector) and _match_fields(ev["object"], field_selector))]
                if batch:
                    yield batch
                if end:
                    return
        finally:
            if timer is not None:
                timer.cancel()
            self.watchers[kind].remove(buf)

    async def watch(self, kind: str, resource_version: str, label_selector: str | None = None,
                    field_selector: str | None = None) -> AsyncIterator[dict]:
        async for batch in self.watch_batches(kind, resource_version, label_selector, field_selector):
            for ev in batch:
                yield ev

    def drop_watches(self) -> None:
        """Fault injection: terminates every open watch stream."""
        for ws in self.watchers.values():
            for w in ws:
                w.push(None)

    def compact(self, kind: str | None = None) -> None:
        """Fault injection: the watch cache forgets its history (etcd compaction), so a watch
        resumed from any resourceVersion seen so far is answered 410 Gone."""
        for k in ([kind] if kind else list(self.history)):
            self.history[k].clear()
            self.compacted[k] = self.rv   # a watch from here on misses nothing

    def inject_watch_error(self, kind: str, code: int = 410, message: str = "too old resource version") -> None:
        """Fault injection: every open watch of `kind` receives an ERROR event (the API server
        sends one in-stream when a watcher's resourceVersion expires) and ends."""
        ev = {"type": "ERROR", "object": {"kind": "Status", "apiVersion": "v1", "status": "Failure",
                                          "message": message, "reason": "Expired" if code == 410 else "",
                                          "code": code}}
        for w in self.watchers[kind]:
            w.push(ev)
            w.push(None)


class _WatchBuffer:
    """One open watch: events appended by the store, drained by the watcher's task."""

    __slots__ = ("evs", "waiter")

    def __init__(self):
        self.evs: deque = deque()
        self.waiter: asyncio.Future | None = None

    def push(self, ev: dict | None) -> None:
        self.evs.append(ev)
        w = self.waiter
        if w is not None and not w.done():
            w.set_result(None)


class InProcKube:
    """`KubeClient`-compatible facade over a FakeKubeStore (no sockets)."""

    completes_inline = True   # calls need no running Task (see NativeServer._eager)

    def __init__(self, store: FakeKubeStore):
        self.store = store
        self.calls = 0

    async def _rtt(self) -> None:
        self.calls += 1
        if self.store.faults.latency_s > 0:
            await asyncio.sleep(self.store.faults.latency_s)

    async def get_pod(self, ns, name):
        self.calls += 1
        if self.store.faults.latency_s > 0:   # inline: no coroutine per call
            await asyncio.sleep(self.store.faults.latency_s)
        return self.store.get_pod(ns, name)

    async def patch_pod(self, ns, name, patch):
        self.calls += 1
        if self.store.faults.latency_s > 0:   # inline: no coroutine per call
            await asyncio.sleep(self.store.faults.latency_s)
        return self.store.patch_pod(ns, name, patch)

    async def bind_pod(self, ns, name, uid, node, annotations=None):
        self.calls += 1
        if self.store.faults.latency_s > 0:   # inline: no coroutine per call
            await asyncio.sleep(self.store.faults.latency_s)
        self.store.bind_pod(ns, name, uid, node, annotations)

    async def create_pod(self, pod):
        self.calls += 1
        if self.store.faults.latency_s > 0:   # inline: no coroutine per call
            await asyncio.sleep(self.store.faults.latency_s)
        return self.store.create_pod(pod)

    async def delete_pod(self, ns, name):
        self.calls += 1
        if self.store.faults.latency_s > 0:   # inline: no coroutine per call
            await asyncio.sleep(self.store.faults.latency_s)
        self.store.delete_pod(ns, name)

    async def list_pods(self, label_selector=None, field_selector=None, namespace=None):
        await self._rtt()
        return self.store.list_pods(label_selector, field_selector, namespace)

    async def get_node(self, name):
        await self._rtt()
        return self.store.get_node(name)

    async def list_nodes(self, label_selector=None):
        await self._rtt()
        return self.store.list_nodes(label_selector)

    async def patch_node(self, name, patch):
        await self._rtt()
        return self.store.patch_node(name, patch)

    async def patch_node_status(self, name, patch):
        return await self.patch_node(name, patch)

    async def create_event(self, ns, involved, reason, message, etype="Warning"):
        self.store.add_event({"namespace": ns, "involvedObject": involved, "reason": reason,
                              "message": message, "type": etype})

    def watch(self, resource, resource_version, timeout_s=300, label_selector=None, field_selector=None):
        return self.store.watch(resource, resource_version, label_selector, field_selector)   # no extra async-gen hop

    def watch_batches(self, resource, resource_version, timeout_s=300, label_selector=None, field_selector=None):
        return self.store.watch_batches(resource, resource_version, label_selector, field_selector)

    async def get_lease(self, ns, name):
        await self._rtt()
        return self.store.get_lease(ns, name)

    async def create_lease(self, ns, lease):
        await self._rtt()
        return self.store.create_lease(ns, lease)

    async def update_lease(self, ns, name, lease):
        await self._rtt()
        return self.store.update_lease(ns, name, lease)

    async def close(self):
        return None


# ---------------------------------------------------------------------- HTTP facade
def _err(e: ApiError) -> web.Response:
    body = {"kind": "Status", "apiVersion": "v1", "status": "Failure", "message": e.message,
            "reason": e.reason, "code": e.status}
    return web.json_response(body, status=e.status)


def make_app(store: FakeKubeStore) -> web.Application:
    routes = web.RouteTableDef()

    async def lat():
        if store.faults.latency_s > 0:
            await asyncio.sleep(store.faults.latency_s)

    async def stream_watch(request: web.Request, kind: str, label_selector=None, field_selector=None
                           ) -> web.StreamResponse:
        resp = web.StreamResponse(headers={"Content-Type": "application/json"})
        try:
            gen = store.watch(kind, request.query.get("resourceVersion", "0"), label_selector, field_selector)
            await resp.prepare(request)
            async for ev in gen:
                await resp.write(json.dumps(ev, separators=(",", ":")).encode() + b"\n")
        except ApiError as e:
            if not resp.prepared:
                return _err(e)
            # the stream is already open: the API server reports the failure in-stream
            status = {"kind": "Status", "apiVersion": "v1", "status": "Failure", "message": e.message,
                      "reason": e.reason, "code": e.status}
            try:
                await resp.write(json.dumps({"type": "ERROR", "object": status}, separators=(",", ":")).encode()
                                 + b"\n")
            except (ConnectionResetError, RuntimeError):
                pass
        except (ConnectionResetError, asyncio.CancelledError):
            pass
        return resp

    def listing(kind: str, items: list, rv: str, request: web.Request | None = None) -> web.Response:
        md = {"resourceVersion": rv}
        limit = int(request.query.get("limit", "0") or 0) if request is not None else 0
        if limit > 0:
            # `limit` / `continue` pages over the list in key order. A token is good for the
            # resourceVersion it was issued at; one the store has moved past is 410 Expired (a real
            # API server keeps the snapshot until etcd compacts it: the client's fallback is the
            # same either way)
            items = sorted(items, key=lambda p: (pu.meta(p).get("namespace", ""), pu.meta(p).get("name", "")))
            start = 0
            tok = request.query.get("continue", "")
            if tok:
                t_rv, _, off = tok.partition(":")
                if t_rv != rv:
                    return _err(ApiError(410, "The provided continue parameter is too old", "Expired"))
                start = int(off or 0)
            page = items[start:start + limit]
            if start + limit < len(items):
                md["continue"] = f"{rv}:{start + limit}"
            items = page
        return web.json_response({"kind": kind, "apiVersion": "v1", "metadata": md, "items": items})

    @routes.get("/api/v1/pods")
    async def list_all_pods(request):
        await lat()
        ls, fs = request.query.get("labelSelector"), request.query.get("fieldSelector")
        if request.query.get("watch") in ("1", "true"):
            return await stream_watch(request, "pods", ls, fs)
        items, rv = store.list_pods(ls, fs)
        return listing("PodList", items, rv, request)

    @routes.get("/api/v1/namespaces/{ns}/pods")
    async def list_ns_pods(request):
        await lat()
        items, rv = store.list_pods(request.query.get("labelSelector"), request.query.get("fieldSelector"),
                                    request.match_info["ns"])
        return listing("PodList", items, rv, request)

    @routes.post("/api/v1/namespaces/{ns}/pods")
    async def create_pod(request):
        await lat()
        body = await request.json()
        body.setdefault("metadata", {})["namespace"] = request.match_info["ns"]
        try:
            return web.json_response(store.create_pod(body), status=201)
        except ApiError as e:
            return _err(e)

    @routes.get("/api/v1/namespaces/{ns}/pods/{name}")
    async def get_pod(request):
        await lat()
        try:
            return web.json_response(store.get_pod(request.match_info["ns"], request.match_info["name"]))
        except ApiError as e:
            return _err(e)

    @routes.patch("/api/v1/namespaces/{ns}/pods/{name}")
    async def patch_pod(request):
        await lat()
        try:
            return web.json_response(store.patch_pod(request.match_info["ns"], request.match_info["name"],
                                                     await request.json()))
        except ApiError as e:
            return _err(e)

    @routes.put("/api/v1/namespaces/{ns}/pods/{name}")
    async def put_pod(request):
        await lat()
        try:
            return web.json_response(store.update_pod(request.match_info["ns"], request.match_info["name"],
                                                      await request.json()))
        except ApiError as e:
            return _err(e)

    @routes.delete("/api/v1/namespaces/{ns}/pods/{name}")
    async def delete_pod(request):
        await lat()
        try:
            store.delete_pod(request.match_info["ns"], request.match_info["name"])
            return web.json_response({"kind": "Status", "status": "Success"})
        except ApiError as e:
            return _err(e)

    @routes.post("/api/v1/namespaces/{ns}/pods/{name}/binding")
    async def bind(request):
        await lat()
        body = await request.json()
        try:
            store.bind_pod(request.match_info["ns"], request.match_info["name"],
                           (body.get("metadata") or {}).get("uid", ""), (body.get("target") or {}).get("name", ""),
                           (body.get("metadata") or {}).get("annotations"))
            resp = web.json_response({"kind": "Status", "status": "Success"}, status=201)
            if store.faults.close_after_binding:
                resp.force_close()
            return resp
        except ApiError as e:
            return _err(e)

    @routes.get("/api/v1/nodes")
    async def list_nodes(request):
        await lat()
        ls = request.query.get("labelSelector")
        if request.query.get("watch") in ("1", "true"):
            return await stream_watch(request, "nodes", ls)
        items, rv = store.list_nodes(ls)
        return listing("NodeList", items, rv)

    @routes.post("/api/v1/nodes")
    async def create_node(request):
        await lat()
        return web.json_response(store.add_node(await request.json()), status=201)

    @routes.get("/api/v1/nodes/{name}")
    async def get_node(request):
        await lat()
        try:
            return web.json_response(store.get_node(request.match_info["name"]))
        except ApiError as e:
            return _err(e)

    @routes.patch("/api/v1/nodes/{name}")
    @routes.patch("/api/v1/nodes/{name}/status")
    async def patch_node(request):
        await lat()
        try:
            return web.json_response(store.patch_node(request.match_info["name"], await request.json()))
        except ApiError as e:
            return _err(e)

    @routes.get("/apis/coordination.k8s.io/v1/namespaces/{ns}/leases/{name}")
    async def get_lease(request):
        await lat()
        try:
            return web.json_response(store.get_lease(request.match_info["ns"], request.match_info["name"]))
        except ApiError as e:
            return _err(e)

    @routes.post("/apis/coordination.k8s.io/v1/namespaces/{ns}/leases")
    async def create_lease(request):
        await lat()
        try:
            return web.json_response(store.create_lease(request.match_info["ns"], await request.json()), status=201)
        except ApiError as e:
            return _err(e)

    @routes.put("/apis/coordination.k8s.io/v1/namespaces/{ns}/leases/{name}")
    async def update_lease(request):
        await lat()
        try:
            return web.json_response(store.update_lease(request.match_info["ns"], request.match_info["name"],
                                                        await request.json()))
        except ApiError as e:
            return _err(e)

    @routes.post("/api/v1/namespaces/{ns}/events")
    async def event(request):
        store.add_event(await request.json())
        return web.json_response({}, status=201)

    mutating = {"inflight": 0, "peak": 0}

    @web.middleware
    async def admission(request, handler):
        # kube-apiserver's max-in-flight filter: over the limit, refused before any handling
        limit = store.faults.max_mutating_inflight
        if limit <= 0 or request.method not in ("POST", "PUT", "PATCH", "DELETE"):
            return await handler(request)
        if mutating["inflight"] >= limit:
            store._count("throttled")
            return web.json_response({"kind": "Status", "apiVersion": "v1", "status": "Failure",
                                      "message": "Too many requests, please try again later.",
                                      "reason": "TooManyRequests", "code": 429},
                                     status=429, headers={"Retry-After": str(store.faults.retry_after_s)})
        mutating["inflight"] += 1
        mutating["peak"] = max(mutating["peak"], mutating["inflight"])
        store.counts["peak_mutating_inflight"] = mutating["peak"]
        try:
            return await handler(request)
        finally:
            mutating["inflight"] -= 1

    app = web.Application(client_max_size=16 * 1024 * 1024, middlewares=[admission])
    app.add_routes(routes)
    app[STORE_KEY] = store

    async def _close_watches(_app):
        store.drop_watches()

    app.on_shutdown.append(_close_watches)
    return app


STORE_KEY = web.AppKey("store", FakeKubeStore)


async def serve(store: FakeKubeStore, host: str = "127.0.0.1", port: int = 0) -> tuple[web.AppRunner, int]:
    runner = web.AppRunner(make_app(store), access_log=None, shutdown_timeout=1.0)
    await runner.setup()
    site = web.TCPSite(runner, host, port, backlog=1024)
    await site.start()
    port = site._server.sockets[0].getsockname()[1]  # type: ignore[union-attr]
    return runner, port


def store_summary(store: FakeKubeStore) -> dict[str, Any]:
    bound = sum(1 for p in store.pods.values() if pu.node_name_of(p))
    return {"pods": len(store.pods), "bound": bound, "nodes": len(store.nodes), "rv": store.rv,
            "bindings": len(store.bindings), "calls": dict(store.counts)}
