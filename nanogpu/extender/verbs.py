"""Extender verbs: filter / prioritize / bind.

Reference: pkg/scheduler/predicate.go:19-53, priority.go:19-42, bind.go:26-82 and the
dealer calls behind them (dealer.go:89-203). The reference holds ONE mutex across
filter, score and the API writes of bind; here filter/prioritize are lock-free reads of
per-node snapshots and bind is

    reserve (native ledger, µs)  ->  POST binding (+ annotations)  ->  commit  ->  PATCH label
                                  \\-> binding refused: rollback

so binds for different pods overlap their API round trips (the reference's
bind rate is bounded by 1 / (2 x RTT)).
"""
from __future__ import annotations

import asyncio
import logging
import time
from collections import OrderedDict

from .. import types as T
from ..k8s import podutil as pu
from ..k8s.client import ApiError
from ..obs import Metrics, Span, Tracer
from ..state.cluster import N, ClusterState, SchedulingError
from .wire import (BindingArgs, ExtenderArgs, PreemptionArgs, binding_result, filter_result,
                   preemption_result, priority_list)

log = logging.getLogger(__name__)


class PodCache:
    """Pods seen in filter/prioritize by UID, so bind can skip the reference's live GET
    (bind.go:61-82) when the object is fresh. Bounded LRU."""

    def __init__(self, cap: int = 16384):
        self.cap = cap
        self.d: OrderedDict[str, dict] = OrderedDict()

    def put(self, pod: dict) -> None:
        uid = pu.pod_uid(pod)
        if not uid:
            return
        self.d[uid] = pod
        self.d.move_to_end(uid)
        if len(self.d) > self.cap:
            self.d.popitem(last=False)

    def pop(self, uid: str) -> dict | None:
        return self.d.pop(uid, None)


class Extender:
    def __init__(self, state: ClusterState, api, metrics: Metrics | None = None,
                 tracer: Tracer | None = None, verify_pod_on_bind: bool = False,
                 api_retries: int = 2, record_events: bool = True, assume_label: bool = True):
        self.state = state
        self.assume_label = assume_label   # PATCH the reference's assume label beside the binding
        self.api = api
        self.metrics = metrics or Metrics()
        self.tracer = tracer or Tracer()
        self.verify_pod_on_bind = verify_pod_on_bind
        self.api_retries = api_retries
        self.record_events = record_events
        self.pods = PodCache()
        self._bg: set[asyncio.Task] = set()
        m = self.metrics
        # labelled children the bind path touches on every pod
        self._m_bind_latency = m.child(m.verb_latency, "bind")
        self._m_bind_ok = m.child(m.verb_total, "bind", "ok")
        self._m_bind_err = m.child(m.verb_total, "bind", "error")
        self._m_patch = m.child(m.bind_phase, "patch")
        self._m_binding = m.child(m.bind_phase, "binding")

    # ------------------------------------------------------------------ filter
    def filter(self, body) -> dict:
        t0 = time.perf_counter()
        try:
            args = ExtenderArgs.decode(body)
        except ValueError as e:
            self.metrics.child(self.metrics.verb_total, "filter", "bad_request").inc()
            return filter_result(None, {}, str(e))
        with self.tracer.span("filter", pu.pod_key(args.pod)) as sp:
            names = args.node_names
            node_objs = None
            if names is None:
                if args.nodes is None:
                    self.metrics.child(self.metrics.verb_total, "filter", "error").inc()
                    return filter_result(None, {}, T.FILTER_NODE_CACHE_ERROR)
                # nodeCacheCapable=false: full Node objects in the request (the reference rejects this)
                for n in args.nodes:
                    self.state.try_register_node(n)
                node_objs = {pu.meta(n).get("name"): n for n in args.nodes}
                names = list(node_objs)
            self.pods.put(args.pod)
            try:
                ok, failed = self.state.filter(args.pod, names)
            except Exception as e:   # a protocol answer, never a 500 (every node fails with the reason)
                log.exception("filter %s", pu.pod_key(args.pod))
                ok, failed = [], {n: f"nano-gpu: {type(e).__name__}: {e}" for n in names}
            sp.note = f"{len(ok)}/{len(names)} fit"
        self.metrics.child(self.metrics.verb_latency, "filter").observe(time.perf_counter() - t0)
        self.metrics.child(self.metrics.verb_total, "filter", "ok").inc()
        if node_objs is not None:
            return filter_result(None, failed, nodes=[node_objs[n] for n in ok])
        return filter_result(ok, failed)

    # ------------------------------------------------------------------ prioritize
    def prioritize(self, body) -> list[dict]:
        """Raises ValueError on a malformed body (server maps it to 400; reference panics,
        routes.go:102-104)."""
        t0 = time.perf_counter()
        args = ExtenderArgs.decode(body)
        names = args.node_names
        if names is None:
            names = [pu.meta(n).get("name") for n in (args.nodes or [])]
            for n in args.nodes or []:
                self.state.try_register_node(n)
        with self.tracer.span("prioritize", pu.pod_key(args.pod)):
            self.pods.put(args.pod)
            try:
                scores = self.state.score(args.pod, names)
            except Exception:
                log.exception("prioritize %s", pu.pod_key(args.pod))
                scores = [0] * len(names)            # ScoreMin everywhere (dealer.go:147)
        self.metrics.child(self.metrics.verb_latency, "prioritize").observe(time.perf_counter() - t0)
        self.metrics.child(self.metrics.verb_total, "prioritize", "ok").inc()
        return priority_list(names, scores)

    # ------------------------------------------------------------------ preemption
    def preempt(self, body) -> dict:
        """kube-scheduler's preemptVerb. Its victims free `nano-gpu/gpu-percent` as a
        node-wide scalar; whether the pod then fits depends on which devices, partitions and
        HBM pools those shares held. A candidate node stays only if the preemptor fits once
        its victims' shares are released. This is simulated on a copy of the node in the
        ledger (Ledger::fits_without). Victims are passed through unchanged: kube-scheduler
        chose them for every resource, not only GPU. Raises ValueError on a malformed body."""
        t0 = time.perf_counter()
        args = PreemptionArgs.decode(body)
        keep: dict[str, list[str]] = {}
        try:
            demand, _ = pu.ledger_view(self.state.pod_demand(args.pod))
        except pu.TooManyGpuContainers:
            return preemption_result(keep, args.pdb)
        with self.tracer.span("preempt", pu.pod_key(args.pod)) as sp:
            for node, uids in args.victims.items():
                e = self.state.node_entry(node)
                if e is None:
                    continue
                rc, _ = self.state.ledger.fits_without(e.id, uids, demand, self.state.options)
                if rc == N.OK:
                    keep[node] = uids
            sp.note = f"{len(keep)}/{len(args.victims)} nodes"
        self.metrics.child(self.metrics.verb_latency, "preempt").observe(time.perf_counter() - t0)
        self.metrics.child(self.metrics.verb_total, "preempt", "ok").inc()
        return preemption_result(keep, args.pdb)

    # ------------------------------------------------------------------ bind
    async def bind(self, body) -> dict:
        t0 = time.perf_counter()
        try:
            args = BindingArgs.decode(body)
        except ValueError as e:
            self.metrics.child(self.metrics.verb_total, "bind", "bad_request").inc()
            return binding_result(str(e))
        err = ""
        with self.tracer.span("bind", f"{args.pod_namespace}/{args.pod_name}") as sp:
            try:
                await self._bind(args, sp)
            except (SchedulingError, ApiError, asyncio.TimeoutError, OSError) as e:
                err = str(e) or e.__class__.__name__
                sp.ok = False
                sp.note = err
            except Exception as e:   # reported in ExtenderBindingResult.Error, not as a crash
                log.exception("bind %s/%s", args.pod_namespace, args.pod_name)
                err = f"nano-gpu: {type(e).__name__}: {e}"
                sp.ok = False
                sp.note = err
        dt = time.perf_counter() - t0
        self.metrics.child(self.metrics.verb_latency, "bind").observe(dt)
        self.metrics.child(self.metrics.verb_total, "bind", "error" if err else "ok").inc()
        if err:
            log.info("bind %s/%s -> %s failed: %s", args.pod_namespace, args.pod_name, args.node, err)
        return binding_result(err)

    async def _get_pod(self, args: BindingArgs) -> dict:
        """bind.go:61-82: live GET, re-GET once on UID mismatch."""
        pod = await self.api.get_pod(args.pod_namespace, args.pod_name)
        if args.pod_uid and pu.pod_uid(pod) != args.pod_uid:
            pod = await self.api.get_pod(args.pod_namespace, args.pod_name)
            if pu.pod_uid(pod) != args.pod_uid:
                raise SchedulingError(f"pod {args.pod_name} in ns {args.pod_namespace}'s uid is "
                                      f"{pu.pod_uid(pod)}, and it's not equal with expected {args.pod_uid}")
        return pod

    @staticmethod
    def _backoff(e: ApiError, attempt: int) -> float:
        """5 ms x 2^k, or a 429's Retry-After when it asks for longer (kube-apiserver: 1 s), at
        most 2 s a wait: the bind holds kube-scheduler's request, which times out at 30 s (the
        native writer waits the same way, BindIo::kMaxRetryAfterS)."""
        b = 0.005 * (2 ** attempt)
        ra = getattr(e, "retry_after", None)
        return min(2.0, max(b, ra)) if e.status == 429 and ra else b

    async def _retry(self, op: str, fn, *a):
        for attempt in range(self.api_retries + 1):
            try:
                return await fn(*a)
            except ApiError as e:
                self.metrics.child(self.metrics.api_errors, op, str(e.status)).inc()
                if e.status < 500 and e.status != 429 or attempt == self.api_retries:
                    raise
                wait = self._backoff(e, attempt)
            await asyncio.sleep(wait)

    async def _retry_after(self, first: ApiError, op: str, fn, *a):
        """`_retry` for a call whose first attempt already failed with `first`."""
        self.metrics.child(self.metrics.api_errors, op, str(first.status)).inc()
        if first.status < 500 and first.status != 429 or self.api_retries == 0:
            raise first
        await asyncio.sleep(self._backoff(first, 0))
        for attempt in range(1, self.api_retries + 1):
            try:
                return await fn(*a)
            except ApiError as e:
                self.metrics.child(self.metrics.api_errors, op, str(e.status)).inc()
                if e.status < 500 and e.status != 429 or attempt == self.api_retries:
                    raise
                wait = self._backoff(e, attempt)
            await asyncio.sleep(wait)

    async def _bind(self, args: BindingArgs, sp) -> None:
        pod = None if self.verify_pod_on_bind else self.pods.pop(args.pod_uid)
        tp = time.perf_counter()
        if pod is None or (args.pod_uid and pu.pod_uid(pod) != args.pod_uid):
            pod = await self._get_pod(args)
            sp.phases["get"] = time.perf_counter() - tp
        if pu.is_completed(pod):
            raise SchedulingError(f"pod {args.pod_name}/{args.pod_namespace} already deleted or completed")
        uid = pu.pod_uid(pod)
        t1 = time.perf_counter()
        plan, fresh = self.state.reserve(pod, args.node)
        sp.phases["reserve"] = time.perf_counter() - t1
        names = [c.get("name", "") for c in pu.containers(pod)]
        ns, name = pu.pod_ns_name(pod)
        await self._write(args.pod_namespace, args.pod_name, uid, args.node, names, plan, fresh, sp, (ns, name))

    async def bind_prepared(self, p: dict) -> dict:
        """Bind whose ledger reservation already ran in the native front door
        (native/src/frontend.cpp::prepare_bind); only the API writes and commit remain.
        Runs once per pod at the burst rate, so it records its span and metrics directly."""
        t0 = time.perf_counter()
        ns, name = p["ns"], p["name"]
        sp = Span("bind", f"{ns}/{name}", time.time())
        err = ""
        try:
            rc = p["rc"]
            if rc not in (N.OK, N.OK_EXISTING):
                raise self.state.reserve_error(p["demand"], p["node"], rc)
            sp.phases["reserve"] = 0.0
            await self._write(ns, name, p["uid"], p["node"], p["containers"], p["plan"], rc == N.OK, sp, (ns, name))
        except (SchedulingError, ApiError, asyncio.TimeoutError, OSError) as e:
            err = str(e) or e.__class__.__name__
            sp.ok = False
            sp.note = err
        except Exception as e:
            sp.ok = False
            sp.note = repr(e)
            raise
        finally:
            sp.dur = time.perf_counter() - t0
            self.tracer.buf.append(sp)
        self._m_bind_latency.observe(sp.dur)
        if err:
            self._m_bind_err.inc()
            log.info("bind %s/%s -> %s failed: %s", ns, name, p["node"], err)
        else:
            self._m_bind_ok.inc()
        return binding_result(err)

    async def _write(self, ns: str, name: str, uid: str, node: str, names: list[str], plan, fresh: bool, sp,
                     pod_ns_name: tuple[str, str]) -> None:
        """Second half of bind: the binding, commit, then the assume label (fixes reference
        D1/D2: a failed binding rolls the reservation back and reports the error).

        The Binding itself carries the placement annotations, which kube-apiserver sets on
        the pod together with spec.nodeName (setPodHostAndAnnotations): a bound pod never
        lacks them, and a refused binding writes nothing. The label follows as a PATCH that
        restates spec.nodeName (pu.label_patch), so it lands only on a pod bound to `node`.
        Nothing is ever un-annotated: no write of this bind can have landed on a pod that is
        not bound here (a pod bound elsewhere keeps its placement untouched)."""
        t2 = time.perf_counter()
        ann = pu.placement_annotations(names, plan, {T.ANNOTATION_ASSUME_TIME: f"{time.time():.6f}"})
        try:
            try:
                try:
                    await self.api.bind_pod(ns, name, uid, node, ann)
                except ApiError as e0:
                    await self._retry_after(e0, "bind", self.api.bind_pod, ns, name, uid, node, ann)
            except (ApiError, OSError, asyncio.TimeoutError) as e:
                # a retried POST whose first attempt landed (409), or an answer lost to a 5xx or
                # the transport: the pod already on this node means the bind succeeded
                if isinstance(e, ApiError) and not (e.conflict or e.status >= 500 or e.status == 429):
                    raise
                try:
                    landed = pu.node_name_of(await self.api.get_pod(ns, name)) == node
                except (ApiError, OSError, asyncio.TimeoutError):
                    landed = False
                if not landed:
                    raise
        except BaseException as e:
            # D2: the reference leaves the cache debited when the binding POST fails
            if fresh:
                self.state.rollback(uid)
                self.metrics.rollbacks.inc()
                if self.record_events and isinstance(e, ApiError):
                    self._background(self.api.create_event(
                        ns, {"kind": "Pod", "name": name, "namespace": ns, "uid": uid}, "FailedBinding",
                        f"nano-gpu bind failed: {e}"))
            raise
        t3 = time.perf_counter()
        self.state.commit(uid)
        self.metrics.pods_bound.inc()
        if self.assume_label:
            # bound, annotations on the pod with the binding: kube-scheduler is answered now and
            # the label follows (as the native writer does), retried in the background
            self._background(self._label(ns, name, pu.label_patch(node)))
        sp.phases["binding"] = t3 - t2
        self._m_binding.observe(t3 - t2)

    async def _label(self, ns: str, name: str, patch: dict) -> None:
        t = time.perf_counter()
        try:
            try:   # first attempt at once; the retry loop only after an API error
                await self.api.patch_pod(ns, name, patch)
            except ApiError as e:
                await self._retry_after(e, "patch", self.api.patch_pod, ns, name, patch)
        except (ApiError, OSError, asyncio.TimeoutError) as e:
            log.warning("bind %s/%s: label PATCH failed (%s); retrying in the background", ns, name, e)
            await self._relabel(ns, name, patch)
        self._m_patch.observe(time.perf_counter() - t)

    async def _relabel(self, ns: str, name: str, patch: dict) -> None:
        for attempt in range(6):
            await asyncio.sleep(0.05 * (2 ** attempt))
            try:
                await self.api.patch_pod(ns, name, patch)
                return
            except ApiError as e:
                if e.not_found or e.status == 422:   # gone, or no longer on this node
                    return
            except (OSError, asyncio.TimeoutError):
                pass

    def _background(self, coro) -> None:
        t = asyncio.ensure_future(coro)
        self._bg.add(t)
        t.add_done_callback(self._bg.discard)

    async def drain(self, timeout_s: float = 2.0) -> None:
        """Stop: the label PATCHes and events still in the background get `timeout_s` to land
        (a graceful shutdown leaves no bound pod without its label), then are cancelled, before
        the API client closes. The label is eventual: a process killed in between leaves a bound
        pod without it; its placement annotations came with the binding, and this extender's
        own rebuild reads those (the reference's label selector is the only reader of it)."""
        if not self._bg:
            return
        _, pending = await asyncio.wait(list(self._bg), timeout=timeout_s)
        for t in pending:
            t.cancel()
        if pending:
            await asyncio.gather(*pending, return_exceptions=True)
