"""HTTP API of the extender: one route table, two front doors.

Reference routes (pkg/routes/routes.go:19-27, 176-210; pprof.go:10-21):
  POST /scheduler/filter | /scheduler/priorities | /scheduler/bind, GET /version,
  POST /status, GET /debug/pprof/*.
Kept wire-compatible (paths, JSON keys, status codes: bind answers 500 when Error is
set, routes.go:147-168). Fixed: prioritize answers 400 on a bad body instead of
panicking (D10); /status is also served on GET (D9) and is read under the ledger's
locks (D8). Added: /metrics, /healthz, /readyz, /debug/{trace,stacks,profile,state,frag}.

Front doors:
  * `NativeServer` (default): the C++ epoll server in nanogpu._native (native/src/
    frontend.cpp) answers filter / priorities itself with no Python on the path and
    queues everything else (bind, status, metrics, debug, and requests its fast path
    declines) to `Router.dispatch` on the asyncio loop;
  * `start()` : aiohttp, every route in Python (fallback / debugging).
"""
from __future__ import annotations

import asyncio
import json
import logging
import time
from urllib.parse import parse_qs

from aiohttp import web

from .. import types as T
from ..obs import sample_profile, thread_stacks
from .verbs import Extender

log = logging.getLogger(__name__)

JSON = "application/json; charset=utf-8"
TEXT = "text/plain; charset=utf-8"
PROM = "text/plain; version=0.0.4; charset=utf-8"


def _dumps(o) -> bytes:
    return json.dumps(o, separators=(",", ":")).encode()


_BIND_OK = _dumps({"Error": ""})


def _load(raw: bytes):
    if not raw:
        raise ValueError("Please send a request body")
    return json.loads(raw)


class Router:
    """(method, path) -> handler; handlers return (status, content-type, body bytes)."""

    def __init__(self, ext: Extender, ready: asyncio.Event | None = None, extra_status=None):
        self.ext = ext
        self.ready = ready
        self.extra_status = extra_status
        self.extra_metrics = None       # () -> bytes appended to /metrics (the runtime's)
        self.native = None          # NativeServer, for /metrics
        self.serving = lambda: True  # False on a standby replica (leader election)
        g, p = "GET", "POST"
        self.table = {
            (p, "/scheduler/filter"): self.filter, (p, "/scheduler/priorities"): self.prioritize,
            (p, "/scheduler/bind"): self.bind, (p, "/scheduler/preemption"): self.preempt,
            (g, "/version"): self.version,
            (p, "/status"): self.status, (g, "/status"): self.status, (g, "/metrics"): self.metrics,
            (g, "/healthz"): self.healthz, (g, "/readyz"): self.readyz, (g, "/debug/trace"): self.trace,
            (g, "/debug/stacks"): self.stacks, (g, "/debug/pprof/goroutine/"): self.stacks,
            (g, "/debug/profile"): self.profile, (g, "/debug/pprof/profile/"): self.profile,
            (g, "/debug/state"): self.state, (g, "/debug/frag"): self.frag, (g, "/debug/pprof/"): self.pprof_index,
            (g, "/debug/pprof/cmdline/"): self.cmdline, (g, "/debug/pprof/heap/"): self.heap,
            (g, "/debug/pprof/trace/"): self.trace, (g, "/debug/pprof/threadcreate/"): self.threads,
            (g, "/debug/pprof/symbol/"): self.pprof_na, (g, "/debug/pprof/block/"): self.pprof_na,
            (g, "/debug/pprof/mutex/"): self.pprof_na,
        }
        self.paths = {path for _, path in self.table}

    async def dispatch(self, method: str, path: str, query: dict, body: bytes) -> tuple[int, str, bytes]:
        h = self.table.get((method, path))
        if path.startswith("/scheduler/") and h is not None and not self.serving():
            return 503, JSON, _dumps({"Error": "nano-gpu-scheduler: this replica is not the leader"})
        if h is None:
            if path in self.paths:
                return 405, TEXT, b"405: Method Not Allowed"
            return 404, TEXT, b"404: Not Found"
        return await h(query, body)

    # ---------------------------------------------------------------- verbs
    async def filter(self, q, body):
        try:
            args = _load(body)
        except ValueError as e:  # includes JSONDecodeError
            return 200, JSON, _dumps({"Nodes": None, "NodeNames": None, "FailedNodes": None, "Error": str(e)})
        return 200, JSON, _dumps(self.ext.filter(args))

    async def prioritize(self, q, body):
        try:
            return 200, JSON, _dumps(self.ext.prioritize(_load(body)))
        except ValueError as e:
            return 400, JSON, _dumps({"error": str(e)})

    async def bind(self, q, body):
        try:
            args = _load(body)
        except ValueError as e:
            return 500, JSON, _dumps({"Error": str(e)})
        res = await self.ext.bind(args)
        return (500 if res.get("Error") else 200), JSON, _dumps(res)

    async def preempt(self, q, body):
        try:
            return 200, JSON, _dumps(self.ext.preempt(_load(body)))
        except ValueError as e:
            return 400, JSON, _dumps({"error": str(e)})

    # ---------------------------------------------------------------- ops
    async def version(self, q, body):
        return 200, TEXT, T.VERSION.encode()

    async def status(self, q, body):
        out = self.ext.state.status()
        if self.extra_status:
            out = self.extra_status(out)
        return 200, JSON, _dumps(out)

    async def metrics(self, q, body):
        st = self.ext.state
        f = st.frag()
        m = self.ext.metrics
        m.frag_pct.set(f["frag_pct"])
        m.frag_mib.set(f["frag_mib"])
        m.free_pct.set(f["pct_free_total"])
        m.nodes.set(st.ledger.n_nodes)
        m.pods.set(st.ledger.n_pods)
        text = m.render()
        if self.native is not None:
            text += self.native.render_metrics()
        if self.extra_metrics is not None:
            text += self.extra_metrics()
        return 200, PROM, text

    async def healthz(self, q, body):
        return 200, TEXT, b"ok"

    async def readyz(self, q, body):
        if self.ready is not None and not self.ready.is_set():
            return 503, TEXT, b"informers not synced"
        if not self.serving():
            return 503, TEXT, b"standby (not the leader)"
        return 200, TEXT, b"ok"

    async def trace(self, q, body):
        return 200, JSON, _dumps(self.ext.tracer.dump(int(q.get("limit", "512")), q.get("verb")))

    async def stacks(self, q, body):
        return 200, TEXT, thread_stacks().encode()

    async def profile(self, q, body):
        secs = min(60.0, float(q.get("seconds", "5")))
        text = await asyncio.get_running_loop().run_in_executor(None, sample_profile, secs)
        return 200, TEXT, text.encode()

    async def state(self, q, body):
        st = self.ext.state
        out = {"policy": st.policy, "compat": st.options.compat, "load_aware": st.options.load_aware,
               "nodes": st.ledger.n_nodes, "pods": st.ledger.n_pods, "epoch": st.ledger.epoch,
               "plan_cache": st.ledger.cache_size, "ledger_path": st.ledger.path, "ledger_bytes": st.ledger.bytes,
               "pods_in_ledger": st.ledger.pods_on(-1)[:1000], "time": time.time()}
        if self.native is not None:
            out["native_frontend"] = self.native.fe.stats()
        return 200, JSON, _dumps(out)

    async def frag(self, q, body):
        return 200, JSON, _dumps(self.ext.state.frag(int(q.get("min_request", "0"))))

    async def pprof_index(self, q, body):
        return 200, TEXT, (b"Python/native equivalents of the reference's Go pprof routes (pprof.go:10-21):\n"
                           b"goroutine/ profile/?seconds= heap/ trace/ threadcreate/ cmdline/ symbol/ block/ mutex/\n")

    async def cmdline(self, q, body):
        import sys

        return 200, TEXT, "\x00".join(sys.argv).encode()

    async def heap(self, q, body):
        """Live Python objects by type (top 40) + tracemalloc top sites when tracing is on."""
        import collections
        import gc
        import tracemalloc

        counts = collections.Counter(type(o).__name__ for o in gc.get_objects())
        lines = [f"gc objects: {sum(counts.values())}  gc counts: {gc.get_count()}  frozen: {gc.get_freeze_count()}"]
        lines += [f"{n:10d} {t}" for t, n in counts.most_common(40)]
        if tracemalloc.is_tracing():
            lines.append("-- tracemalloc top 20")
            lines += [str(st) for st in tracemalloc.take_snapshot().statistics("lineno")[:20]]
        st = self.ext.state
        lines.append(f"-- native ledger: {st.ledger.bytes} B at {st.ledger.path or '(heap)'}, "
                     f"{st.ledger.n_nodes} nodes, {st.ledger.n_pods} pods, plan cache {st.ledger.cache_size}")
        return 200, TEXT, "\n".join(lines).encode()

    async def threads(self, q, body):
        import threading

        return 200, TEXT, "\n".join(f"{t.ident} {t.name} daemon={t.daemon}"
                                     for t in threading.enumerate()).encode()

    async def pprof_na(self, q, body):
        return 200, TEXT, (b"not applicable: verbs do not share one mutex here (per-node robust mutexes in the "
                           b"native ledger, lock-free reads for filter/priorities); see /debug/state\n")


# ------------------------------------------------------------------------ aiohttp front door
def make_app(ext: Extender, ready: asyncio.Event | None = None, extra_status=None,
             router: Router | None = None) -> web.Application:
    router = router or Router(ext, ready, extra_status)

    async def handle(request: web.Request):
        body = await request.read()
        status, ctype, out = await router.dispatch(request.method, request.path, dict(request.query), body)
        mime, _, cs = ctype.partition("; charset=")
        return web.Response(status=status, body=out, content_type=mime.split(";")[0],
                            charset=cs or None)

    app = web.Application(client_max_size=64 * 1024 * 1024)
    app.router.add_route("*", "/{tail:.*}", handle)
    app[EXTENDER_KEY] = ext
    return app


EXTENDER_KEY = web.AppKey("extender", Extender)


async def start(app: web.Application, host: str = "0.0.0.0", port: int = T.DEFAULT_PORT,
                reuse_port: bool = False) -> tuple[web.AppRunner, int]:
    runner = web.AppRunner(app, access_log=None, shutdown_timeout=2.0)
    await runner.setup()
    site = web.TCPSite(runner, host, port, reuse_port=reuse_port or None, backlog=1024)
    await site.start()
    bound = site._server.sockets[0].getsockname()[1]  # type: ignore[union-attr]
    return runner, bound


# ------------------------------------------------------------------------ native front door
class NativeServer:
    """C++ epoll front door (nanogpu._native.Frontend) bridged to the asyncio Router."""

    def __init__(self, router: Router, host: str = "0.0.0.0", port: int = T.DEFAULT_PORT, threads: int = 2):
        from ..native import core

        self.router = router
        st = router.ext.state
        self.fe = core().Frontend(st.ledger, host, port, threads)
        self.port = self.fe.port
        self._tasks: set[asyncio.Task] = set()
        self._loop: asyncio.AbstractEventLoop | None = None
        router.native = self
        self._inline_api = bool(getattr(router.ext.api, "completes_inline", False))
        self.take_wait_max_s = 0.0
        st.add_listener(self.sync_options)
        self.sync_options()

    def sync_options(self) -> None:
        st = self.router.ext.state
        self.fe.set_options(st.options, bool(st.score_normalize), bool(st.nominate), bool(st.decisive_filter),
                            int(st.priority_lead))

    def start(self) -> None:
        self._loop = asyncio.get_running_loop()
        self._loop.add_reader(self.fe.notify_fd(), self._drain)

    def _drain(self) -> None:
        reqs = self.fe.take()
        if reqs:
            # oldest request's wait between the worker's hand-off and this drain
            self.take_wait_max_s = max(self.take_wait_max_s, time.monotonic() - reqs[0][6])
        for rid, method, path, query, body, pod_json, _t, prepared in reqs:
            if prepared is not None:
                if self._inline_api:
                    self._eager(rid, self.router.ext.bind_prepared(prepared))
                else:
                    t = asyncio.ensure_future(self._prepared(rid, prepared))
                    self._tasks.add(t)
                    t.add_done_callback(self._tasks.discard)
                continue
            if pod_json:
                try:
                    self.router.ext.pods.put(json.loads(pod_json))
                except ValueError:
                    pass
            t = asyncio.ensure_future(self._one(rid, method, path, query, body))
            self._tasks.add(t)
            t.add_done_callback(self._tasks.discard)
        self.fe.flush()      # one wake-up per worker for all binds answered above

    async def _prepared(self, rid: int, p: dict) -> None:
        try:
            res = await self.router.ext.bind_prepared(p)
        except Exception as e:
            self._respond_bind(rid, None, e)
            return
        self._respond_bind(rid, res)

    def _eager(self, rid: int, coro) -> None:
        """Runs a prepared bind's coroutine in place until it first suspends. Used with
        API clients that answer in-process (`completes_inline`: the fake-cluster mode's
        store): the bind then finishes here, saving the Task allocation and two loop
        iterations per bind; if it does suspend, the rest runs in a Task that resumes
        exactly where the coroutine stopped (what asyncio's eager task factory does in
        Python >= 3.12). Network clients (aiohttp needs a current Task) use _prepared."""
        try:
            fut = coro.send(None)
        except StopIteration as done:
            self._respond_bind(rid, done.value, notify=False)
            return
        except Exception as e:
            self._respond_bind(rid, None, e, notify=False)
            return
        t = asyncio.ensure_future(self._resume(rid, coro, fut))
        self._tasks.add(t)
        t.add_done_callback(self._tasks.discard)

    async def _resume(self, rid: int, coro, fut) -> None:
        try:
            while True:
                try:
                    if fut is None:
                        await asyncio.sleep(0)          # bare yield (sleep(0))
                    else:
                        await asyncio.wait((fut,))      # the coroutine reads fut's outcome itself
                except asyncio.CancelledError as c:
                    try:
                        coro.throw(c)                   # lets the bind roll its reservation back
                    except BaseException:
                        pass
                    raise
                try:
                    fut = coro.send(None)
                except StopIteration as done:
                    self._respond_bind(rid, done.value)
                    return
        except asyncio.CancelledError:
            raise
        except Exception as e:
            self._respond_bind(rid, None, e)

    def _respond_bind(self, rid: int, res: dict | None, exc: Exception | None = None, notify: bool = True) -> None:
        if exc is not None:
            log.error("prepared bind failed", exc_info=exc)
            self.fe.respond(rid, 500, JSON, _dumps({"Error": f"internal error: {exc}"}), notify)
        elif res.get("Error"):
            self.fe.respond(rid, 500, JSON, _dumps(res), notify)
        else:
            self.fe.respond(rid, 200, JSON, _BIND_OK, notify)

    async def _one(self, rid: int, method: str, path: str, query: str, body: bytes) -> None:
        try:
            q = {k: v[-1] for k, v in parse_qs(query).items()} if query else {}
            status, ctype, out = await self.router.dispatch(method, path, q, body)
        except Exception as e:  # never leave kube-scheduler hanging
            log.exception("%s %s failed", method, path)
            status, ctype, out = 500, JSON, _dumps({"Error": f"internal error: {e}"})
        self.fe.respond(rid, status, ctype, out)

    def render_metrics(self) -> bytes:
        s = self.fe.stats()
        lines = ["# HELP nanogpu_native_verb_total verbs answered by the native front door",
                 "# TYPE nanogpu_native_verb_total counter"]
        for verb in ("filter", "priorities"):
            lines.append(f'nanogpu_native_verb_total{{verb="{verb}"}} {s[verb]["count"]}')
        lines += ["# HELP nanogpu_native_verb_seconds_total time spent in native verbs",
                  "# TYPE nanogpu_native_verb_seconds_total counter"]
        for verb in ("filter", "priorities"):
            lines.append(f'nanogpu_native_verb_seconds_total{{verb="{verb}"}} {s[verb]["seconds_total"]:.9f}')
        lines += ["# HELP nanogpu_native_deferred_total requests handed to the Python runtime",
                  "# TYPE nanogpu_native_deferred_total counter",
                  f"nanogpu_native_deferred_total {s['python']['deferred']}",
                  "# TYPE nanogpu_native_connections_total counter",
                  f"nanogpu_native_connections_total {s['connections']}",
                  "# HELP nanogpu_native_bind_handoffs_total binds answered natively with the pod another "
                  "worker process's filter parsed (shared-ledger handoff)",
                  "# TYPE nanogpu_native_bind_handoffs_total counter",
                  f"nanogpu_native_bind_handoffs_total {s.get('bind_handoffs', 0)}",
                  "# TYPE nanogpu_native_pods_published_total counter",
                  f"nanogpu_native_pods_published_total {s.get('pods_published', 0)}"]
        kw = self.fe.kube_writer_stats()
        if kw is not None:
            lines += ["# HELP nanogpu_native_binds_total binds finished by the native API writer",
                      "# TYPE nanogpu_native_binds_total counter",
                      f'nanogpu_native_binds_total{{result="ok"}} {kw["ok"]}',
                      f'nanogpu_native_binds_total{{result="error"}} {kw["failed"]}',
                      "# TYPE nanogpu_native_bind_rollbacks_total counter",
                      f"nanogpu_native_bind_rollbacks_total {kw['rollbacks']}",
                      "# TYPE nanogpu_native_api_retries_total counter",
                      f"nanogpu_native_api_retries_total {kw['retries']}",
                      "# HELP nanogpu_native_api_write_seconds_total time in the bind's API writes: the "
                      "binding and the label PATCH behind it, then label-PATCH retries",
                      "# TYPE nanogpu_native_api_write_seconds_total counter",
                      f'nanogpu_native_api_write_seconds_total{{op="binding+patch"}} {kw["binding_seconds_total"]:.9f}',
                      f'nanogpu_native_api_write_seconds_total{{op="patch_retry"}} {kw["patch_seconds_total"]:.9f}',
                      "# HELP nanogpu_native_api_timeouts_total bind API requests unanswered within the "
                      "writer's timeout (failed over to the slow path)",
                      "# TYPE nanogpu_native_api_timeouts_total counter",
                      f"nanogpu_native_api_timeouts_total {kw.get('timeouts', 0)}",
                      "# TYPE nanogpu_native_label_failures_total counter",
                      f"nanogpu_native_label_failures_total {kw['label_failures']}",
                      "# TYPE nanogpu_native_binds_inflight gauge",
                      f"nanogpu_native_binds_inflight {kw['inflight']}",
                      "# HELP nanogpu_native_api_throttled_total API answers 429 TooManyRequests (kube-apiserver's "
                      "max-in-flight admission); each was re-sent after its Retry-After",
                      "# TYPE nanogpu_native_api_throttled_total counter",
                      f"nanogpu_native_api_throttled_total {kw.get('throttled', 0)}",
                      "# TYPE nanogpu_native_bind_window_cuts_total counter",
                      f"nanogpu_native_bind_window_cuts_total {kw.get('window_cuts', 0)}",
                      "# HELP nanogpu_native_bindings_first_total bindings sent ahead of their label PATCH "
                      "because the admission window had no room for both",
                      "# TYPE nanogpu_native_bindings_first_total counter",
                      f"nanogpu_native_bindings_first_total {kw.get('bindings_first', 0)}",
                      "# HELP nanogpu_native_bind_window binds the writer keeps in flight at most now",
                      "# TYPE nanogpu_native_bind_window gauge",
                      f"nanogpu_native_bind_window {kw.get('window', 0)}"]
        return ("\n".join(lines) + "\n").encode()

    def enable_native_writes(self, config, threads: int, retries: int, record_events: bool,
                             evented: bool = True, label: bool = True, timeout_s: float = 30.0,
                             inline_io: bool = False, batch_labels: bool = False, max_binds: int = 0) -> bool:
        """Hands the bind's API writes to the front door's C++ writer threads (native/src/
        kubewriter.cpp) when the API server is a REST endpoint this process reaches with a
        bearer token or a client certificate; False (Python writes) otherwise."""
        from urllib.parse import urlsplit

        u = urlsplit(config.server)
        if u.scheme not in ("http", "https") or not u.hostname:
            return False
        tls = u.scheme == "https"
        self.fe.set_kube_writer(u.hostname, u.port or (443 if tls else 80), tls, config.token or "",
                                config.token_file or "", config.ca_file or "", config.cert_file or "",
                                config.key_file or "", bool(config.insecure), threads, retries, record_events,
                                evented, label, timeout_s, inline_io, batch_labels, max_binds)
        return True

    async def stop(self) -> None:
        if self._loop is not None:
            self._loop.remove_reader(self.fe.notify_fd())
        for t in list(self._tasks):
            try:
                await asyncio.wait_for(asyncio.shield(t), 2.0)
            except (asyncio.TimeoutError, Exception):
                pass
        self.router.ext.state.remove_listener(self.sync_options)
        await asyncio.get_running_loop().run_in_executor(None, self.fe.stop)
