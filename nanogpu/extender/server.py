"""HTTP API of the extender (aiohttp).

Reference routes (pkg/routes/routes.go:19-27, 176-210; pprof.go:10-21):
  POST /scheduler/filter | /scheduler/priorities | /scheduler/bind, GET /version,
  POST /status, GET /debug/pprof/*.
Kept wire-compatible (paths, JSON keys, status codes: bind answers 500 when Error is
set, routes.go:147-168). Fixed: prioritize answers 400 on a bad body instead of
panicking (D10); /status is also served on GET (D9) and is read under the ledger's
locks (D8). Added: /metrics, /healthz, /readyz, /debug/{trace,stacks,profile,state,frag}.
"""
from __future__ import annotations

import asyncio
import json
import logging
import time

from aiohttp import web

from .. import types as T
from ..obs import sample_profile, thread_stacks
from .verbs import Extender

log = logging.getLogger(__name__)


def _dumps(o) -> str:
    return json.dumps(o, separators=(",", ":"))


async def _read_json(request: web.Request):
    raw = await request.read()
    if not raw:
        raise ValueError("Please send a request body")
    return json.loads(raw)


def make_app(ext: Extender, ready: asyncio.Event | None = None, extra_status=None) -> web.Application:
    routes = web.RouteTableDef()

    @routes.post("/scheduler/filter")
    async def filter_route(request: web.Request):
        try:
            body = await _read_json(request)
        except ValueError as e:  # includes JSONDecodeError
            return web.json_response({"Nodes": None, "NodeNames": None, "FailedNodes": None, "Error": str(e)},
                                     dumps=_dumps)
        return web.json_response(ext.filter(body), dumps=_dumps)

    @routes.post("/scheduler/priorities")
    async def prioritize_route(request: web.Request):
        try:
            body = await _read_json(request)
            return web.json_response(ext.prioritize(body), dumps=_dumps)
        except ValueError as e:
            return web.json_response({"error": str(e)}, status=400, dumps=_dumps)

    @routes.post("/scheduler/bind")
    async def bind_route(request: web.Request):
        try:
            body = await _read_json(request)
        except ValueError as e:
            return web.json_response({"Error": str(e)}, status=500, dumps=_dumps)
        res = await ext.bind(body)
        return web.json_response(res, status=500 if res.get("Error") else 200, dumps=_dumps)

    @routes.get("/version")
    async def version(_):
        return web.Response(text=T.VERSION)

    async def status(_):
        body = ext.state.status()
        if extra_status:
            body = extra_status(body)
        return web.json_response(body, dumps=_dumps)

    routes.post("/status")(status)
    routes.get("/status")(status)

    @routes.get("/metrics")
    async def metrics(_):
        st = ext.state
        f = st.frag()
        m = ext.metrics
        m.frag_pct.set(f["frag_pct"])
        m.frag_mib.set(f["frag_mib"])
        m.free_pct.set(f["pct_free_total"])
        m.nodes.set(st.ledger.n_nodes)
        m.pods.set(st.ledger.n_pods)
        return web.Response(body=m.render(), content_type="text/plain", charset="utf-8")

    @routes.get("/healthz")
    async def healthz(_):
        return web.Response(text="ok")

    @routes.get("/readyz")
    async def readyz(_):
        if ready is not None and not ready.is_set():
            return web.Response(status=503, text="informers not synced")
        return web.Response(text="ok")

    @routes.get("/debug/trace")
    async def trace(request: web.Request):
        limit = int(request.query.get("limit", "512"))
        return web.json_response(ext.tracer.dump(limit, request.query.get("verb")), dumps=_dumps)

    @routes.get("/debug/stacks")
    @routes.get("/debug/pprof/goroutine/")
    async def stacks(_):
        return web.Response(text=thread_stacks())

    @routes.get("/debug/profile")
    @routes.get("/debug/pprof/profile/")
    async def profile(request: web.Request):
        secs = min(60.0, float(request.query.get("seconds", "5")))
        loop = asyncio.get_running_loop()
        text = await loop.run_in_executor(None, sample_profile, secs)
        return web.Response(text=text)

    @routes.get("/debug/state")
    async def state(_):
        st = ext.state
        return web.json_response({
            "policy": st.policy, "compat": st.options.compat, "load_aware": st.options.load_aware,
            "nodes": st.ledger.n_nodes, "pods": st.ledger.n_pods, "epoch": st.ledger.epoch,
            "plan_cache": st.ledger.cache_size, "ledger_path": st.ledger.path, "ledger_bytes": st.ledger.bytes,
            "pods_in_ledger": st.ledger.pods_on(-1)[:1000], "time": time.time()}, dumps=_dumps)

    @routes.get("/debug/frag")
    async def frag(request: web.Request):
        return web.json_response(ext.state.frag(int(request.query.get("min_request", "0"))), dumps=_dumps)

    @routes.get("/debug/pprof/")
    async def pprof_index(_):
        return web.Response(text="goroutine/ profile/ (Python equivalents of the reference's pprof routes)\n")

    app = web.Application(client_max_size=64 * 1024 * 1024)
    app.add_routes(routes)
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
