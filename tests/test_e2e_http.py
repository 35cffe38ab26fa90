"""End-to-end over real HTTP: fake apiserver <- extender <- fake kube-scheduler.

SURVEY §7.3 minimum slice (BASELINE configs 1 and 2): one node with
`nano-gpu/gpu-percent: 800` and an MI355X topology annotation, one pod with a 20% limit,
filter -> priorities -> bind, then check annotations + label + binding + /status, and
that deleting the pod frees the share.
"""
import asyncio
import json

import aiohttp

from nanogpu import types as T
from nanogpu.app import Config, Runtime
from nanogpu.k8s import podutil as pu
from nanogpu.k8s.fake_apiserver import FakeKubeStore, serve
from nanogpu.sim.driver import HttpExtenderClient, SchedulerDriver, node_capacities
from nanogpu.topology.model import synthetic_mi355x


async def _wait(pred, timeout=5.0):
    loop = asyncio.get_running_loop()
    end = loop.time() + timeout
    while loop.time() < end:
        if pred():
            return True
        await asyncio.sleep(0.01)
    return pred()


async def _stack(nodes, **cfg_kw):
    store = FakeKubeStore()
    for n in nodes:
        store.add_node(n)
    api_runner, api_port = await serve(store)
    cfg = Config(kube_api=f"http://127.0.0.1:{api_port}", port=0, host="127.0.0.1",
                 policy_config_path="/nonexistent/policy.yaml", **cfg_kw)
    rt = Runtime(cfg)
    await rt.start()
    return store, api_runner, rt


def test_minimum_slice_one_pod_binpack():
    async def main():
        node = pu.make_node("mi355x-0", 8, synthetic_mi355x(8).to_json())
        store, api_runner, rt = await _stack([node])
        base = f"http://127.0.0.1:{rt.bound_port}"
        client = HttpExtenderClient(base)
        try:
            drv = SchedulerDriver(client, _ApiShim(store), ["mi355x-0"], node_capacities([node]))
            pod = pu.make_pod("p1", [("main", 20)])
            stats = await drv.run([pod])
            assert stats.scheduled == 1, stats.summary()
            got = store.get_pod("default", "p1")
            ann = got["metadata"]["annotations"]
            assert ann[T.container_annotation("main")] == "0"
            assert ann[T.ANNOTATION_GPU_ASSUME] == "true"
            # the assume label follows the binding in the writer's next label batch (<= ~1 ms)
            for _ in range(200):
                if (store.get_pod("default", "p1")["metadata"].get("labels") or {}).get(T.LABEL_GPU_ASSUME):
                    break
                await asyncio.sleep(0.005)
            got = store.get_pod("default", "p1")
            assert got["metadata"]["labels"][T.LABEL_GPU_ASSUME] == "true"
            assert got["spec"]["nodeName"] == "mi355x-0"
            assert ("default", "p1", "mi355x-0") in store.bindings
            async with aiohttp.ClientSession() as s:
                async with s.post(base + "/status") as r:
                    status = await r.json()
                async with s.get(base + "/version") as r:
                    assert (await r.text()) == T.VERSION
                async with s.get(base + "/metrics") as r:
                    assert "nanogpu_verb_latency_seconds" in await r.text()
            gpus = status["mi355x-0"]["GPUs"]
            assert gpus[0]["Percent"] == 80 and all(g["Percent"] == 100 for g in gpus[1:])
            # the operator's view of the same body (python -m nanogpu.top)
            from nanogpu import top
            table = top.render(await asyncio.get_running_loop().run_in_executor(None, top.fetch, base))
            dev0 = next(r for r in table.splitlines() if r.startswith("mi355x-0") and r.split()[1] == "0")
            assert "20%" in dev0 and "ok" in dev0
            assert "1 nodes, 8 devices, 7.8 device-equivalents free, 10.3% of the free compute" in table
            # delete frees the share (reference only Forgets on delete: D3)
            store.delete_pod("default", "p1")
            assert await _wait(lambda: rt.state.status()["mi355x-0"]["GPUs"][0]["Percent"] == 100)
        finally:
            await client.close()
            await rt.stop()
            await api_runner.cleanup()

    asyncio.run(main())


class _ApiShim:
    """Creates pods directly in the store (the driver's kubectl)."""

    def __init__(self, store):
        self.store = store

    async def create_pod(self, pod):
        return self.store.create_pod(pod)


def test_filter_requires_node_cache_capable_or_nodes():
    async def main():
        node = pu.make_node("n0", 2)
        store, api_runner, rt = await _stack([node])
        base = f"http://127.0.0.1:{rt.bound_port}"
        try:
            async with aiohttp.ClientSession() as s:
                body = {"Pod": pu.make_pod("x", [("c", 10)])}
                async with s.post(base + "/scheduler/filter", data=json.dumps(body)) as r:
                    res = await r.json()
                assert res["Error"] == T.FILTER_NODE_CACHE_ERROR
                # nodeCacheCapable=false flavour: full Node objects (the reference rejects this)
                body["Nodes"] = {"items": [node]}
                async with s.post(base + "/scheduler/filter", data=json.dumps(body)) as r:
                    res = await r.json()
                assert res["Error"] == "" and [pu.meta(n)["name"] for n in res["Nodes"]["items"]] == ["n0"]
                # bad JSON on priorities: 400, not a crash (D10)
                async with s.post(base + "/scheduler/priorities", data=b"{nope") as r:
                    assert r.status == 400
                # bind of an unknown pod: 500 with Error set (routes.go:147-168)
                async with s.post(base + "/scheduler/bind", data=json.dumps(
                        {"PodName": "ghost", "PodNamespace": "default", "PodUID": "u", "Node": "n0"})) as r:
                    assert r.status == 500 and (await r.json())["Error"]
        finally:
            await rt.stop()
            await api_runner.cleanup()

    asyncio.run(main())


def test_burst_spread_mixed_percent_no_overcommit():
    """BASELINE config 3 (scaled): mixed {10,25,50} burst, spread policy, 4 nodes."""
    async def main():
        nodes = [pu.make_node(f"n{i}", 8, synthetic_mi355x(8).to_json()) for i in range(4)]
        store, api_runner, rt = await _stack(nodes, priority="spread")
        client = HttpExtenderClient(f"http://127.0.0.1:{rt.bound_port}")
        try:
            import random

            rng = random.Random(1)
            pods = [pu.make_pod(f"p{i}", [("c", rng.choice([10, 25, 50]))]) for i in range(120)]
            drv = SchedulerDriver(client, _ApiShim(store), [f"n{i}" for i in range(4)], node_capacities(nodes))
            stats = await drv.run(pods)
            assert stats.scheduled + stats.failed == 120
            # device-level invariant from the API objects themselves
            used = {}
            for p in store.pods.values():
                if not pu.node_name_of(p):
                    continue
                for c, (pct, _) in zip(pu.containers(p), pu.pod_demand(p)):
                    idx = pu.container_assignment(p, c["name"])[0]
                    used[(pu.node_name_of(p), idx)] = used.get((pu.node_name_of(p), idx), 0) + pct
            assert used and max(used.values()) <= 100
            st = rt.state.status()
            for (n, i), u in used.items():
                assert st[n]["GPUs"][i]["Percent"] == 100 - u
        finally:
            await client.close()
            await rt.stop()
            await api_runner.cleanup()

    asyncio.run(main())


def test_debug_routes_reference_pprof_paths():
    """Every reference pprof path (pprof.go:10-21) answers, plus the added debug routes."""
    async def main():
        node = pu.make_node("n0", 2)
        store, api_runner, rt = await _stack([node])
        base = f"http://127.0.0.1:{rt.bound_port}"
        try:
            async with aiohttp.ClientSession() as s:
                for p in ("", "cmdline/", "profile/?seconds=0.05", "symbol/", "trace/", "heap/", "goroutine/",
                          "block/", "threadcreate/", "mutex/"):
                    async with s.get(f"{base}/debug/pprof/{p}") as r:
                        assert r.status == 200, p
                for p in ("/debug/trace", "/debug/stacks", "/debug/state", "/debug/frag", "/healthz", "/readyz",
                          "/metrics", "/status"):
                    async with s.get(base + p) as r:
                        assert r.status == 200, p
        finally:
            await rt.stop()
            await api_runner.cleanup()

    asyncio.run(main())


def test_client_follows_a_rotated_service_account_token(tmp_path):
    """Projected service-account tokens rotate while the extender runs: the client re-reads
    the token file when it changes and retries once after a 401."""
    from aiohttp import web

    from nanogpu.k8s.client import KubeClient, KubeConfig

    tok = tmp_path / "token"
    tok.write_text("t1\n")
    valid = {"tok": "t1"}
    seen = []

    async def get_pod(request):
        seen.append(request.headers.get("Authorization"))
        if request.headers.get("Authorization") != f"Bearer {valid['tok']}":
            return web.json_response({"kind": "Status", "message": "Unauthorized", "reason": "Unauthorized"},
                                     status=401)
        return web.json_response({"metadata": {"name": request.match_info["name"]}})

    async def main():
        app = web.Application()
        app.router.add_get("/api/v1/namespaces/{ns}/pods/{name}", get_pod)
        runner = web.AppRunner(app)
        await runner.setup()
        site = web.TCPSite(runner, "127.0.0.1", 0)
        await site.start()
        port = site._server.sockets[0].getsockname()[1]
        c = KubeClient(KubeConfig(server=f"http://127.0.0.1:{port}", token="t1", token_file=str(tok)),
                       token_check_s=3600.0)
        try:
            assert (await c.get_pod("default", "a"))["metadata"]["name"] == "a"
            tok.write_text("t2\n")                      # kubelet rotates the file
            valid["tok"] = "t2"                         # the old token stops working
            assert (await c.get_pod("default", "b"))["metadata"]["name"] == "b"
            assert seen == ["Bearer t1", "Bearer t1", "Bearer t2"]
            assert (await c.get_pod("default", "c"))["metadata"]["name"] == "c"
            assert seen[-1] == "Bearer t2"
        finally:
            await c.close()
            await runner.cleanup()

    asyncio.run(main())


def test_top_cli_reports_an_unreachable_extender(capsys):
    from nanogpu import top

    assert top.main(["--url", "http://127.0.0.1:9"]) == 1      # discard port: refused
    assert "nanogpu.top: http://127.0.0.1:9" in capsys.readouterr().err
    st = {"n1": {"GPUs": [{"Percent": 50, "PercentTotal": 100, "MemoryMiB": 1024, "MemoryMiBTotal": 4096,
                           "MemoryPool": 0, "GPU": 0, "Partition": 0, "Healthy": True,
                           "MemoryBoundTenants": 1, "HBMHot": True},
                          {"Percent": 100, "PercentTotal": 100, "MemoryMiB": 1024, "MemoryMiBTotal": 4096,
                           "MemoryPool": 0, "GPU": 0, "Partition": 1, "Healthy": False}]}}
    out = top.render(st).splitlines()
    assert "50%" in out[1] and "(pool)" not in out[1]
    assert out[1].endswith("ok  streaming x1  HBM-hot")            # declared + measured streamers
    assert "streaming" not in out[2] and "HBM-hot" not in out[2]
    assert "(pool)" in out[2] and "UNHEALTHY" in out[2]          # second member of one HBM pool
    assert "1.5 device-equivalents free, 33.3% of the free compute" in out[-1]
