"""kube-apiserver's max-in-flight admission.

kube-apiserver refuses mutating requests beyond --max-mutating-requests-inflight (default 200)
with 429 TooManyRequests and `Retry-After: 1`, before handling them. The API servers here model
that (native/src/apiserver.cpp set_max_mutating_inflight, fake_apiserver Faults); the native
writer starts under the limit (Config.writer_max_binds) and, when it is pushed over, halves its
window and re-sends the refused binds after their Retry-After (kubewriter_evented.cpp, BindIo
admission). The reference binds one pod at a time under its global lock and never gets there
(/root/reference/pkg/dealer/dealer.go:155-203).
"""
from __future__ import annotations

import asyncio
import json

import aiohttp
import pytest

from nanogpu import types as T
from nanogpu.app import Config, Runtime
from nanogpu.k8s import podutil as pu
from nanogpu.topology.model import synthetic_mi355x


def _server(limit: int, latency_s: float):
    from nanogpu import _native as NN

    srv = NN.ApiServer("127.0.0.1", 0, 4, 1 << 15)
    srv.set_max_mutating_inflight(limit)
    srv.set_latency(latency_s)
    return srv


def test_native_api_server_answers_429_with_retry_after_over_the_limit():
    """Requests held by the modelled round trip count as in flight: the third concurrent PATCH
    against a limit of 2 is refused with 429 + Retry-After: 1 and does not touch the pod."""
    srv = _server(2, 0.3)

    async def main():
        p = pu.make_pod("p", [("main", 10)])
        st, _ = srv.call("POST", "/api/v1/namespaces/default/pods", json.dumps(p))   # in-process: no limit
        assert st == 201
        url = f"http://127.0.0.1:{srv.port}/api/v1/namespaces/default/pods/p"
        async with aiohttp.ClientSession() as s:
            async def patch(k):
                async with s.patch(url, data=json.dumps({"metadata": {"labels": {f"k{k}": "v"}}}),
                                   headers={"Content-Type": "application/merge-patch+json"}) as r:
                    return r.status, r.headers.get("Retry-After"), await r.json()
            got = await asyncio.gather(*(patch(k) for k in range(3)))
            async with s.get(url) as r:   # reads are not limited
                assert r.status == 200
                labels = (await r.json())["metadata"]["labels"]
        codes = sorted(g[0] for g in got)
        assert codes == [200, 200, 429], got
        refused = next(g for g in got if g[0] == 429)
        assert refused[1] == "1" and refused[2]["reason"] == "TooManyRequests"
        assert sum(1 for k in range(3) if f"k{k}" in labels) == 2
        adm = json.loads(srv.stats())["admission"]
        assert adm == {"max_mutating_inflight": 2, "peak_mutating_inflight": 2, "too_many_requests": 1}

    try:
        asyncio.run(main())
    finally:
        srv.stop()


def test_writer_starts_under_the_limit_shared_by_the_workers():
    """3/4 of the limit over the extender's processes, two requests a bind (binding + label)."""
    assert Config().writer_max_binds() == 75
    assert Config(workers=2).writer_max_binds() == 37
    assert Config(workers=2, assume_label=False).writer_max_binds() == 75
    assert Config(api_max_inflight=0).writer_max_binds() == 0          # threads x 8
    assert Config(api_inflight_share=8).writer_max_binds() == 9


@pytest.mark.parametrize("mode", ["evented", "inline"])
def test_a_burst_over_the_admission_limit_binds_every_pod_once(mode):
    """1,000 pods driven by the native kube-scheduler stand-in against a 200-request limit at a
    30 ms round trip (a loaded kube-apiserver), with the writer started far over it (375 binds,
    750 requests in flight): the server refuses the excess with 429; the writer halves its
    window, re-sends every refused
    bind after its Retry-After and ends under the limit. Every pod is bound exactly once with
    its placement annotations and label, no bind fails, and the ledger holds exactly the burst's
    demand (no double accounting)."""
    from nanogpu.sim.driver import NativeSchedulerDriver, node_capacities

    srv = _server(200, 0.03)

    async def main():
        nodes = []
        for i in range(64):
            st, body = srv.call("POST", "/api/v1/nodes", json.dumps(pu.make_node(f"n{i:02d}", 8, synthetic_mi355x(8).to_json())))
            assert st in (200, 201)
            nodes.append(json.loads(body))
        # a writer sized for a 1000-request limit: it is pushed over the real one at once
        rt = Runtime(Config(kube_api=f"http://127.0.0.1:{srv.port}", port=0, host="127.0.0.1",
                            policy_config_path="/nonexistent", bind_writer_mode=mode, api_max_inflight=1000))
        await rt.start()
        loop = asyncio.get_running_loop()
        try:
            pods = []
            for i in range(1000):
                p = pu.make_pod(f"b{i}", [("main", (10, 25, 50)[i % 3], 8 * 1024)])
                st, body = srv.call("POST", "/api/v1/namespaces/default/pods", json.dumps(p))
                assert st == 201
                pods.append(json.loads(body))
            drv = NativeSchedulerDriver("127.0.0.1", rt.bound_port, [n["metadata"]["name"] for n in nodes],
                                        node_capacities(nodes), bind_threads=512)
            res = await asyncio.wait_for(loop.run_in_executor(None, drv.run, pods), 90)
            assert res.scheduled == 1000 and res.failed == 0 and res.bind_errors == 0, \
                (res.scheduled, res.failed, res.bind_errors)
            for _ in range(500):   # the last label answers (and any throttled label re-sent)
                if rt.native.fe.kube_writer_stats()["inflight"] == 0:
                    break
                await asyncio.sleep(0.01)
            kw = rt.native.fe.kube_writer_stats()
            adm = json.loads(srv.stats())["admission"]
            print("admission", adm, {k: kw[k] for k in ("throttled", "throttle_resends", "window_cuts", "window")})
            assert adm["too_many_requests"] > 0, adm          # the server was pushed over its limit
            assert adm["peak_mutating_inflight"] <= 200
            assert kw["throttled"] > 0 and kw["throttle_resends"] > 0 and kw["window_cuts"] > 0, kw
            assert kw["failed"] == 0 and kw["rollbacks"] == 0 and kw["inflight"] == 0, kw
            assert kw["window"] < 375, kw                     # ended inside the limit
            demand = 0
            for p in pods:
                st, body = srv.call("GET", f"/api/v1/namespaces/default/pods/{pu.meta(p)['name']}", "")
                got = json.loads(body)
                assert got["spec"].get("nodeName"), got
                assert got["metadata"]["labels"].get(T.GPU_ASSUME) == "true", got
                assert T.container_annotation("main") in got["metadata"]["annotations"], got
                demand += pu.pod_demand(got)[0][0]
            assert json.loads(srv.stats())["bindings"] == 1000
            led = rt.state.ledger
            assert led.n_pods == 1000
            used = sum(100 - d["pct_free"] for n in nodes
                       for d in led.snapshot(rt.state.node_entry(n["metadata"]["name"]).id)["devices"])
            assert used == demand
        finally:
            await rt.stop()
            srv.stop()

    asyncio.run(main())


def test_a_saturated_window_sends_bindings_first_and_labels_after():
    """A burst faster than the admission window drains (a 20-request limit shared as 7 binds, a
    20 ms round trip): bindings go alone while the window has no room for a binding and its
    label, so kube-scheduler's binds keep the window's whole rate, and the labels follow in
    batches as room frees up. Every pod is bound once and labelled, nothing goes over the
    server's limit (no 429), and the ledger holds exactly the burst's demand."""
    from nanogpu.sim.driver import NativeSchedulerDriver, node_capacities

    srv = _server(20, 0.02)

    async def main():
        nodes = []
        for i in range(16):
            st, body = srv.call("POST", "/api/v1/nodes", json.dumps(pu.make_node(f"n{i:02d}", 8, synthetic_mi355x(8).to_json())))
            assert st in (200, 201)
            nodes.append(json.loads(body))
        rt = Runtime(Config(kube_api=f"http://127.0.0.1:{srv.port}", port=0, host="127.0.0.1",
                            policy_config_path="/nonexistent", api_max_inflight=20))
        assert Config(api_max_inflight=20).writer_max_binds() == 7
        await rt.start()
        loop = asyncio.get_running_loop()
        try:
            pods = []
            for i in range(300):
                p = pu.make_pod(f"s{i}", [("main", (10, 25, 50)[i % 3], 8 * 1024)])
                st, body = srv.call("POST", "/api/v1/namespaces/default/pods", json.dumps(p))
                assert st == 201
                pods.append(json.loads(body))
            drv = NativeSchedulerDriver("127.0.0.1", rt.bound_port, [n["metadata"]["name"] for n in nodes],
                                        node_capacities(nodes), bind_threads=64)
            res = await asyncio.wait_for(loop.run_in_executor(None, drv.run, pods), 90)
            assert res.scheduled == 300 and res.failed == 0 and res.bind_errors == 0
            for _ in range(1000):   # the labels trailing the bindings
                if rt.native.fe.kube_writer_stats()["inflight"] == 0:
                    break
                await asyncio.sleep(0.01)
            kw = rt.native.fe.kube_writer_stats()
            adm = json.loads(srv.stats())["admission"]
            assert kw["bindings_first"] > 100, kw         # the window was the bound
            assert adm["too_many_requests"] == 0 and adm["peak_mutating_inflight"] <= 14, adm
            assert kw["failed"] == 0 and kw["inflight"] == 0 and kw["label_failures"] == 0, kw
            for p in pods:
                st, body = srv.call("GET", f"/api/v1/namespaces/default/pods/{pu.meta(p)['name']}", "")
                got = json.loads(body)
                assert got["spec"].get("nodeName") and got["metadata"]["labels"].get(T.GPU_ASSUME) == "true", got
            assert json.loads(srv.stats())["bindings"] == 300 and rt.state.ledger.n_pods == 300
        finally:
            await rt.stop()
            srv.stop()

    asyncio.run(main())


def test_python_writer_honours_retry_after():
    """The Python bind path (fallback, and the reference's semantics) waits out a 429's
    Retry-After instead of its 5 ms backoff, and the fake API server refuses over its limit."""
    from nanogpu.extender.verbs import Extender
    from nanogpu.k8s.client import ApiError

    e = ApiError(429, "Too many requests", "TooManyRequests", 1.0)
    assert e.throttled and Extender._backoff(e, 0) == 1.0
    assert Extender._backoff(ApiError(500, "x"), 2) == pytest.approx(0.02)
    assert Extender._backoff(ApiError(429, "x"), 0) == pytest.approx(0.005)   # no header: the backoff
    # a long Retry-After is cut to 2 s: the bind holds kube-scheduler's 30 s extender request
    assert Extender._backoff(ApiError(429, "x", "TooManyRequests", 60.0), 0) == 2.0

    from nanogpu.k8s.client import KubeClient, KubeConfig
    from nanogpu.k8s.fake_apiserver import Faults, FakeKubeStore, serve

    async def main():
        store = FakeKubeStore(faults=Faults(latency_s=0.2, max_mutating_inflight=1))
        store.create_pod(pu.make_pod("p", [("main", 10)]))
        runner, port = await serve(store)
        kc = KubeClient(KubeConfig(server=f"http://127.0.0.1:{port}"))
        try:
            res = await asyncio.gather(kc.patch_pod("default", "p", {"metadata": {"labels": {"a": "1"}}}),
                                       kc.patch_pod("default", "p", {"metadata": {"labels": {"b": "1"}}}),
                                       return_exceptions=True)
            errs = [r for r in res if isinstance(r, ApiError)]
            assert len(errs) == 1 and errs[0].status == 429 and errs[0].retry_after == 1.0, res
            assert store.counts.get("throttled") == 1
        finally:
            await kc.close()
            await runner.cleanup()

    asyncio.run(main())
