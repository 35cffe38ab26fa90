"""Control plane: pod/node controllers, restart rebuild, policy hot reload, Prometheus
telemetry, API fault injection and concurrent-bind invariants.

Reference behaviours covered (and the defects fixed): controller
allocate/release (controller.go:210-243; D3 release on delete, D4 no 1 s sleep), rebuild
from annotations (dealer.go:58-72, 271-301; D14 completed pods skipped), policy reload
(context.go:44-59; D7 reload reaches scheduling), Prometheus query + fallback
(prometheus.go:68-83; D12 errors surfaced), bind rollback (D2) and retries (D1).
"""
import asyncio
import time
import json
import math

import pytest
from aiohttp import web

from nanogpu import _native as N
from nanogpu import types as T
from nanogpu.app import Config, Runtime
from nanogpu.config.policy import MetricQuery, PolicySpec, Period, parse_duration, parse_policy
from nanogpu.extender.verbs import Extender
from nanogpu.k8s import podutil as pu
from nanogpu.k8s.fake_apiserver import Faults, FakeKubeStore, InProcKube
from nanogpu.state.cluster import ClusterState
from nanogpu.telemetry.poller import LoadPoller
from nanogpu.telemetry.prom import PromClient, PromError
from nanogpu.topology.model import synthetic_mi355x


async def wait_for(pred, timeout=5.0):
    end = asyncio.get_running_loop().time() + timeout
    while asyncio.get_running_loop().time() < end:
        if pred():
            return True
        await asyncio.sleep(0.005)
    return pred()


def node(name="n0", gpus=8, partition="SPX"):
    t = synthetic_mi355x(gpus, partition)
    return pu.make_node(name, len(t.devices), t.to_json(), {"amd.com/gpu.present": "true"})


def annotated(name, node_name, plan, pct=20, phase="Running"):
    p = pu.make_pod(name, [(f"c{i}", pct) for i in range(len(plan))])
    p["metadata"]["annotations"].update({T.container_annotation(f"c{i}"): ",".join(map(str, idx))
                                         for i, idx in enumerate(plan)})
    p["metadata"]["annotations"][T.ANNOTATION_GPU_ASSUME] = "true"
    p["metadata"]["labels"][T.LABEL_GPU_ASSUME] = "true"
    p["spec"]["nodeName"] = node_name
    p["status"]["phase"] = phase
    return p


async def runtime(store, **kw):
    rt = Runtime(Config(port=0, host="127.0.0.1", policy_config_path=kw.pop("policy", "/nonexistent"), **kw),
                 api=InProcKube(store))
    await rt.start()
    return rt


def free(rt, n="n0"):
    return [g["Percent"] for g in rt.state.status()[n]["GPUs"]]


# ----------------------------------------------------------------------------- controllers
def test_controller_allocates_foreign_pods_and_releases_on_completion_and_delete():
    async def main():
        store = FakeKubeStore()
        store.add_node(node())
        rt = await runtime(store)
        try:
            store.create_pod(annotated("a", "n0", [[3]], 30))
            store.create_pod(annotated("b", "n0", [[3], [5]], 20))
            assert await wait_for(lambda: free(rt)[3] == 50 and free(rt)[5] == 80)
            store.set_phase("default", "a", "Succeeded")             # completed -> release
            assert await wait_for(lambda: free(rt)[3] == 80)
            store.delete_pod("default", "b")                          # D3: delete releases
            assert await wait_for(lambda: free(rt)[3] == 100 and free(rt)[5] == 100)
            # same name, new object: the old incarnation is released
            store.create_pod(annotated("c", "n0", [[1]], 50))
            assert await wait_for(lambda: free(rt)[1] == 50)
            store.delete_pod("default", "c")
            store.create_pod(annotated("c", "n0", [[2]], 50))
            assert await wait_for(lambda: free(rt)[1] == 100 and free(rt)[2] == 50)
        finally:
            await rt.stop()

    asyncio.run(main())


def test_restart_rebuilds_ledger_from_annotations_skipping_completed():
    async def main():
        store = FakeKubeStore()
        store.add_node(node())
        store.create_pod(annotated("a", "n0", [[0]], 40))
        store.create_pod(annotated("b", "n0", [[0], [7]], 30))
        store.create_pod(annotated("done", "n0", [[6]], 90, phase="Succeeded"))   # D14
        pend = pu.make_pod("pending", [("c", 10)])
        store.create_pod(pend)
        rt = await runtime(store)
        try:
            f = free(rt)
            assert f[0] == 30 and f[7] == 70 and f[6] == 100 and rt.state.ledger.n_pods == 2
        finally:
            await rt.stop()

    asyncio.run(main())


def test_restart_puts_back_an_assume_label_the_last_incarnation_did_not_write():
    """the bind answers once the binding (placement annotations) landed and the
    reference's `nano-gpu/assume` label follows; a process killed in between leaves a placed pod
    without the label, which the reference lists assumed pods by (dealer.go:59, 280). The next
    start's relist re-applies it, guarded by the pod's node; a completed pod, a pod without the
    placement and a pod already labelled are left alone."""
    async def main():
        store = FakeKubeStore()
        store.add_node(node())
        for name, phase in (("placed", "Running"), ("done", "Succeeded")):
            p = annotated(name, "n0", [[2]], 40, phase=phase)
            del p["metadata"]["labels"][T.LABEL_GPU_ASSUME]
            store.create_pod(p)
        store.create_pod(annotated("labelled", "n0", [[3]], 40))
        foreign = pu.make_pod("foreign", [("c", 10)])
        foreign["spec"]["nodeName"] = "n0"
        store.create_pod(foreign)
        patches_before = store.counts.get("patch_pod", 0)
        rt = await runtime(store)
        try:
            ctl = rt.controllers[-1]
            assert await wait_for(lambda: ctl.relabeled == 1)
            labels = {n: (store.get_pod("default", n)["metadata"].get("labels") or {}).get(T.LABEL_GPU_ASSUME)
                      for n in ("placed", "done", "labelled", "foreign")}
            assert labels == {"placed": "true", "done": None, "labelled": "true", "foreign": None}, labels
            assert store.counts.get("patch_pod", 0) - patches_before == 1
            assert free(rt)[2] == 60 and free(rt)[3] == 60      # the rebuild itself is unchanged
        finally:
            await rt.stop()

    asyncio.run(main())


def test_node_capacity_change_and_delete():
    async def main():
        store = FakeKubeStore()
        store.add_node(node("n0", 8))
        rt = await runtime(store)
        try:
            assert len(free(rt)) == 8
            store.add_node(node("n0", 4))                     # D20: capacity refresh
            assert await wait_for(lambda: len(free(rt)) == 4)
            store.delete_node("n0")
            assert await wait_for(lambda: "n0" not in rt.state.status())
        finally:
            await rt.stop()

    asyncio.run(main())


# ----------------------------------------------------------------------------- policy
def test_policy_parse_and_durations():
    assert parse_duration("15s") == 15 and parse_duration("1m30s") == 90 and parse_duration("500ms") == 0.5
    with pytest.raises(ValueError):
        parse_duration("15 parsecs")
    spec = parse_policy("""
apiVersion: v1
kind: public-dynamic-scheduler
spec:
  syncPeriod: [{name: gpu_core_usage_avg, period: 15s}, {name: gpu_memory_usage_avg, period: 1m}]
  priority: [{name: x, weight: 2}]
  scheduling: {policy: spread, compat: true, topologyWeight: 2.5, scoreNormalize: true}
  metricsPreset: amd
""")
    assert spec.period_of("gpu_core_usage_avg") == 15 and spec.active_duration("gpu_memory_usage_avg") == 360
    assert spec.policy == "spread" and spec.compat and spec.topology_weight == 2.5 and spec.score_normalize
    assert "gpu_gfx_activity" in spec.query_for(T.GPU_CORE_USAGE_METRIC).query
    assert "cardNode" in spec.query_for("other").fallback
    with pytest.raises(ValueError):
        parse_policy("spec: {scheduling: {policy: magic}}")
    # the node agent's own exporter (nanogpu/agent/metrics.py) as the telemetry source
    agent = parse_policy("spec: {metricsPreset: nanogpu-agent}")
    q = agent.query_for(T.GPU_CORE_USAGE_METRIC).query.format(node="n0", card=3)
    assert q == 'avg_over_time(nanogpu_device_busy_percent{node="n0",device="3"}[1m]) / 100'
    assert "nanogpu_device_vram_used_bytes" in agent.query_for(T.GPU_MEMORY_USAGE_METRIC).query
    with pytest.raises(ValueError):
        parse_policy("spec: {metricsPreset: nvidia}")


def test_policy_hot_reload_reaches_scheduling(tmp_path):
    async def main():
        store = FakeKubeStore()
        store.add_node(node())
        path = tmp_path / "policy.yaml"
        path.write_text("spec: {scheduling: {policy: binpack}}\n")
        rt = await runtime(store, policy=str(path), policy_reload_s=0.05)
        try:
            assert rt.state.policy == "binpack"
            await asyncio.sleep(0.02)
            path.write_text("spec: {scheduling: {policy: spread, scoreNormalize: true}}\n")
            import os
            os.utime(path, (os.stat(path).st_atime, os.stat(path).st_mtime + 5))
            assert await wait_for(lambda: rt.state.policy == "spread" and rt.state.score_normalize)
            # a broken file keeps the last good policy (reference panics: stats.go:19)
            path.write_text("spec: [unclosed\n")
            os.utime(path, (os.stat(path).st_atime, os.stat(path).st_mtime + 10))
            await asyncio.sleep(0.2)
            assert rt.state.policy == "spread" and rt.watcher.errors >= 1
        finally:
            await rt.stop()

    asyncio.run(main())


# ----------------------------------------------------------------------------- telemetry
async def fake_prometheus(series):
    """series: {metric: {(node, card): [values...]}} -> /api/v1/query vectors."""
    hits = []

    async def query(request):
        q = request.query["query"]
        hits.append(q)
        if "broken" in q:
            return web.json_response({"status": "error", "error": "bad query"}, status=400)
        if any(f'"{n}"' in q for n in series.get("slow_nodes", ())):
            await asyncio.sleep(2)                       # an exporter that hangs
        fail = series.get("fail_nodes", ())
        if any(f'"{n}"' in q for n in fail):
            return web.json_response({"status": "error", "error": "exporter down"}, status=503)
        for metric, by in series.items():
            if metric in ("fail_nodes", "slow_nodes"):
                continue
            if q.startswith(metric) and "node" not in q:
                # cluster-wide query: every node and card (plus one series with no node label)
                res = [{"metric": {"node": n, "card": str(c)}, "value": [0, str(v)]}
                       for (n, c), vals in by.items() for v in vals]
                res.append({"metric": {"card": "0"}, "value": [0, "0.99"]})
                return web.json_response({"status": "success", "data": {"resultType": "vector", "result": res}})
            if q.startswith(metric) and 'card="' not in q and 'cardNode="' not in q:
                # batched query: every card of the node, each series labelled with its card
                res = [{"metric": {"node": n, "card": str(c)}, "value": [0, str(v)]}
                       for (n, c), vals in by.items() if f'"{n}"' in q for v in vals]
                return web.json_response({"status": "success", "data": {"resultType": "vector", "result": res}})
            if q.startswith(metric):
                for (n, c), vals in by.items():
                    if f'"{n}"' in q and (f'card="{c}"' in q or f'cardNode="{c}"' in q):
                        if "cardNode" in q and by.get("primary_only"):
                            continue
                        return web.json_response({"status": "success", "data": {"resultType": "vector", "result": [
                            {"metric": {"node": n}, "value": [0, str(v)]} for v in vals]}})
        return web.json_response({"status": "success", "data": {"resultType": "vector", "result": []}})

    app = web.Application()
    app.router.add_get("/api/v1/query", query)
    runner = web.AppRunner(app)
    await runner.setup()
    site = web.TCPSite(runner, "127.0.0.1", 0)
    await site.start()
    return runner, site._server.sockets[0].getsockname()[1], hits


def test_prom_client_semantics():
    async def main():
        runner, port, hits = await fake_prometheus({
            "gpu_core_usage_avg": {("n0", 0): [0.2, 0.7], ("n0", 1): [float("nan")], ("n0", 2): [-3]}})
        c = PromClient(f"http://127.0.0.1:{port}")
        try:
            q = MetricQuery('{metric}{{node=~"{node}",card="{card}"}} /100', '{metric}{{node="{node}",cardNode="{card}"}} /100')
            assert await c.query_latest("n0", "gpu_core_usage_avg", 0, q) == 0.7      # last sample wins
            assert await c.query_latest("n0", "gpu_core_usage_avg", 1, q) == 0.0      # NaN -> 0
            assert await c.query_latest("n0", "gpu_core_usage_avg", 2, q) == 0.0      # negative -> 0
            assert await c.query_latest("n0", "gpu_core_usage_avg", 9, q) is None
            assert any("cardNode" in h for h in hits)                                 # fallback tried
            with pytest.raises(PromError):                                             # D12: not swallowed
                await c.query("broken")
        finally:
            await c.close()
            await runner.cleanup()

    asyncio.run(main())


def test_load_poller_feeds_ledger_remain_load():
    async def main():
        runner, port, _ = await fake_prometheus({
            "gpu_core_usage_avg": {("n0", 0): [0.95], ("n0", 1): [0.05]},
            "gpu_memory_usage_avg": {("n0", 0): [0.91]}})
        st = ClusterState(load_aware=True)
        n = node("n0", 2)
        st.register_node(n)
        spec = PolicySpec(sync_period=(Period("gpu_core_usage_avg", 15), Period("gpu_memory_usage_avg", 15)))
        poller = LoadPoller(st, PromClient(f"http://127.0.0.1:{port}"), lambda: [n], spec=spec, base_backoff_s=0.01)
        try:
            await poller.sync_metric("gpu_core_usage_avg")
            await poller.sync_metric("gpu_memory_usage_avg")
            gpus = st.status()["n0"]["GPUs"]
            # usage = ceil(10*0.95)/10 + ceil(10*0.91)/10 = 2.0 -> RemainLoad 0; card 1: 0.1 -> 2 - 0 = 2
            assert gpus[0]["RemainLoad"] == 0 and gpus[1]["RemainLoad"] == 2
            # stale samples age out (period + 5 min)
            poller.refresh_node("n0", 2, now=1e12)
            assert st.status()["n0"]["GPUs"][0]["RemainLoad"] == 2
        finally:
            await poller.prom.close()
            await runner.cleanup()

    asyncio.run(main())


def test_load_poller_one_query_per_node_and_a_failing_node_never_delays_the_others():
    """Reference node.go:57-83: a failing `node/metric` key is re-queued with rate limiting
    while the other keys keep their period. Here one exporter hangs and one answers 503;
    every other node is refreshed each period, with one query per node for all its cards."""
    async def main():
        names = [f"n{i}" for i in range(6)]
        series = {"gpu_core_usage_avg": {(n, c): [0.3] for n in names for c in range(8)},
                  "slow_nodes": ("n1",), "fail_nodes": ("n2",)}
        runner, port, hits = await fake_prometheus(series)
        st = ClusterState(load_aware=True)
        nodes = [node(n, 8) for n in names]
        for n in nodes:
            st.register_node(n)
        spec = PolicySpec(sync_period=(Period("gpu_core_usage_avg", 0.05),))
        poller = LoadPoller(st, PromClient(f"http://127.0.0.1:{port}"), lambda: nodes, spec=spec,
                            base_backoff_s=10.0, concurrency=4)
        try:
            poller.restart()
            await asyncio.sleep(0.6)
            healthy = [n for n in names if n not in ("n1", "n2")]
            # ~12 periods went by: every healthy node was refreshed in (nearly) all of them
            for n in healthy:
                t = poller.store.data[(n, "gpu_core_usage_avg", 0)].t
                assert asyncio.get_running_loop().time() - t < 0.2, n
            per_node = {n: sum(1 for h in hits if f'"{n}"' in h) for n in names}
            assert min(per_node[n] for n in healthy) >= 8, per_node
            assert all('card="' not in h for h in hits)          # batched: no per-card queries
            assert ("n2", "gpu_core_usage_avg", 0) not in poller.store.data and poller.errors >= 1
            # n2's key was re-queued with backoff after each failure, then dropped after 5 as in
            # the reference (it comes back with the next period's tick)
            assert poller.queue.dropped >= 1 or poller.queue.retries.get("n2/gpu_core_usage_avg", 0) >= 1
            assert st.status()["n0"]["GPUs"][7]["RemainLoad"] == 2 - 0   # ceil(3)/10 -> usage 0.3
        finally:
            await poller.stop()
            await poller.prom.close()
            await runner.cleanup()

    asyncio.run(main())


def test_load_aware_spread_moves_off_the_loaded_device():
    """End to end: Prometheus samples -> poller -> ledger -> placement changes with the load."""
    async def main():
        series = {"gpu_core_usage_avg": {("n0", 0): [0.95], ("n0", 1): [0.05]}}
        runner, port, _ = await fake_prometheus(series)
        st = ClusterState(policy="spread", load_aware=True)
        n = node("n0", 2)
        st.register_node(n)
        spec = PolicySpec(sync_period=(Period("gpu_core_usage_avg", 15),))
        poller = LoadPoller(st, PromClient(f"http://127.0.0.1:{port}"), lambda: [n], spec=spec)
        nid = st.node_entry("n0").id
        try:
            await poller.sync_metric("gpu_core_usage_avg")
            _, plan, _ = st.ledger.assume(nid, [(10, 0)], st.options)
            assert plan == [[1]]                      # GPU 0 is busy
            series["gpu_core_usage_avg"] = {("n0", 0): [0.05], ("n0", 1): [0.95]}
            await poller.sync_metric("gpu_core_usage_avg")
            _, plan, _ = st.ledger.assume(nid, [(10, 0)], st.options)
            assert plan == [[0]]                      # the load moved, so does the pod
        finally:
            await poller.prom.close()
            await runner.cleanup()

    asyncio.run(main())


# ----------------------------------------------------------------------------- faults
def _ext(store, **kw):
    st = ClusterState()
    for n in store.nodes.values():
        st.register_node(n)
    return st, Extender(st, InProcKube(store), **kw)


async def _bind(ext, store, pod, node_name="n0"):
    m = pu.meta(pod)
    ext.filter({"Pod": pod, "NodeNames": [node_name]})
    return await ext.bind({"PodName": m["name"], "PodNamespace": m["namespace"], "PodUID": m["uid"],
                           "Node": node_name})


def test_bind_retries_transient_5xx_and_rolls_back_on_permanent_failure():
    async def main():
        store = FakeKubeStore(faults=Faults(bind_error_rate=0.5, seed=3))
        store.add_node(node("n0", 2))
        st, ext = _ext(store, api_retries=4)
        ok = 0
        for i in range(20):
            p = store.create_pod(pu.make_pod(f"p{i}", [("c", 5)]))
            r = await _bind(ext, store, p)
            ok += r["Error"] == ""
        assert ok >= 15                                     # retried through 50 % 5xx
        store.faults.bind_error_rate = 1.0
        before = st.status()["n0"]["GPUs"][0]["Percent"]
        p = store.create_pod(pu.make_pod("doomed", [("c", 10)]))
        r = await _bind(ext, store, p)
        assert r["Error"] and st.status()["n0"]["GPUs"][0]["Percent"] == before     # D2 rollback
        await asyncio.sleep(0.01)
        ann = store.get_pod("default", "doomed")["metadata"].get("annotations") or {}
        assert T.ANNOTATION_GPU_ASSUME not in ann                                   # un-annotated
        assert any(e["reason"] == "FailedBinding" for e in store.events)

    asyncio.run(main())


def test_status_dumps_the_plan_cache_valid_at_the_current_generation():
    """/status carries each node's cached plans like the reference's NodeInfo.PlanCache
    (node.go:18-23); a change to the node (a bind) invalidates them."""
    store = FakeKubeStore()
    store.add_node(node("n0", 2))
    st, ext = _ext(store)
    st.nominate = False   # (a one-node filter nominates: the node would change under the dump)
    p = store.create_pod(pu.make_pod("a", [("c", 30)]))
    ext.filter({"Pod": p, "NodeNames": ["n0"]})
    big = store.create_pod(pu.make_pod("b", [("c", 100), ("d", 100), ("e", 100)]))
    ext.filter({"Pod": big, "NodeNames": ["n0"]})
    cache = st.status()["n0"]["PlanCache"]
    fits = [v for v in cache.values() if v["Fits"]]
    assert len(fits) == 1 and fits[0]["GPUIndexes"] in ([[0]], [[1]]) and fits[0]["Score"] > 0
    assert any(not v["Fits"] and v["GPUIndexes"] == [] for v in cache.values())   # 3 GPUs on a 2-GPU node
    json.dumps(st.status())
    r = asyncio.run(_bind(ext, store, p))
    assert r["Error"] == ""
    assert st.status()["n0"]["PlanCache"] == {}      # computed at an older generation


def test_bind_conflict_on_already_bound_same_node_is_success():
    async def main():
        store = FakeKubeStore()
        store.add_node(node("n0", 2))
        st, ext = _ext(store)
        p = store.create_pod(pu.make_pod("a", [("c", 20)]))
        assert (await _bind(ext, store, p))["Error"] == ""
        # kube-scheduler retries the same bind (e.g. after a timeout): idempotent
        assert (await _bind(ext, store, p))["Error"] == ""
        assert st.status()["n0"]["GPUs"][0]["Percent"] == 80
        # a completed pod is refused (bind.go:46-50)
        q = store.create_pod(pu.make_pod("b", [("c", 20)]))
        store.set_phase("default", "b", "Failed")
        ext.pods.d.clear()
        assert "completed" in (await _bind(ext, store, store.get_pod("default", "b")))["Error"]

    asyncio.run(main())


def test_concurrent_binds_never_overcommit_with_api_latency():
    async def main():
        store = FakeKubeStore(faults=Faults(latency_s=0.001))
        store.add_node(node("n0", 2))
        st, ext = _ext(store)
        pods = [store.create_pod(pu.make_pod(f"p{i}", [("c", 30)])) for i in range(20)]
        # all filters first (every one sees room), then all binds race
        for p in pods:
            ext.filter({"Pod": p, "NodeNames": ["n0"]})
        res = await asyncio.gather(*[ext.bind({"PodName": pu.meta(p)["name"], "PodNamespace": "default",
                                                "PodUID": pu.meta(p)["uid"], "Node": "n0"}) for p in pods])
        ok = sum(r["Error"] == "" for r in res)
        assert ok == 6                                       # 3 x 30 % per device, 2 devices
        used = {}
        for p in store.pods.values():
            if pu.node_name_of(p):
                i = pu.container_assignment(p, "c")[0]
                used[i] = used.get(i, 0) + 30
        assert all(v <= 100 for v in used.values())
        assert [g["Percent"] for g in st.status()["n0"]["GPUs"]] == [100 - used.get(0, 0), 100 - used.get(1, 0)]

    asyncio.run(main())


def test_reservation_ttl_sweeper_releases_lost_binds():
    st = ClusterState()
    st.register_node(node("n0", 1))
    pod = pu.make_pod("lost", [("c", 40)])
    st.reserve(pod, "n0")                 # a worker reserved, then died before commit
    assert st.status()["n0"]["GPUs"][0]["Percent"] == 60
    assert st.sweep_reservations(3600.0) == []
    assert st.sweep_reservations(0.0) == [pu.pod_uid(pod)]
    assert st.status()["n0"]["GPUs"][0]["Percent"] == 100
    assert not math.isnan(0.0)


def test_sweeps_never_release_a_pod_that_moved_on():
    """The scans run off the event loop, so a bind can commit a reservation (or adopt a
    nomination) between the scan and the release: those releases are state-checked."""
    st = ClusterState()
    st.register_node(node("n0", 1))
    pod = pu.make_pod("racer", [("c", 40)])
    st.reserve(pod, "n0")
    uid = pu.pod_uid(pod)
    assert st.ledger.expired_reservations(0.0) == [uid]
    st.commit(uid)                                    # the bind commits after the scan
    assert st.ledger.drop_reservation(uid) != N.OK    # the sweep's release is a no-op
    assert st.status()["n0"]["GPUs"][0]["Percent"] == 60
    assert st.sweep_reservations(0.0) == []


# ----------------------------------------------------------------------------- preemption
def test_preemption_verb_keeps_only_nodes_where_the_victims_free_a_fitting_device():
    """preemptVerb (not in the reference): kube-scheduler frees gpu-percent as a node-wide
    scalar. A 100 % pod needs one whole device, so victims spread over two devices do not
    make room even though their percents add up."""
    st = ClusterState(policy="binpack")
    for n in ("n0", "n1"):
        st.register_node(node(n, 2))
    pods = {}
    for name, nd in (("a", "n0"), ("x", "n0"), ("b", "n1"), ("c", "n1")):
        pods[name] = p = pu.make_pod(name, [("m", 50)])
        st.reserve(p, nd)
        st.commit(pu.pod_uid(p))
    # n0: a and x share device 0 (binpack) and device 1 is free -> take x's device 1 away
    hog = pu.make_pod("hog", [("m", 100)])
    st.reserve(hog, "n0")
    st.commit(pu.pod_uid(hog))
    assert sorted(free_of(st, "n0")) == [0, 0] and sorted(free_of(st, "n1")) == [0, 100]
    ext = Extender(st, api=None)
    uid = pu.pod_uid
    big = pu.make_pod("big", [("m", 100)])
    body = {"Pod": big, "NodeNameToMetaVictims": {
        "n0": {"Pods": [{"UID": uid(pods["a"])}], "NumPDBViolations": 0},           # 50 % of device 0 only
        "n1": {"Pods": [{"UID": uid(pods["b"])}, {"UID": uid(pods["c"])}], "NumPDBViolations": 1},
        "ghost": {"Pods": [{"UID": "nope"}]}}}
    res = ext.preempt(body)
    assert set(res["NodeNameToMetaVictims"]) == {"n1"}
    assert res["NodeNameToMetaVictims"]["n1"] == {"Pods": [{"UID": uid(pods["b"])}, {"UID": uid(pods["c"])}],
                                                  "NumPDBViolations": 1}
    # victims holding a whole device on n0 (the hog) do make room there; nothing changed in the ledger
    res = ext.preempt({"Pod": big, "NodeNameToMetaVictims": {"n0": {"Pods": [{"UID": uid(hog)}]}}})
    assert set(res["NodeNameToMetaVictims"]) == {"n0"}
    assert sorted(free_of(st, "n0")) == [0, 0]
    # the full-pod form (nodeCacheCapable=false) carries pod objects
    res = ext.preempt({"Pod": big, "NodeNameToVictims": {"n1": {"Pods": [pods["b"], pods["c"]]}}})
    assert set(res["NodeNameToMetaVictims"]) == {"n1"}
    with pytest.raises(ValueError):
        ext.preempt([1, 2])


def free_of(st, n):
    return [g["Percent"] for g in st.status()[n]["GPUs"]]


def test_preemption_route_over_http():
    async def main():
        store = FakeKubeStore()
        store.add_node(node("n0", 1))
        rt = await runtime(store)
        try:
            p = pu.make_pod("low", [("m", 60)])
            rt.state.reserve(p, "n0")
            rt.state.commit(pu.pod_uid(p))
            body = json.dumps({"Pod": pu.make_pod("high", [("m", 80)]),
                               "NodeNameToMetaVictims": {"n0": {"Pods": [{"UID": pu.pod_uid(p)}]}}}).encode()
            import aiohttp

            async with aiohttp.ClientSession() as s:
                async with s.post(f"http://127.0.0.1:{rt.bound_port}/scheduler/preemption", data=body) as r:
                    assert r.status == 200
                    out = await r.json()
                async with s.post(f"http://127.0.0.1:{rt.bound_port}/scheduler/preemption", data=b"[") as r:
                    assert r.status == 400
            assert list(out["NodeNameToMetaVictims"]) == ["n0"]
        finally:
            await rt.stop()

    asyncio.run(main())


def test_measured_hbm_activity_steers_memory_bound_shares_without_touching_load():
    """A device whose measured HBM activity (types.GPU_HBM_ACTIVITY_METRIC, the agent's
    nanogpu_device_mem_busy_percent) is at or above the threshold counts as holding a streaming
    tenant, declared or not: a memory-bound share goes to the quiet device, a compute-bound one
    still packs best-fit. The metric stays out of the reference's load sum (RemainLoad)."""
    from nanogpu.k8s.podutil import Req

    async def main():
        series = {T.GPU_HBM_ACTIVITY_METRIC: {("n0", 0): [0.85], ("n0", 1): [0.10]}}
        runner, port, _ = await fake_prometheus(series)
        st = ClusterState(policy="binpack", load_aware=True)
        n = node("n0", 2)
        st.register_node(n)
        nid = st.node_entry("n0").id
        assert st.ledger.reserve(nid, "cb", [(30, 0)], st.options)[0] == N.OK   # device 0 is fuller
        spec = PolicySpec(sync_period=(Period(T.GPU_HBM_ACTIVITY_METRIC, 15),))
        poller = LoadPoller(st, PromClient(f"http://127.0.0.1:{port}"), lambda: [n], spec=spec)
        mb = [Req(20, 0, N.FLAG_MEM_BOUND)]
        try:
            _, plan, _ = st.ledger.assume(nid, mb, st.options)
            assert plan == [[0]]                      # nothing measured yet: best fit
            await poller.sync_metric(T.GPU_HBM_ACTIVITY_METRIC)
            devs = st.ledger.snapshot(nid)["devices"]
            assert [d["mem_hot"] for d in devs] == [True, False]
            assert [d["remain_load"] for d in devs] == [T.LOAD_TOTAL, T.LOAD_TOTAL]   # not load
            _, plan, _ = st.ledger.assume(nid, mb, st.options)
            assert plan == [[1]]                      # the measured streamer is avoided
            _, plan, _ = st.ledger.assume(nid, [(20, 0)], st.options)
            assert plan == [[0]]                      # compute-bound shares still pack
            # a stale sample (period + 5 min) clears the mark
            poller.refresh_node("n0", 2, now=1e12)
            assert [d["mem_hot"] for d in st.ledger.snapshot(nid)["devices"]] == [False, False]
            _, plan, _ = st.ledger.assume(nid, mb, st.options)
            assert plan == [[0]]
        finally:
            await poller.prom.close()
            await runner.cleanup()

    asyncio.run(main())


def test_hbm_activity_presets_query_the_agent_and_the_amd_exporter():
    for preset, needle in (("nanogpu-agent", "nanogpu_device_mem_busy_percent"), ("amd", "gpu_umc_activity")):
        spec = parse_policy(f"spec:\n  metricsPreset: {preset}\n  syncPeriod:\n"
                            f"  - name: {T.GPU_HBM_ACTIVITY_METRIC}\n    period: 15s\n")
        q = spec.query_for(T.GPU_HBM_ACTIVITY_METRIC)
        assert needle in q.query and needle in q.batch and "{card}" not in q.batch


def test_cluster_scoped_metrics_one_query_per_metric_for_every_node():
    """`metricsScope: cluster`: one PromQL query per metric and period for the whole cluster
    (series grouped by their node label) instead of one per node: 1000 GPU nodes cost one query
    per 15 s, not 1000. A failed query backs off its one key; node-scoped is the default."""
    async def main():
        names = [f"n{i}" for i in range(5)]
        series = {"gpu_core_usage_avg": {(n, c): [0.05 if n != "n3" else 0.95] for n in names for c in range(2)}}
        runner, port, hits = await fake_prometheus(series)
        st = ClusterState(load_aware=True)
        nodes = [node(n, 2) for n in names]
        for n in nodes:
            st.register_node(n)
        spec = parse_policy("spec:\n  metricsScope: cluster\n  syncPeriod:\n"
                            "  - {name: gpu_core_usage_avg, period: 15s}\n")
        assert spec.metrics_scope == "cluster"
        poller = LoadPoller(st, PromClient(f"http://127.0.0.1:{port}"), lambda: nodes, spec=spec)
        try:
            assert poller.enqueue("gpu_core_usage_avg") == 1 and poller.queue.queued == {"*/gpu_core_usage_avg"}
            await poller.sync_metric("gpu_core_usage_avg")
            assert hits == ["gpu_core_usage_avg /100"]
            status = st.status()
            assert [g["RemainLoad"] for g in status["n3"]["GPUs"]] == [1, 1]    # usage ceil(9.5)/10 = 1.0
            assert all(g["RemainLoad"] == 2 for n in names if n != "n3" for g in status[n]["GPUs"])
            assert poller.polls == len(names)
        finally:
            await poller.prom.close()
            await runner.cleanup()
        with pytest.raises(ValueError):
            parse_policy("spec:\n  metricsScope: region\n")
        assert parse_policy("spec: {}\n").metrics_scope == "node"

    asyncio.run(main())


def test_owner_learning_through_the_poller_and_the_python_verbs():
    """Prometheus HBM activity -> poller marks the device hot -> the period's learner makes the
    lone tenant's owner streaming -> the Python verbs place the owner's next pod as memory-bound
    (off the hot device); a pod of another owner still packs best-fit."""
    from nanogpu.k8s.podutil import make_pod

    async def main():
        st = ClusterState(policy="binpack", load_aware=True)
        n = node("n0", 2)
        st.register_node(n)
        nid = st.node_entry("n0").id

        def owned(name, owner):
            p = make_pod(name, [("main", 20, 0)])
            p["metadata"]["uid"] = f"uid-{name}"
            p["metadata"]["ownerReferences"] = [{"kind": "Job", "name": owner, "uid": f"{owner}-uid"}]
            return p

        a = owned("a", "job1")
        plan, fresh = st.reserve(a, "n0")
        assert fresh and plan == [[0]]
        st.commit("uid-a")
        series = {T.GPU_HBM_ACTIVITY_METRIC: {("n0", 0): [0.9], ("n0", 1): [0.0]}}
        runner, port, _ = await fake_prometheus(series)
        spec = PolicySpec(sync_period=(Period(T.GPU_HBM_ACTIVITY_METRIC, 15),))
        poller = LoadPoller(st, PromClient(f"http://127.0.0.1:{port}"), lambda: [n], spec=spec)
        try:
            await poller.sync_metric(T.GPU_HBM_ACTIVITY_METRIC)
            # "a" was bound just now: the hot mark may have been measured on a tenant before it
            assert poller.learn_owners() == (0, 0)
            later = time.monotonic() + 16          # one period on: the mark's window covers "a"
            assert poller.learn_owners(now=later) == (1, 0) and poller.owners_learned == 1
            assert st.pod_demand(owned("b", "job1"))[0].flags == N.FLAG_MEM_BOUND
            assert st.reserve(owned("b", "job1"), "n0")[0] == [[1]]      # off the hot device
            assert st.reserve(owned("c", "job2"), "n0")[0] == [[0]]      # other owner: best fit
        finally:
            await poller.prom.close()
            await runner.cleanup()

    asyncio.run(main())


def test_poller_counts_queries_and_learned_owners_in_extender_metrics():
    from nanogpu.obs import Metrics

    async def main():
        series = {T.GPU_HBM_ACTIVITY_METRIC: {("n0", 0): [0.9]}, "fail_nodes": ("n1",)}
        runner, port, _ = await fake_prometheus(series)
        st = ClusterState(policy="binpack")
        nodes = [node("n0", 2), node("n1", 2)]
        for n in nodes:
            st.register_node(n)
        m = Metrics()
        spec = PolicySpec(sync_period=(Period(T.GPU_HBM_ACTIVITY_METRIC, 15),))
        poller = LoadPoller(st, PromClient(f"http://127.0.0.1:{port}"), lambda: nodes, spec=spec, metrics=m)
        try:
            await poller.sync_metric(T.GPU_HBM_ACTIVITY_METRIC)
            poller.learn_owners()
            text = m.render().decode()
            assert 'nanogpu_metric_queries_total{result="ok"} 1.0' in text
            assert 'nanogpu_metric_queries_total{result="error"} 1.0' in text
            assert 'nanogpu_stream_owners_total{event="learned"} 0.0' in text
        finally:
            await poller.prom.close()
            await runner.cleanup()

    asyncio.run(main())


def test_hbm_ticker_learns_owners_each_period():
    from nanogpu.k8s.podutil import make_pod

    async def main():
        st = ClusterState(policy="binpack")
        n = node("n0", 2)
        st.register_node(n)
        p = make_pod("a", [("main", 20, 0)])
        p["metadata"]["uid"] = "uid-a"
        p["metadata"]["ownerReferences"] = [{"kind": "Job", "name": "j", "uid": "job-uid", "controller": True}]
        st.reserve(p, "n0")
        st.commit("uid-a")
        runner, port, _ = await fake_prometheus({T.GPU_HBM_ACTIVITY_METRIC: {("n0", 0): [0.8]}})
        spec = PolicySpec(sync_period=(Period(T.GPU_HBM_ACTIVITY_METRIC, 0.05),))
        poller = LoadPoller(st, PromClient(f"http://127.0.0.1:{port}"), lambda: [n], spec=spec)
        try:
            poller.restart()
            for _ in range(100):
                if poller.owners_learned:
                    break
                await asyncio.sleep(0.02)
            assert poller.owners_learned == 1 and st.ledger.is_stream_owner("job-uid")
        finally:
            await poller.stop()
            await poller.prom.close()
            await runner.cleanup()

    asyncio.run(main())


def test_demand_memo_without_the_owner_lookup_does_not_hide_a_learned_owner():
    """A caller that asks for a pod's demand without the streaming-owner lookup (the pod
    controller's GPU check) must not fix the unflagged demand for the verbs that use it."""
    from nanogpu.k8s.podutil import make_pod

    st = ClusterState(policy="binpack")
    st.ledger.set_stream_owner("rs-9", True)
    p = make_pod("x", [("main", 20, 0)])
    p["metadata"]["uid"] = "uid-memo-x"
    p["metadata"]["ownerReferences"] = [{"kind": "ReplicaSet", "name": "rs", "uid": "rs-9", "controller": True}]
    assert pu.pod_demand(p) == [(20, 0)] and not hasattr(pu.pod_demand(p)[0], "flags")
    assert st.pod_demand(p)[0].flags == N.FLAG_MEM_BOUND


def test_hbm_hot_threshold_is_a_policy_knob():
    spec = parse_policy("spec:\n  hbmHotThreshold: 0.66\n")
    assert spec.hbm_hot_threshold == 0.66
    st = ClusterState()
    poller = LoadPoller(st, None, lambda: [], spec=spec)
    assert poller.hbm_threshold == 0.66
    with pytest.raises(ValueError):
        parse_policy("spec:\n  hbmHotThreshold: 1.5\n")
    assert LoadPoller(st, None, lambda: []).hbm_threshold == T.HBM_HOT_THRESHOLD


def test_deleted_node_slot_goes_when_its_last_share_does():
    """A deleted Node: nominations on it are dropped at once; a committed pod keeps the slot
    until it is released, then the sweeper's retry removes it; a node registered again under
    the same name meanwhile is left alone."""
    from nanogpu import _native as NN
    from nanogpu.state.cluster import ClusterState
    from nanogpu.topology.model import synthetic_mi355x

    st = ClusterState()
    for n in ("a", "b"):
        st.register_node(pu.make_node(n, 8, synthetic_mi355x(8).to_json()))
    ida, idb = st.node_ids(["a", "b"])
    assert st.ledger.nominate(ida, "nom", [(10, 0)], st.options) == NN.OK
    assert st.forget_node("a") and st.ledger.find_node("a") < 0          # nomination dropped
    assert st.ledger.lookup("nom") is None
    assert st.ledger.reserve(idb, "held", [(10, 0)], st.options)[0] == NN.OK
    st.ledger.commit("held")
    assert not st.forget_node("b") and st.ledger.find_node("b") == idb    # still holds a share
    assert st.retry_removals() == []
    st.ledger.release("held")
    assert st.retry_removals() == ["b"] and st.ledger.find_node("b") < 0
    # re-registered before the retry: not removed
    st.register_node(pu.make_node("c", 8, synthetic_mi355x(8).to_json()))
    idc = st.node_ids(["c"])[0]
    assert st.ledger.reserve(idc, "held2", [(10, 0)], st.options)[0] == NN.OK
    assert not st.forget_node("c")
    st.register_node(pu.make_node("c", 8, synthetic_mi355x(8).to_json()))
    st.ledger.release("held2")
    assert st.retry_removals() == [] and st.ledger.find_node("c") >= 0


def test_hbm_activity_is_read_through_the_devices_own_calibration():
    """the same quarter-GPU streamer reads 30.1 % on the calibration box and
    20.7 % on another (28.7 % for the whole chip there). The agent publishes each GPU's own scale
    (GpuSpec.hbm_busy_cal, probe.calibrate.hbm_busy_calibration); the poller maps readings through
    it onto the reference curve, so the same tenant is classified the same on both boxes."""
    from nanogpu.telemetry.store import normalize_hbm_activity as norm

    cal = [[25, 20.7], [100, 28.7]]
    assert norm(0.207, cal) == pytest.approx(0.301, abs=1e-3)      # the box's 25 % streamer -> reference's
    assert norm(0.287, cal) == pytest.approx(0.544, abs=1e-3)      # its whole-chip streamer
    assert norm(0.0, cal) == 0.0 and norm(0.9, cal) <= 1.0
    assert norm(0.207, []) == 0.207 and norm(0.207, None) == 0.207   # no calibration: as read
    xs = [i / 100 for i in range(101)]
    assert all(norm(a, cal) <= norm(b, cal) for a, b in zip(xs, xs[1:]))   # monotone
    # the calibration box's own scale is the identity at its points
    assert norm(0.301, [[25, 30.1], [100, 54.4]]) == pytest.approx(0.301, abs=1e-3)

    async def main():
        # a 17 % reading: under the hot threshold as read, a quarter-GPU streamer's on this box
        series = {T.GPU_HBM_ACTIVITY_METRIC: {("n0", 0): [0.17], ("n0", 1): [0.17], ("n1", 0): [0.17]}}
        runner, port, _ = await fake_prometheus(series)
        st = ClusterState(policy="binpack", load_aware=True)
        t = synthetic_mi355x(2)
        t.gpus[0].hbm_busy_cal = cal          # GPU 0 calibrated, GPU 1 not
        t2 = synthetic_mi355x(2)
        n0 = pu.make_node("n0", 2, t.to_json(), {"amd.com/gpu.present": "true"})
        n1 = pu.make_node("n1", 2, t2.to_json(), {"amd.com/gpu.present": "true"})
        st.register_node(n0)
        st.register_node(n1)
        assert st.node_entry("n0").topology.gpus[0].hbm_busy_cal == cal   # through the annotation
        spec = PolicySpec(sync_period=(Period(T.GPU_HBM_ACTIVITY_METRIC, 15),))
        poller = LoadPoller(st, PromClient(f"http://127.0.0.1:{port}"), lambda: [n0, n1], spec=spec)
        try:
            await poller.sync_metric(T.GPU_HBM_ACTIVITY_METRIC)
            d0 = st.ledger.snapshot(st.node_entry("n0").id)["devices"]
            d1 = st.ledger.snapshot(st.node_entry("n1").id)["devices"]
            assert [d["mem_hot"] for d in d0] == [True, False]
            assert d0[0]["mem_busy"] == 25 and d0[1]["mem_busy"] == 17
            assert not d1[0]["mem_hot"]
        finally:
            await poller.prom.close()
            await runner.cleanup()

    asyncio.run(main())


def test_agent_calibration_lands_on_each_whole_gpu(monkeypatch):
    """agent.node.calibrate measures each SPX GPU's scale on its own HIP ordinal and mem_busy
    file and publishes it in the topology annotation (probe calls stubbed: no GPU here)."""
    from nanogpu.agent import node as A
    from nanogpu.probe import calibrate as C
    from nanogpu.topology.model import NodeTopology

    class P:
        @staticmethod
        def device_count():
            return 2

    calls = []
    monkeypatch.setattr(C, "local_gpu_facts", lambda device=0, use_probe=True: {"props": {"gcn_arch": "gfx950"}})
    monkeypatch.setattr(C, "hbm_bandwidth", lambda *a, **k: 5994.0)
    monkeypatch.setattr(C, "mem_busy_files", lambda h: {0: "busy0", 1: "busy1"})
    monkeypatch.setattr(C, "hbm_busy_calibration",
                        lambda P_, k, f, seconds=3.0: calls.append((k, f)) or [[25, 20.0 + k], [100, 28.0 + k]])
    import nanogpu.native as NV
    monkeypatch.setattr(NV, "probe", lambda *a, **k: P)
    host = {"gpus": [{"parent": 0, "compute_partition": "SPX"}, {"parent": 1, "compute_partition": "SPX"}]}
    topo = synthetic_mi355x(2)
    out = A.calibrate(topo, host=host, busy_s=0.0)
    assert calls == [(0, "busy0"), (1, "busy1")]
    assert out["hbm_busy_cal"] == {0: [[25, 20.0], [100, 28.0]], 1: [[25, 21.0], [100, 29.0]]}
    back = NodeTopology.from_json(topo.to_json())
    assert back.gpus[1].hbm_busy_cal == [[25, 21.0], [100, 29.0]]


def test_a_ledger_larger_than_the_tmpfs_is_refused_at_start(tmp_path, monkeypatch):
    """a region past the /dev/shm emptyDir's size would SIGBUS on first touch; the
    extender refuses to start and names the sizes instead."""
    import os as _os

    from nanogpu import app as A

    class St:
        f_bavail, f_frsize = 16, 1 << 20      # 16 MiB free
    monkeypatch.setattr(_os, "statvfs", lambda d: St)
    with pytest.raises(SystemExit, match="needs .* MiB"):
        A.check_region_space(str(tmp_path / "ledger"), 4096, 1 << 20)
    A.check_region_space(str(tmp_path / "ledger"), 8, 64)   # a small one fits
