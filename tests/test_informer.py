"""Informer = client-go reflector: LIST once, WATCH from the last resourceVersion, re-LIST only
on 410 Gone / an ERROR event / a transport failure (client-go v0.18, /root/reference/go.mod:16;
informers started at /root/reference/pkg/controller/controller.go:136).

The fake API server injects the faults a real one produces: watch streams that end at
timeoutSeconds, etcd compaction (a resumed watch answered 410), and in-stream ERROR events.
"""
import asyncio

from nanogpu.k8s import podutil as pu
from nanogpu.k8s.fake_apiserver import Faults, FakeKubeStore, InProcKube, serve
from nanogpu.k8s.client import KubeClient, KubeConfig
from nanogpu.k8s.informer import Informer

from test_control_plane import annotated, node, runtime, wait_for


def test_clean_watch_end_resumes_without_a_list():
    async def main():
        store = FakeKubeStore(faults=Faults(watch_timeout_s=0.02))
        inf = Informer(InProcKube(store), "pods")
        seen = []
        inf.add_handler(lambda et, o, old: seen.append((et, pu.meta(o)["name"])))
        inf.start()
        try:
            await asyncio.wait_for(inf.synced.wait(), 2)
            for i in range(5):
                store.create_pod(pu.make_pod(f"p{i}", [("c", 10)]))
                await asyncio.sleep(0.03)            # across several watch timeouts
            assert await wait_for(lambda: len(seen) == 5)
            assert inf.rewatches >= 3
            assert inf.relists == 1 and store.counts["list_pods"] == 1
            assert seen == [("ADDED", f"p{i}") for i in range(5)]   # nothing lost or repeated
        finally:
            await inf.stop()

    asyncio.run(main())


def test_pod_deleted_while_the_watch_was_down_is_released_after_the_410_relist():
    async def main():
        store = FakeKubeStore()
        store.add_node(node("n0"))
        rt = await runtime(store)
        try:
            p = store.create_pod(annotated("gone", "n0", [[0]], pct=30))
            uid = pu.pod_uid(p)
            led = rt.state.ledger
            assert await wait_for(lambda: led.lookup(uid) is not None)
            inf = rt.pod_informer
            lists = store.counts["list_pods"]
            # no await between these: the watch ends, the pod goes, the watch cache is compacted
            # before the informer can resume, so its resume is answered 410 Gone
            store.drop_watches()
            store.delete_pod("default", "gone")
            store.compact()
            assert await wait_for(lambda: led.lookup(uid) is None)
            assert inf.expired >= 1 and store.counts["list_pods"] == lists + 1
            assert rt.state.status()["n0"]["GPUs"][0]["Percent"] == 100
        finally:
            await rt.stop()

    asyncio.run(main())


def test_in_stream_error_event_forces_a_relist_and_other_ends_do_not():
    async def main():
        store = FakeKubeStore()
        inf = Informer(InProcKube(store), "nodes")
        inf.start()
        try:
            await asyncio.wait_for(inf.synced.wait(), 2)
            store.add_node(node("n0"))
            assert await wait_for(lambda: inf.get("n0") is not None)
            store.drop_watches()                    # clean end
            assert await wait_for(lambda: inf.rewatches >= 1)
            store.add_node(node("n1"))
            assert await wait_for(lambda: inf.get("n1") is not None)
            assert inf.relists == 1
            store.inject_watch_error("nodes", 410)  # in-stream expiry
            assert await wait_for(lambda: inf.relists == 2)
            assert inf.expired == 1
            store.add_node(node("n2"))
            assert await wait_for(lambda: inf.get("n2") is not None)
        finally:
            await inf.stop()

    asyncio.run(main())


def test_rest_watch_over_http_resumes_and_relists_on_410():
    """Same semantics through the REST client against the HTTP fake API server."""
    async def main():
        store = FakeKubeStore(faults=Faults(watch_timeout_s=0.05))
        runner, port = await serve(store)
        api = KubeClient(KubeConfig(server=f"http://127.0.0.1:{port}"))
        inf = Informer(api, "pods")
        inf.start()
        try:
            await asyncio.wait_for(inf.synced.wait(), 5)
            store.create_pod(pu.make_pod("a", [("c", 10)]))
            assert await wait_for(lambda: inf.get("default/a") is not None)
            await asyncio.sleep(0.2)
            assert inf.rewatches >= 2 and inf.relists == 1
            store.drop_watches()
            store.delete_pod("default", "a")
            store.compact()
            assert await wait_for(lambda: inf.get("default/a") is None)
            assert inf.relists == 2 and inf.expired >= 1
        finally:
            await inf.stop()
            await api.close()
            await runner.cleanup()

    asyncio.run(main())
