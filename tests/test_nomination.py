"""Priorities-time nominations under kube-scheduler's score combining.

kube-scheduler adds the extender's priority x weight x 10 to its own plugin scores
(nanogpu/sim/kubescore.py; /root/reference/README.md:43-58 configures the extender with
weight 1), so the extender's top node is not always the node it binds. A nomination the bind
does not adopt holds capacity until the bind lands elsewhere or its TTL passes; the ledger
counts adopted vs moved nominations and raises the score lead it wants before nominating.
"""
import asyncio
import json

from nanogpu.k8s import podutil as pu
from nanogpu.sim.driver import FastExtenderClient, SchedulerDriver, node_capacities
from nanogpu.sim.kubescore import KubeScoring
from nanogpu.k8s.fake_apiserver import InProcKube

from test_containers import _runtime
from test_control_plane import wait_for
from test_frontend import _dumps, _http


def test_kube_combining_overrides_a_small_extender_lead():
    ks = KubeScoring()
    pod = ks.pod_requests([(50, 0)])
    # n0: the extender's pick by one point, but its CPUs / memory are mostly requested already
    busy = (200_000, 2 << 40)
    assert ks.total(61, busy, pod) < ks.total(60, (0, 0), pod)
    # a ten-point lead is 100 combined points: more than any plugin gap here
    assert ks.total(70, busy, pod) < ks.total(60, (0, 0), pod) + 100
    assert ks.select([5, 9, 9, 1]) in (1, 2)


def test_wrong_nominations_are_counted_and_raise_the_margin():
    """--priority-lead 0 (raw scores, as the reference): kube-scheduler's plugins can move the
    pod off a close nomination; the ledger counts it and nominates less eagerly."""
    async def main():
        store, rt = await _runtime(2, priority_lead=0)
        led = rt.state.ledger
        client = FastExtenderClient("127.0.0.1", rt.bound_port, pool=8)
        loop = asyncio.get_running_loop()
        try:
            nodes = [store.nodes[n] for n in ("n0", "n1")]
            # n0 GPU 0 has a 40 % hole, n1 GPU 0 a 45 % one: a 30 % share scores 90 on n0 and 85
            # on n1 (the leftover), a 5-point lead the extender nominates
            for name, pct, node in (("b0", 60, "n0"), ("b1", 55, "n1")):
                base = store.create_pod(pu.make_pod(name, [("c", pct)]))
                m = pu.meta(base)
                await loop.run_in_executor(None, _http, rt.bound_port, [
                    ("POST", "/scheduler/filter", _dumps({"Pod": base, "NodeNames": [node]})),
                    ("POST", "/scheduler/bind", _dumps({"PodName": name, "PodNamespace": "default",
                                                        "PodUID": m["uid"], "Node": node}))])
            pod = pu.make_pod("p", [("c", 30)])
            scores = await client.prioritize({"Pod": pod, "Nodes": None, "NodeNames": ["n0", "n1"]})
            assert [h["Score"] for h in scores] == [90, 85]
            led.drop_nomination(pu.pod_uid(pod))
            # ...but n0's CPUs and memory are mostly requested already, so kube-scheduler's own
            # plugins outweigh 5 x 10 points and it binds the pod on n1
            drv = SchedulerDriver(client, InProcKube(store), ["n0", "n1"], node_capacities(nodes),
                                  kube=KubeScoring(), resource_fit=False)
            drv.used["n0"] = (250_000, 3 << 40)
            stats = await drv.run([pod])
            assert stats.scheduled == 1
            assert pu.node_name_of(store.get_pod("default", "p")) == "n1"
            c = led.nomination_counts()
            assert c["moved"] >= 1, c
            assert led.nomination_margin == 2
            # the next near-tie (a 5-point lead is still >= 2) nominates again; a 1-point one
            # would not
            q = pu.make_pod("q", [("c", 30)])
            await client.prioritize({"Pod": q, "Nodes": None, "NodeNames": ["n0", "n1"]})
            assert led.lookup(pu.pod_uid(q))["state"] == "nominated"
        finally:
            await client.close()
            await rt.stop()

    asyncio.run(main())


def test_the_priorities_lead_keeps_kube_scheduler_on_the_nomination():
    """The default lead (nanogpu.types.PRIORITY_LEAD): the same near-tie is answered with the
    nominated node 100 points ahead, which kube-scheduler's own plugins (busy CPUs / memory on
    n0) cannot overturn, so the bind adopts the nomination and the margin stays 0."""
    from nanogpu import types as T

    async def main():
        store, rt = await _runtime(2)
        led = rt.state.ledger
        client = FastExtenderClient("127.0.0.1", rt.bound_port, pool=8)
        loop = asyncio.get_running_loop()
        try:
            nodes = [store.nodes[n] for n in ("n0", "n1")]
            for name, pct, node in (("b0", 60, "n0"), ("b1", 55, "n1")):
                base = store.create_pod(pu.make_pod(name, [("c", pct)]))
                m = pu.meta(base)
                await loop.run_in_executor(None, _http, rt.bound_port, [
                    ("POST", "/scheduler/filter", _dumps({"Pod": base, "NodeNames": [node]})),
                    ("POST", "/scheduler/bind", _dumps({"PodName": name, "PodNamespace": "default",
                                                        "PodUID": m["uid"], "Node": node}))])
            pod = pu.make_pod("p", [("c", 30)])
            scores = await client.prioritize({"Pod": pod, "Nodes": None, "NodeNames": ["n0", "n1"]})
            assert [h["Score"] for h in scores] == [85 + T.PRIORITY_LEAD, 85]
            led.drop_nomination(pu.pod_uid(pod))
            drv = SchedulerDriver(client, InProcKube(store), ["n0", "n1"], node_capacities(nodes),
                                  kube=KubeScoring(), resource_fit=False)
            drv.used["n0"] = (250_000, 3 << 40)
            stats = await drv.run([pod])
            assert stats.scheduled == 1
            assert pu.node_name_of(store.get_pod("default", "p")) == "n0"
            c = led.nomination_counts()
            assert c["moved"] == 0 and c["adopted"] >= 1, c
            assert led.nomination_margin == 0
        finally:
            await client.close()
            await rt.stop()

    asyncio.run(main())


def test_a_wrong_nomination_never_blocks_a_pod_after_its_ttl():
    async def main():
        # (a TTL of 1 s: a slow shared host must not expire it between two requests)
        store, rt = await _runtime(2, nomination_ttl_s=1.0)
        loop = asyncio.get_running_loop()
        try:
            # n0 has one 40 % hole left on its last GPU; n1 is empty
            base = store.create_pod(pu.make_pod("base", [("c", 100)] * 7 + [("d", 60)]))
            m = pu.meta(base)
            await loop.run_in_executor(None, _http, rt.bound_port, [
                ("POST", "/scheduler/filter", _dumps({"Pod": base, "NodeNames": ["n0"]})),
                ("POST", "/scheduler/bind", _dumps({"PodName": "base", "PodNamespace": "default",
                                                    "PodUID": m["uid"], "Node": "n0"}))])
            a = store.create_pod(pu.make_pod("a", [("c", 40)]))
            b = store.create_pod(pu.make_pod("b", [("c", 40)]))
            both = ["n0", "n1"]
            # a is nominated on n0 (exact fit) and then never bound: kube-scheduler went elsewhere
            # and the pod was deleted before its bind
            await loop.run_in_executor(None, _http, rt.bound_port, [
                ("POST", "/scheduler/filter", _dumps({"Pod": a, "NodeNames": both})),
                ("POST", "/scheduler/priorities", _dumps({"Pod": a, "NodeNames": both}))])
            assert rt.state.ledger.lookup(pu.pod_uid(a))["state"] == "nominated"
            res = await loop.run_in_executor(None, _http, rt.bound_port, [
                ("POST", "/scheduler/filter", _dumps({"Pod": b, "NodeNames": both}))])
            assert json.loads(res[0][1])["NodeNames"] == ["n1"]           # held for a while...
            assert await wait_for(lambda: rt.state.ledger.lookup(pu.pod_uid(a)) is None, timeout=6)
            res = await loop.run_in_executor(None, _http, rt.bound_port, [
                ("POST", "/scheduler/filter", _dumps({"Pod": b, "NodeNames": both}))])
            assert json.loads(res[0][1])["NodeNames"] == both             # ...never longer than the TTL
        finally:
            await rt.stop()

    asyncio.run(main())
