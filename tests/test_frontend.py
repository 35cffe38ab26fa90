"""Native C++ front door (native/src/frontend.cpp) against the Python verbs.

The Python Extender is the specification: for every request the native fast path
answers, the response bytes must equal `json.dumps(<python verb>(body))`; everything the
fast path declines (bind, ops routes, Nodes-only filters, unknown nodes, malformed JSON)
must come back from Python through the eventfd bridge, in order, on the same connection.
"""
import asyncio
import json
import random
import socket

import pytest
from hypothesis import given, settings
from hypothesis import strategies as st

from nanogpu import _native as N
from nanogpu import types as T
from nanogpu.app import Config, Runtime
from nanogpu.k8s import podutil as pu
from nanogpu.k8s.fake_apiserver import FakeKubeStore, InProcKube
from nanogpu.k8s.quantity import QuantityError, quantity_to_mib, quantity_value
from nanogpu.topology.model import synthetic_mi355x


def _dumps(o) -> bytes:
    return json.dumps(o, separators=(",", ":")).encode()


async def _runtime(n_nodes=4, partition="SPX", **kw):
    store = FakeKubeStore()
    for i in range(n_nodes):
        devs = 8 * {"SPX": 1, "CPX": 8}[partition]
        store.add_node(pu.make_node(f"n{i}", devs, synthetic_mi355x(8, partition).to_json()))
    rt = Runtime(Config(port=0, host="127.0.0.1", policy_config_path="/nonexistent", **kw), api=InProcKube(store))
    await rt.start()
    assert rt.native is not None
    return store, rt


def _http(port: int, reqs: list[tuple[str, str, bytes]], chunked: bool = False) -> list[tuple[int, bytes]]:
    """Sends all requests on ONE keep-alive connection (pipelined), returns (status, body)."""
    s = socket.create_connection(("127.0.0.1", port))
    out = b""
    for method, path, body in reqs:
        if chunked and body:
            mid = len(body) // 2
            enc = b"".join(f"{len(p):x}\r\n".encode() + p + b"\r\n" for p in (body[:mid], body[mid:]) if p) + b"0\r\n\r\n"
            out += f"{method} {path} HTTP/1.1\r\nHost: x\r\nTransfer-Encoding: chunked\r\n\r\n".encode() + enc
        else:
            out += f"{method} {path} HTTP/1.1\r\nHost: x\r\nContent-Length: {len(body)}\r\n\r\n".encode() + body
    s.sendall(out)
    res, buf = [], b""
    s.settimeout(10)
    while len(res) < len(reqs):
        while b"\r\n\r\n" not in buf:
            buf += s.recv(65536)
        head, _, rest = buf.partition(b"\r\n\r\n")
        status = int(head.split(b" ")[1])
        clen = int([h.split(b":")[1] for h in head.split(b"\r\n") if h.lower().startswith(b"content-length")][0])
        while len(rest) < clen:
            rest += s.recv(65536)
        res.append((status, rest[:clen]))
        buf = rest[clen:]
    s.close()
    return res


def _pods(rng, n):
    out = []
    for i in range(n):
        cs = [(f"c{k}", rng.choice([0, 5, 10, 25, 50, 100, 200]), rng.choice([0, 0, 8192, 65536]))
              for k in range(rng.choice([1, 1, 2, 3]))]
        pod = pu.make_pod(f"p{i}", cs)
        mb = rng.choice([None, None, "true", "c0", "c1, c2"])   # memory-bound containers
        if mb:
            pod["metadata"]["annotations"][T.ANNOTATION_MEMORY_BOUND] = mb
        out.append(pod)
    return out


@pytest.mark.parametrize("policy,partition,normalize", [("binpack", "SPX", False), ("spread", "CPX", True),
                                                        ("random", "SPX", False), ("firstfit", "SPX", True)])
def test_native_filter_and_priorities_are_byte_identical(policy, partition, normalize):
    async def main():
        store, rt = await _runtime(4, partition, priority=policy, score_normalize=normalize)
        ext = rt.extender
        rng = random.Random(7)
        names = [f"n{i}" for i in range(4)]
        loop = asyncio.get_running_loop()
        try:
            for k, pod in enumerate(_pods(rng, 40)):
                pod = store.create_pod(pod)
                body = {"Pod": pod, "Nodes": None, "NodeNames": rng.sample(names, rng.randint(1, 4))}
                raw = _dumps(body)
                got = await loop.run_in_executor(None, _http, rt.bound_port,
                                                 [("POST", "/scheduler/filter", raw),
                                                  ("POST", "/scheduler/priorities", raw)])
                assert got[0] == (200, _dumps(ext.filter(json.loads(raw)))), got[0]
                assert got[1] == (200, _dumps(ext.prioritize(json.loads(raw)))), got[1]
                fit = json.loads(got[0][1])["NodeNames"]
                if fit and k % 2 == 0:   # change state between requests
                    m = pu.meta(pod)
                    r = await ext.bind({"PodName": m["name"], "PodNamespace": m["namespace"],
                                        "PodUID": m["uid"], "Node": fit[0]})
                    assert r["Error"] == ""
            st_ = rt.native.fe.stats()
            assert st_["filter"]["count"] == 40 and st_["priorities"]["count"] == 40
        finally:
            await rt.stop()

    asyncio.run(main())


def test_deferred_routes_keep_order_on_one_connection():
    async def main():
        store, rt = await _runtime(2)
        loop = asyncio.get_running_loop()
        try:
            pod = store.create_pod(pu.make_pod("a", [("main", 20)]))
            m = pu.meta(pod)
            f = _dumps({"Pod": pod, "NodeNames": ["n0", "n1"]})
            node_objs = _dumps({"Pod": pod, "Nodes": {"items": [store.get_node("n0")]}, "NodeNames": None})
            bind = _dumps({"PodName": "a", "PodNamespace": "default", "PodUID": m["uid"], "Node": "n0"})
            reqs = [("POST", "/scheduler/filter", f),            # native
                    ("POST", "/scheduler/filter", node_objs),    # Python (Nodes-only)
                    ("POST", "/scheduler/priorities", f),        # native, queued behind Python
                    ("POST", "/scheduler/bind", bind),           # Python, pod from the native cache
                    ("GET", "/version", b""),
                    ("POST", "/scheduler/filter", b"{nope"),     # Python error format
                    ("POST", "/scheduler/priorities", b"{nope"), # 400
                    ("GET", "/nothing", b""),
                    ("GET", "/scheduler/filter", b""),           # 405
                    ("GET", "/metrics", b"")]
            res = await loop.run_in_executor(None, _http, rt.bound_port, reqs)
            assert res[0][0] == 200 and json.loads(res[0][1])["NodeNames"] == ["n0", "n1"]
            assert [pu.meta(n)["name"] for n in json.loads(res[1][1])["Nodes"]["items"]] == ["n0"]
            assert [h["Host"] for h in json.loads(res[2][1])] == ["n0", "n1"]
            assert res[3] == (200, b'{"Error":""}')
            assert res[4] == (200, T.VERSION.encode())
            assert res[5][0] == 200 and json.loads(res[5][1])["Error"]
            assert res[6][0] == 400
            assert res[7][0] == 404 and res[8][0] == 405
            assert b'nanogpu_native_verb_total{verb="filter"}' in res[9][1]
            # the bind used the pod cached by the native filter: no GET
            assert store.counts.get("get_pod", 0) == 0
            assert store.get_pod("default", "a")["spec"]["nodeName"] == "n0"
        finally:
            await rt.stop()

    asyncio.run(main())


def test_chunked_body_and_unknown_node_registration():
    async def main():
        store, rt = await _runtime(1)
        loop = asyncio.get_running_loop()
        try:
            pod = store.create_pod(pu.make_pod("a", [("main", 30)]))
            raw = _dumps({"Pod": pod, "NodeNames": ["n0"]})
            res = await loop.run_in_executor(None, lambda: _http(rt.bound_port, [("POST", "/scheduler/filter", raw)],
                                                                  chunked=True))
            assert json.loads(res[0][1])["NodeNames"] == ["n0"]
            # a node the ledger has not seen yet: Python registers it from the informer
            store.add_node(pu.make_node("late", 8, synthetic_mi355x(8).to_json()))
            await asyncio.sleep(0.05)
            raw = _dumps({"Pod": pod, "NodeNames": ["late", "ghost"]})
            res = await loop.run_in_executor(None, _http, rt.bound_port, [("POST", "/scheduler/filter", raw)])
            body = json.loads(res[0][1])
            assert body["NodeNames"] == ["late"] and "ghost" in body["FailedNodes"]
        finally:
            await rt.stop()

    asyncio.run(main())


def test_concurrent_clients_hammer_native_path():
    async def main():
        store, rt = await _runtime(8)
        loop = asyncio.get_running_loop()
        pods = [store.create_pod(pu.make_pod(f"p{i}", [("c", 10)])) for i in range(16)]
        names = [f"n{i}" for i in range(8)]

        def client(k):
            reqs = [("POST", "/scheduler/filter", _dumps({"Pod": pods[(k + j) % 16], "NodeNames": names}))
                    for j in range(50)]
            return _http(rt.bound_port, reqs)

        try:
            outs = await asyncio.gather(*[loop.run_in_executor(None, client, k) for k in range(8)])
            for out in outs:
                assert all(s == 200 and json.loads(b)["NodeNames"] == names for s, b in out)
        finally:
            await rt.stop()

    asyncio.run(main())


def test_policy_reload_reaches_native_path():
    async def main():
        store, rt = await _runtime(2)
        loop = asyncio.get_running_loop()
        try:
            pod = store.create_pod(pu.make_pod("a", [("main", 20)]))
            raw = _dumps({"Pod": pod, "NodeNames": ["n0", "n1"]})
            a = await loop.run_in_executor(None, _http, rt.bound_port, [("POST", "/scheduler/priorities", raw)])
            rt.state.set_policy("spread", compat=True)
            rt.state.score_normalize = True
            b = await loop.run_in_executor(None, _http, rt.bound_port, [("POST", "/scheduler/priorities", raw)])
            assert a[0][1] != b[0][1]
            assert b[0][1] == _dumps(rt.extender.prioritize(json.loads(raw)))
        finally:
            await rt.stop()

    asyncio.run(main())


_q = st.one_of(
    st.integers(0, 10 ** 6).map(str),
    st.builds(lambda a, b, s: f"{a}.{b}{s}", st.integers(0, 999), st.integers(0, 999),
              st.sampled_from(["", "m", "k", "M", "G", "Ki", "Mi", "Gi", "u", "n", "E"])),
    st.builds(lambda a, e: f"{a}e{e}", st.integers(0, 99), st.integers(-5, 8)),
    st.builds(lambda a, s: f"{a}{s}", st.integers(0, 10 ** 5), st.sampled_from(["Ki", "Mi", "Gi", "Ti", "m", "k"])),
)


@settings(max_examples=400, deadline=None)
@given(_q, st.booleans())
def test_native_quantity_matches_python(q, mib):
    got = N.quantity_value(q, mib)
    try:
        want = max(0, quantity_to_mib(q) if mib else quantity_value(q))
    except QuantityError:
        want = None
    if got is None:
        assert want is None or want > 2 ** 62
    else:
        assert got == want, (q, mib)


def test_native_prepared_bind_and_its_error_text():
    # (no nominations: with them the late pod's one-node filter would hold its GPU for its bind)
    async def main():
        store, rt = await _runtime(1, nominate=False)
        loop = asyncio.get_running_loop()
        try:
            big = store.create_pod(pu.make_pod("big", [("c", 100)] * 8))     # fills the node
            other = store.create_pod(pu.make_pod("late", [("c", 100)]))
            reqs = []
            for p in (other, big):
                reqs.append(("POST", "/scheduler/filter", _dumps({"Pod": p, "NodeNames": ["n0"]})))
            for p in (big, other):
                m = pu.meta(p)
                reqs.append(("POST", "/scheduler/bind", _dumps({"PodName": m["name"], "PodNamespace": "default",
                                                                 "PodUID": m["uid"], "Node": "n0"})))
            res = await loop.run_in_executor(None, _http, rt.bound_port, reqs)
            assert res[2] == (200, b'{"Error":""}')
            assert res[3][0] == 500
            assert json.loads(res[3][1])["Error"] == "assume (100) on n0 failed: insufficient gpu resource"
            s = rt.native.fe.stats()
            assert s["bind_reserve"]["count"] == 2 and store.counts.get("get_pod", 0) == 0
            assert [g["Percent"] for g in rt.state.status()["n0"]["GPUs"]] == [0] * 8
        finally:
            await rt.stop()

    asyncio.run(main())


@pytest.mark.parametrize("latency_s", [0.0, 0.001])
def test_native_scheduler_standin_binds_everything(latency_s):
    """native/src/schedsim.cpp drives the real runtime: every pod bound exactly once, no
    device over-committed. With API latency the in-place bind coroutine suspends and is
    resumed by NativeServer._resume."""
    from nanogpu.sim.driver import NativeSchedulerDriver, node_capacities

    async def main():
        store, rt = await _runtime(4)
        store.faults.latency_s = latency_s
        loop = asyncio.get_running_loop()
        try:
            rng = random.Random(3)
            pods = [store.create_pod(pu.make_pod(f"p{i}", [("c", rng.choice([10, 25, 50]))])) for i in range(120)]
            nodes = [f"n{i}" for i in range(4)]
            session = N.SchedulerSession()
            drv = NativeSchedulerDriver("127.0.0.1", rt.bound_port, nodes,
                                        node_capacities([store.get_node(n) for n in nodes]), bind_threads=32,
                                        session=session)
            st = await loop.run_in_executor(None, drv.run, pods[:60])
            # a second run on the same session reuses the first run's keep-alive connections
            drv2 = NativeSchedulerDriver("127.0.0.1", rt.bound_port, nodes,
                                         node_capacities([store.get_node(n) for n in nodes]), bind_threads=32,
                                         session=session)
            st2 = await loop.run_in_executor(None, drv2.run, pods[60:])
            placements = {**drv.placements, **drv2.placements}
            assert st.scheduled + st.failed == 60 and st.scheduled == 60
            assert st2.scheduled + st2.failed == 60 and st.scheduled + st2.scheduled >= 100
            st.scheduled += st2.scheduled
            assert len(placements) == st.scheduled
            bound = {(ns, name): node for ns, name, node in store.bindings}
            assert len(bound) == len(store.bindings) == st.scheduled
            for key, node in placements.items():
                assert bound[tuple(key.split("/"))] == node
            used = {}
            for p in store.pods.values():
                if pu.node_name_of(p):
                    idx = pu.container_assignment(p, "c")[0]
                    k = (pu.node_name_of(p), idx)
                    used[k] = used.get(k, 0) + pu.pod_demand(p)[0][0]
            assert max(used.values()) <= 100
            status = rt.state.status()
            for (n, i), u in used.items():
                assert status[n]["GPUs"][i]["Percent"] == 100 - u
        finally:
            await rt.stop()

    asyncio.run(main())


def test_inline_bind_failure_rolls_back():
    """A binding failure inside the in-place bind: 500 with the error, reservation rolled back
    (a failing label PATCH alone never fails a bind: the Binding carried the placement)."""
    async def main():
        store, rt = await _runtime(1)
        store.faults.bind_error_rate = 1.0
        loop = asyncio.get_running_loop()
        try:
            p = store.create_pod(pu.make_pod("x", [("c", 30)]))
            m = pu.meta(p)
            res = await loop.run_in_executor(None, _http, rt.bound_port, [
                ("POST", "/scheduler/filter", _dumps({"Pod": p, "NodeNames": ["n0"]})),
                ("POST", "/scheduler/bind", _dumps({"PodName": "x", "PodNamespace": "default", "PodUID": m["uid"],
                                                    "Node": "n0"}))])
            assert res[1][0] == 500 and "injected binding failure" in json.loads(res[1][1])["Error"]
            assert rt.state.ledger.lookup(m["uid"]) is None
            assert all(g["Percent"] == 100 for g in rt.state.status()["n0"]["GPUs"])
        finally:
            await rt.stop()

    asyncio.run(main())


def test_priorities_nominate_unique_best_and_bind_adopts():
    """Native priorities nominate the unique top node, so the next pod's filter sees the
    pod before its bind arrives; a tie at the top goes to the first tied node by one point
    (while kube-scheduler follows the nominations); compat mode never nominates; the bind
    adopts the nomination (a failed bind rolls it back)."""
    async def main():
        store, rt = await _runtime(2)
        loop = asyncio.get_running_loop()
        led = rt.state.ledger
        try:
            # n0 nearly full: 7 whole GPUs and 40 % of the last one, so a 60 % share fills
            # that GPU exactly (the unique best fit; on n1 it would leave a 40 % hole)
            base = store.create_pod(pu.make_pod("base", [("c", 100)] * 7 + [("d", 40)]))
            mb = pu.meta(base)
            await loop.run_in_executor(None, _http, rt.bound_port, [
                ("POST", "/scheduler/filter", _dumps({"Pod": base, "NodeNames": ["n0"]})),
                ("POST", "/scheduler/bind", _dumps({"PodName": "base", "PodNamespace": "default",
                                                    "PodUID": mb["uid"], "Node": "n0"}))])
            a = store.create_pod(pu.make_pod("a", [("c", 60)]))
            b = store.create_pod(pu.make_pod("b", [("c", 60)]))
            both = ["n0", "n1"]
            res = await loop.run_in_executor(None, _http, rt.bound_port, [
                ("POST", "/scheduler/filter", _dumps({"Pod": a, "NodeNames": both})),
                ("POST", "/scheduler/priorities", _dumps({"Pod": a, "NodeNames": both})),
                ("POST", "/scheduler/filter", _dumps({"Pod": b, "NodeNames": both}))])
            rec = led.lookup(pu.pod_uid(a))
            assert rec["state"] == "nominated" and rec["node"] == rt.state.node_entry("n0").id
            # b no longer fits n0: a's nomination holds the last GPU
            assert json.loads(res[2][1])["NodeNames"] == ["n1"]
            # a's own next attempt does not count its nomination against itself
            res = await loop.run_in_executor(None, _http, rt.bound_port, [
                ("POST", "/scheduler/filter", _dumps({"Pod": a, "NodeNames": both}))])
            assert json.loads(res[0][1])["NodeNames"] == both
            assert led.lookup(pu.pod_uid(a)) is None
            res = await loop.run_in_executor(None, _http, rt.bound_port, [
                ("POST", "/scheduler/priorities", _dumps({"Pod": a, "NodeNames": both})),
                ("POST", "/scheduler/bind", _dumps({"PodName": "a", "PodNamespace": "default",
                                                    "PodUID": pu.pod_uid(a), "Node": "n0"}))])
            assert res[1] == (200, b'{"Error":""}') and led.lookup(pu.pod_uid(a))["state"] == "committed"
            # a tie at the top (the same node twice) is broken for the one the pod's UID hash
            # picks, which is nominated and answered the priorities lead above the other
            c = store.create_pod(pu.make_pod("c", [("c", 10)]))
            res = await loop.run_in_executor(None, _http, rt.bound_port, [
                ("POST", "/scheduler/priorities", _dumps({"Pod": c, "NodeNames": ["n1", "n1"]}))])
            got = [h["Score"] for h in json.loads(res[0][1])]
            k = N.Ledger.owner_hash(pu.pod_uid(c)) % 2
            assert got[k] == got[1 - k] + rt.state.priority_lead
            rec = led.lookup(pu.pod_uid(c))
            assert rec["state"] == "nominated" and rec["node"] == rt.state.node_entry("n1").id
            led.drop_nomination(pu.pod_uid(c))
            # compat mode (the reference keeps no state between verbs): no nominations
            rt.state.set_policy("binpack", compat=True)
            d = store.create_pod(pu.make_pod("d", [("c", 10)]))
            await loop.run_in_executor(None, _http, rt.bound_port, [
                ("POST", "/scheduler/priorities", _dumps({"Pod": d, "NodeNames": both}))])
            assert led.lookup(pu.pod_uid(d)) is None
            # a failed bind of an adopted nomination rolls it back
            rt.state.set_policy("binpack", compat=False)
            store.faults.bind_error_rate = 1.0
            e = store.create_pod(pu.make_pod("e", [("c", 10)]))
            res = await loop.run_in_executor(None, _http, rt.bound_port, [
                ("POST", "/scheduler/priorities", _dumps({"Pod": e, "NodeNames": both})),
                ("POST", "/scheduler/bind", _dumps({"PodName": "e", "PodNamespace": "default",
                                                    "PodUID": pu.pod_uid(e), "Node": "n1"}))])
            assert res[1][0] == 500 and led.lookup(pu.pod_uid(e)) is None
        finally:
            await rt.stop()

    asyncio.run(main())


@pytest.mark.parametrize("policy,partition", [("binpack", "SPX"), ("spread", "CPX")])
def test_decisive_filter_answers_the_priorities_winner_byte_identical(policy, partition):
    """--decisive-filter: the native filter answers the one node the Python filter answers,
    byte for byte, which is the node priorities would rank first (ties broken by the pod's UID
    hash, as priorities breaks them), and nominates it; failed nodes keep their reasons."""
    async def main():
        store, rt = await _runtime(4, partition, priority=policy, decisive_filter=True)
        ext = rt.extender
        led = rt.state.ledger
        rng = random.Random(11)
        names = [f"n{i}" for i in range(4)]
        loop = asyncio.get_running_loop()
        try:
            for k, pod in enumerate(_pods(rng, 40)):
                pod = store.create_pod(pod)
                uid = pu.pod_uid(pod)
                body = {"Pod": pod, "Nodes": None, "NodeNames": rng.sample(names, rng.randint(1, 4))}
                raw = _dumps(body)
                got = await loop.run_in_executor(None, _http, rt.bound_port, [("POST", "/scheduler/filter", raw)])
                assert got[0] == (200, _dumps(ext.filter(json.loads(raw)))), got[0]
                ans = json.loads(got[0][1])
                fit = ans["NodeNames"]
                assert len(fit) <= 1
                # with the decisive answer's nomination dropped, priorities rank it first
                led.drop_nomination(uid)
                rt.state.decisive_filter = False
                full = ext.filter(json.loads(raw))
                prio = ext.prioritize(json.loads(raw))
                rt.state.decisive_filter = True
                assert set(full["FailedNodes"]) == set(ans["FailedNodes"])
                if full["NodeNames"]:
                    top = max(h["Score"] for h in prio if h["Host"] in full["NodeNames"])
                    winners = [h["Host"] for h in prio if h["Host"] in full["NodeNames"] and h["Score"] == top]
                    assert fit and fit[0] in winners, (fit, prio)
                else:
                    assert fit == []
                led.drop_nomination(uid)
                if fit and k % 2 == 0:
                    got = await loop.run_in_executor(None, _http, rt.bound_port, [("POST", "/scheduler/filter", raw)])
                    rec = led.lookup(uid)
                    wants = any(p > 0 or m > 0 for p, m in pu.ledger_view(rt.state.pod_demand(pod))[0])
                    if wants:
                        assert rec["state"] == "nominated" and rec["node"] == rt.state.node_entry(fit[0]).id
                    m = pu.meta(pod)
                    r = await ext.bind({"PodName": m["name"], "PodNamespace": m["namespace"],
                                        "PodUID": m["uid"], "Node": fit[0]})
                    assert r["Error"] == ""
            # compat mode (the reference's verbs): every fitting node again
            rt.state.set_policy(policy, compat=True)
            pod = store.create_pod(pu.make_pod("cmp", [("c", 10)]))
            raw = _dumps({"Pod": pod, "Nodes": None, "NodeNames": names})
            got = await loop.run_in_executor(None, _http, rt.bound_port, [("POST", "/scheduler/filter", raw)])
            assert len(json.loads(got[0][1])["NodeNames"]) > 1
            assert got[0] == (200, _dumps(ext.filter(json.loads(raw))))
        finally:
            await rt.stop()

    asyncio.run(main())


def test_decisive_filter_takes_one_round_trip_a_pod_through_the_standin():
    """With one feasible node kube-scheduler (the stand-in) skips scoring: every pod bound
    after a filter alone, no priorities call, no device over-committed."""
    from nanogpu.sim.driver import NativeSchedulerDriver, node_capacities

    async def main():
        store, rt = await _runtime(4, decisive_filter=True)
        loop = asyncio.get_running_loop()
        try:
            rng = random.Random(5)
            pods = [store.create_pod(pu.make_pod(f"p{i}", [("c", rng.choice([10, 25, 50]))])) for i in range(80)]
            nodes = [f"n{i}" for i in range(4)]
            drv = NativeSchedulerDriver("127.0.0.1", rt.bound_port, nodes,
                                        node_capacities([store.get_node(n) for n in nodes]), bind_threads=16)
            st = await loop.run_in_executor(None, drv.run, pods)
            assert st.scheduled == 80
            fs = rt.native.fe.stats()
            assert fs["priorities"]["count"] == 0 and fs["filter"]["count"] >= 80
            used = {}
            for p in store.pods.values():
                if pu.node_name_of(p):
                    k = (pu.node_name_of(p), pu.container_assignment(p, "c")[0])
                    used[k] = used.get(k, 0) + pu.pod_demand(p)[0][0]
            assert max(used.values()) <= 100
        finally:
            await rt.stop()

    asyncio.run(main())


def test_a_filter_with_one_fitting_node_nominates_it():
    """kube-scheduler binds a pod whose filter left one node without calling priorities: that
    filter nominates the node (native and Python alike), so the next pods' filters see the pod
    before its bind lands; with two fitting nodes the filter nominates nothing."""
    async def main():
        store, rt = await _runtime(2)
        ext, led = rt.extender, rt.state.ledger
        loop = asyncio.get_running_loop()
        try:
            a = store.create_pod(pu.make_pod("one", [("c", 30)]))
            res = await loop.run_in_executor(None, _http, rt.bound_port, [
                ("POST", "/scheduler/filter", _dumps({"Pod": a, "NodeNames": ["n1"]}))])
            assert json.loads(res[0][1])["NodeNames"] == ["n1"]
            rec = led.lookup(pu.pod_uid(a))
            assert rec["state"] == "nominated" and rec["node"] == rt.state.node_entry("n1").id
            b = store.create_pod(pu.make_pod("two", [("c", 30)]))
            await loop.run_in_executor(None, _http, rt.bound_port, [
                ("POST", "/scheduler/filter", _dumps({"Pod": b, "NodeNames": ["n0", "n1"]}))])
            assert led.lookup(pu.pod_uid(b)) is None
            # the Python verb does the same
            c = store.create_pod(pu.make_pod("three", [("c", 30)]))
            ext.filter({"Pod": c, "NodeNames": ["n0"]})
            assert led.lookup(pu.pod_uid(c))["state"] == "nominated"
            # and the bind adopts the nomination
            m = pu.meta(a)
            res = await loop.run_in_executor(None, _http, rt.bound_port, [
                ("POST", "/scheduler/bind", _dumps({"PodName": m["name"], "PodNamespace": "default",
                                                    "PodUID": m["uid"], "Node": "n1"}))])
            assert res[0] == (200, b'{"Error":""}') and led.lookup(pu.pod_uid(a))["state"] == "committed"
        finally:
            await rt.stop()

    asyncio.run(main())


def _fd_slots() -> int:
    for line in open("/proc/self/status"):
        if line.startswith("FDSize:"):
            return int(line.split()[1])
    return 0


def test_fd_table_is_presized():
    """The front door grows the fd table once at start-up: growth under load waits for an
    RCU grace period (measured 110-130 ms accept4() stalls on the MI355X host)."""
    import resource

    soft = resource.getrlimit(resource.RLIMIT_NOFILE)[0]
    want = 4096 if soft == resource.RLIM_INFINITY else min(4096, soft)
    got = N.presize_fd_table(want)
    if want <= 64:
        pytest.skip("RLIMIT_NOFILE too small")
    assert got == want
    assert _fd_slots() >= want


def test_memory_bound_annotation_reaches_the_ledger_through_the_native_path():
    """filter -> priorities -> bind over the native front door for a pod annotated
    nano-gpu/memory-bound: the reservation the front door makes carries the flag, so the
    device counts it, and the release takes it back."""
    async def main():
        store, rt = await _runtime(1, "SPX")
        loop = asyncio.get_running_loop()
        try:
            pod = pu.make_pod("mb", [("main", 25, 8192)])
            pod["metadata"]["annotations"][T.ANNOTATION_MEMORY_BOUND] = "true"
            pod = store.create_pod(pod)
            raw = _dumps({"Pod": pod, "Nodes": None, "NodeNames": ["n0"]})
            m = pu.meta(pod)
            bind = _dumps({"PodName": m["name"], "PodNamespace": m["namespace"], "PodUID": m["uid"], "Node": "n0"})
            got = await loop.run_in_executor(None, _http, rt.bound_port,
                                             [("POST", "/scheduler/filter", raw),
                                              ("POST", "/scheduler/priorities", raw),
                                              ("POST", "/scheduler/bind", bind)])
            assert [g[0] for g in got] == [200, 200, 200], got
            led = rt.state.ledger
            nid = led.find_node("n0")
            assert [d["mem_bound"] for d in led.snapshot(nid)["devices"]][0] == 1
            store.delete_pod(m["namespace"], m["name"])
            for _ in range(200):
                if led.snapshot(nid)["devices"][0]["mem_bound"] == 0:
                    break
                await asyncio.sleep(0.01)
            assert led.snapshot(nid)["devices"][0]["mem_bound"] == 0
        finally:
            await rt.stop()

    asyncio.run(main())


def test_native_node_id_cache_follows_node_removal_and_return():
    """Each front-door worker caches the node ids of a NodeNames list it has seen; a node
    deleted and re-created (new ledger slot) between identical filter requests must be
    resolved again, and answers stay byte-identical to the Python path."""
    async def main():
        store, rt = await _runtime(4, "SPX")
        ext = rt.extender
        loop = asyncio.get_running_loop()
        try:
            pod = store.create_pod(pu.make_pod("q", [("main", 50, 0)]))
            raw = _dumps({"Pod": pod, "Nodes": None, "NodeNames": ["n0", "n1", "n2", "n3"]})

            async def both():
                got = await loop.run_in_executor(None, _http, rt.bound_port, [("POST", "/scheduler/filter", raw),
                                                                              ("POST", "/scheduler/priorities", raw)])
                assert got[0] == (200, _dumps(ext.filter(json.loads(raw))))
                assert got[1] == (200, _dumps(ext.prioritize(json.loads(raw))))
                return json.loads(got[0][1])

            old_id = rt.state.ledger.find_node("n1")
            assert (await both())["NodeNames"] == ["n0", "n1", "n2", "n3"]
            node1 = store.get_node("n1")
            store.delete_node("n1")
            assert await _wait_until(lambda: rt.state.ledger.find_node("n1") < 0)
            r = await both()
            assert "n1" in r["FailedNodes"] and "n1" not in r["NodeNames"]
            store.add_node(node1)
            assert await _wait_until(lambda: rt.state.ledger.find_node("n1") >= 0)
            assert rt.state.ledger.find_node("n1") != old_id
            assert (await both())["NodeNames"] == ["n0", "n1", "n2", "n3"]
        finally:
            await rt.stop()

    asyncio.run(main())


async def _wait_until(pred, timeout=5.0):
    for _ in range(int(timeout / 0.01)):
        if pred():
            return True
        await asyncio.sleep(0.01)
    return pred()


def test_native_verbs_survive_mutated_bodies():
    """Fuzz: byte-level mutations of a valid filter body (truncation, flipped structure,
    wrong types, odd numbers). The native verb must never crash. Whatever it answers itself
    must equal the Python verb's answer on the same JSON; everything else it declines to
    Python, which is the specification."""
    async def main():
        store, rt = await _runtime(4)
        ext, fe = rt.extender, rt.native.fe
        rng = random.Random(11)
        pods = [store.create_pod(p) for p in _pods(rng, 8)]
        alphabet = b'{}[]:,"0123456789.-eE truefalsenull\\u'
        handled = declined = 0
        try:
            for it in range(3000):
                body = bytearray(_dumps({"Pod": rng.choice(pods), "Nodes": None,
                                         "NodeNames": rng.sample([f"n{i}" for i in range(4)], rng.randint(1, 4))}))
                for _ in range(rng.randint(1, 3)):
                    op, at = rng.random(), rng.randrange(len(body))
                    if op < 0.15:
                        del body[at:]
                    elif op < 0.5:
                        body[at] = rng.choice(alphabet)
                    elif op < 0.75:
                        body.insert(at, rng.choice(alphabet))
                    else:
                        del body[at]
                    if not body:
                        break
                raw = bytes(body)
                ok, _, out = fe.time_verb(raw, False, 1)
                fe.time_verb(raw, True, 1)
                if not ok:
                    declined += 1
                    continue
                handled += 1
                pu._DEMAND_CACHE.clear()   # Python memoises demands per UID (immutable in k8s)
                pu._DEMAND_CACHE_OWNED.clear()
                want = _dumps(ext.filter(json.loads(raw)))
                assert out == want, (raw, out, want)
        finally:
            await rt.stop()
        assert handled > 50 and declined > 50

    asyncio.run(main())


@pytest.mark.parametrize("routes", ["native", "python"])
def test_front_door_survives_mutated_http_framing(routes):
    """Fuzz the HTTP layer: pipelined Content-Length and chunked requests with bytes flipped,
    inserted, deleted or cut off, each on its own connection that the client half-closes.
    The front door must answer or close every one of them and keep serving good requests,
    both on the routes it answers itself and on those it hands to Python (bind, preemption)."""
    def blast(port, data):
        s = socket.create_connection(("127.0.0.1", port))
        s.settimeout(0.5)
        try:
            s.sendall(data)
            s.shutdown(socket.SHUT_WR)
            while s.recv(65536):
                pass
        except (socket.timeout, ConnectionResetError, BrokenPipeError):
            pass
        finally:
            s.close()

    async def main():
        store, rt = await _runtime(4)
        rng = random.Random(3)
        pods = [store.create_pod(p) for p in _pods(rng, 4)]
        loop = asyncio.get_running_loop()
        good = _dumps({"Pod": pods[0], "Nodes": None, "NodeNames": ["n0", "n1"]})
        bodies = {b"/scheduler/bind": _dumps({"PodName": "p0", "PodNamespace": "default",
                                               "PodUID": pods[0]["metadata"]["uid"], "Node": "n0"}),
                  b"/scheduler/preemption": _dumps({"Pod": pods[0], "NodeNameToMetaVictims": {
                      "n0": {"Pods": [{"UID": "x"}], "NumPDBViolations": 0}}})}
        paths = [b"/scheduler/filter", b"/scheduler/priorities", b"/version", b"/status"] if routes == "native" \
            else [b"/scheduler/bind", b"/scheduler/preemption", b"/status"]
        alphabet = b"\r\n: 0123456789abcdefABCDEF-;chunkedContent-LengthTransfer-Encoding"
        try:
            for it in range(400):
                path = rng.choice(paths)
                body = bodies.get(path, good)
                if rng.random() < 0.5:
                    req = b"POST " + path + b" HTTP/1.1\r\nHost: x\r\nContent-Length: " + \
                        str(len(body)).encode() + b"\r\n\r\n" + body
                else:
                    mid = len(body) // 2
                    req = b"POST " + path + b" HTTP/1.1\r\nHost: x\r\nTransfer-Encoding: chunked\r\n\r\n" + \
                        b"".join(f"{len(p):x}\r\n".encode() + p + b"\r\n" for p in (body[:mid], body[mid:])) + \
                        b"0\r\n\r\n"
                data = bytearray(req * rng.randint(1, 3))
                for _ in range(rng.randint(1, 4)):
                    at, op = rng.randrange(len(data)), rng.random()
                    if op < 0.4:
                        data[at] = rng.choice(alphabet)
                    elif op < 0.7:
                        data.insert(at, rng.choice(alphabet))
                    elif op < 0.9:
                        del data[at]
                    else:
                        del data[at:]
                    if not data:
                        break
                await loop.run_in_executor(None, blast, rt.bound_port, bytes(data))
                if it % 50 == 49:
                    got = await loop.run_in_executor(None, _http, rt.bound_port, [("POST", "/scheduler/filter", good)])
                    assert got[0][0] == 200
        finally:
            await rt.stop()

    asyncio.run(main())


def test_escaped_node_names_still_answer_byte_identical():
    """The native verbs reuse each NodeNames token as written; a token with an escape is
    re-quoted, so the reply still equals json.dumps of the Python verb's answer."""
    from nanogpu.extender.verbs import Extender
    from nanogpu.k8s.fake_apiserver import FakeKubeStore, InProcKube
    from nanogpu.state.cluster import ClusterState

    st = ClusterState()
    for n in ("n0", "n1"):
        st.register_node(pu.make_node(n, 8, synthetic_mi355x(8).to_json()))
    ext = Extender(st, InProcKube(FakeKubeStore()))
    fe = N.Frontend(st.ledger, "127.0.0.1", 0, 1)
    try:
        fe.set_options(st.options, False, st.nominate, False, st.priority_lead)   # the Python verb's rules
        raw = ('{"Pod":' + json.dumps(pu.make_pod("p", [("c", 20)])) + ',"NodeNames":["n\\u0030","n1"]}').encode()
        ok, _, out = fe.time_verb(raw, False, 1)
        assert ok and out == _dumps(ext.filter(json.loads(raw)))
        ok, _, out = fe.time_verb(raw, True, 1)
        assert ok and out == _dumps(ext.prioritize(json.loads(raw)))
    finally:
        fe.stop()


def test_sampled_windows_and_their_fitting_subsets_answer_byte_identical():
    """kube-scheduler sends windows of its node order (nodes it counts as full left out) and then
    priorities over exactly the nodes filter answered. The native verbs scan a list 16 bytes at
    a time, resolve names by their predecessor's last successor, and keep a filter's fitting
    subset as a list of its own for that priorities call: names of every length across the
    16-byte blocks, windows that skip filled nodes and lists in other shapes (spaces: the JSON
    parser's path) must all answer what the Python verbs answer."""
    from nanogpu.extender.verbs import Extender
    from nanogpu.state.cluster import ClusterState

    st = ClusterState()
    names = [("n" * (1 + i % 23)) + f"-{i}" for i in range(30)] + ["x", "gpu.rack-2.example.com", "mi355x-node-0000000000000017"]
    for n in names:
        st.register_node(pu.make_node(n, 8, synthetic_mi355x(8).to_json()))
    ext = Extender(st, InProcKube(FakeKubeStore()))
    fe = N.Frontend(st.ledger, "127.0.0.1", 0, 1)
    rng = random.Random(5)
    opts = st.options
    try:
        fe.set_options(opts, False, st.nominate, False, st.priority_lead)
        n_subsets = 0
        for k in range(300):
            if k % 10 == 0:   # fill a node whole, free another: the windows change
                full = rng.choice(names)
                for d in range(8):
                    st.ledger.reserve(st.ledger.find_node(full), f"fill-{k}-{d}", [(100, 0)], opts)
                if k >= 20:
                    for d in range(8):
                        st.ledger.release(f"fill-{k - 20}-{d}")
            start, size = rng.randrange(len(names)), rng.randint(2, len(names))
            window = [names[(start + j) % len(names)] for j in range(size)]
            pod = pu.make_pod(f"p{k}", [("c", rng.choice([10, 25, 50, 100]))])
            body = {"Pod": pod, "Nodes": None, "NodeNames": window}
            raw = _dumps(body) if k % 7 else json.dumps(body).encode()   # spaces: the general path
            ok, _, out = fe.time_verb(raw, False, 1)
            want = _dumps(ext.filter(json.loads(raw)))
            assert ok and out == want, (k, out, want)
            fit = json.loads(out)["NodeNames"]
            if len(fit) < 2:
                continue
            n_subsets += len(fit) < len(window)
            praw = _dumps({"Pod": pod, "Nodes": None, "NodeNames": fit})
            ok, _, out = fe.time_verb(praw, True, 1)
            assert ok and out == _dumps(ext.prioritize(json.loads(praw))), (k, out)
        assert n_subsets > 20
    finally:
        fe.stop()


def test_priorities_reuse_their_filters_placements_only_while_nothing_changed():
    """Priorities right behind its pod's filter reads the placements that filter computed
    (Frontend::reuse_assume) instead of walking the nodes again, as long as the ledger saw no
    mutation in between. A reservation, a release or a telemetry mark in between makes it
    compute afresh: every answer equals the Python verb's on the state of its moment."""
    from nanogpu.extender.verbs import Extender
    from nanogpu.state.cluster import ClusterState

    st = ClusterState(nominate=False)   # no nominations: only the test's own mutations
    names = [f"n{i}" for i in range(6)]
    for n in names:
        st.register_node(pu.make_node(n, 8, synthetic_mi355x(8).to_json()))
    ext = Extender(st, InProcKube(FakeKubeStore()))
    fe = N.Frontend(st.ledger, "127.0.0.1", 0, 1)
    rng = random.Random(9)
    try:
        fe.set_options(st.options, False, st.nominate, False, st.priority_lead)   # the Python verb's rules
        for k in range(200):
            pod = pu.make_pod(f"p{k}", [("c", rng.choice([10, 25, 50]))])
            raw = _dumps({"Pod": pod, "Nodes": None, "NodeNames": names})
            ok, _, out = fe.time_verb(raw, False, 1)
            assert ok and out == _dumps(ext.filter(json.loads(raw)))
            fit = json.loads(out)["NodeNames"]
            what = k % 4
            if what == 1:      # a reservation lands on a fitting node between the two verbs
                st.ledger.reserve(st.ledger.find_node(rng.choice(fit)), f"x{k}", [(rng.choice([10, 50]), 0)],
                                  st.options)
            elif what == 2 and k > 8:   # an older one is released
                st.ledger.release(f"x{k - 7}")
            elif what == 3:    # a device turns HBM-hot
                st.ledger.set_mem_hot(st.ledger.find_node(rng.choice(names)), rng.randrange(8), True)
            praw = _dumps({"Pod": pod, "Nodes": None, "NodeNames": fit})
            ok, _, out = fe.time_verb(praw, True, 1)
            assert ok and out == _dumps(ext.prioritize(json.loads(praw))), (k, what)
    finally:
        fe.stop()


def test_learned_streaming_owner_marks_its_next_pods_memory_bound_on_the_native_path():
    """A device measured HBM-hot while it holds one pod alone makes that pod's controlling
    owner a streaming owner (Ledger::learn_stream_owners). The owner's next unannotated pods
    then reach the ledger memory-bound through the native front door: they keep off the hot
    device that best fit would pick. nano-gpu/memory-bound: "false" opts a pod out."""
    async def main():
        store, rt = await _runtime(1, "SPX")
        loop = asyncio.get_running_loop()
        led = rt.state.ledger
        nid = led.find_node("n0")

        async def schedule(name, ann=None):
            pod = pu.make_pod(name, [("main", 25, 8192)])
            pod["metadata"]["ownerReferences"] = [
                {"apiVersion": "apps/v1", "kind": "ReplicaSet", "name": "rs", "uid": "rs-uid-1", "controller": True}]
            if ann is not None:
                pod["metadata"]["annotations"][T.ANNOTATION_MEMORY_BOUND] = ann
            pod = store.create_pod(pod)
            raw = _dumps({"Pod": pod, "Nodes": None, "NodeNames": ["n0"]})
            m = pu.meta(pod)
            bind = _dumps({"PodName": m["name"], "PodNamespace": m["namespace"], "PodUID": m["uid"], "Node": "n0"})
            got = await loop.run_in_executor(None, _http, rt.bound_port,
                                             [("POST", "/scheduler/filter", raw),
                                              ("POST", "/scheduler/priorities", raw),
                                              ("POST", "/scheduler/bind", bind)])
            assert [g[0] for g in got] == [200, 200, 200], got
            for _ in range(200):
                rec = led.lookup(m["uid"])
                if rec and rec["state"] == "committed":
                    return rec
                await asyncio.sleep(0.01)
            raise AssertionError(f"{name} not committed")

        try:
            a = await schedule("a")
            assert a["owner"] == N.Ledger.owner_hash("rs-uid-1")
            (dev_a,) = a["plan"][0]
            assert led.learn_stream_owners(True) == (0, 0)         # nothing measured hot yet
            assert led.set_mem_hot(nid, dev_a, True) == N.OK
            assert led.learn_stream_owners(True) == (1, 0) and led.is_stream_owner("rs-uid-1")
            b = await schedule("b")                                # same owner, no annotation
            (dev_b,) = b["plan"][0]
            assert dev_b != dev_a                                  # best fit alone would stack it on a
            mb = [d["mem_bound"] for d in led.snapshot(nid)["devices"]]
            assert mb[dev_b] == 1 and sum(mb) == 1                 # b reached the ledger memory-bound
            await schedule("c", ann="false")                       # opted out
            assert sum(d["mem_bound"] for d in led.snapshot(nid)["devices"]) == 1
            assert led.set_mem_hot(nid, dev_a, False) == N.OK      # a's device cooled: forgotten
            assert led.learn_stream_owners(True) == (0, 1) and not led.is_stream_owner("rs-uid-1")
        finally:
            await rt.stop()

    asyncio.run(main())


def test_owner_learned_between_priorities_and_bind_is_tolerated():
    """the owner-derived memory-bound flag is read per request, so a learning
    pass between a pod's priorities and its bind gives the bind a different demand than the one
    scored. That is tolerated by design: the bind adopts the priorities-time nomination (the
    ledger keeps the nominated plan and its demand), so the pod lands where it was nominated and
    commits; the next pods of the owner are the ones placed as memory-bound."""
    async def main():
        store, rt = await _runtime(1, "SPX")
        loop = asyncio.get_running_loop()
        led = rt.state.ledger
        try:
            pod = pu.make_pod("p", [("main", 25, 8192)])
            pod["metadata"]["ownerReferences"] = [
                {"apiVersion": "apps/v1", "kind": "ReplicaSet", "name": "rs", "uid": "rs-late", "controller": True}]
            pod = store.create_pod(pod)
            raw = _dumps({"Pod": pod, "Nodes": None, "NodeNames": ["n0"]})
            got = await loop.run_in_executor(None, _http, rt.bound_port,
                                             [("POST", "/scheduler/filter", raw), ("POST", "/scheduler/priorities", raw)])
            assert [g[0] for g in got] == [200, 200]
            uid = pu.pod_uid(pod)
            nom = led.lookup(uid)
            assert nom is not None and nom["state"] == "nominated"
            led.set_stream_owner("rs-late", True)          # learned in between
            m = pu.meta(pod)
            bind = _dumps({"PodName": m["name"], "PodNamespace": m["namespace"], "PodUID": uid, "Node": "n0"})
            got = await loop.run_in_executor(None, _http, rt.bound_port, [("POST", "/scheduler/bind", bind)])
            assert got[0] == (200, b'{"Error":""}')
            for _ in range(200):
                rec = led.lookup(uid)
                if rec and rec["state"] == "committed":
                    break
                await asyncio.sleep(0.01)
            assert rec["state"] == "committed" and rec["plan"] == nom["plan"]
            assert sum(d["pct_free"] for d in led.snapshot(led.find_node("n0"))["devices"]) == 8 * 100 - 25
        finally:
            await rt.stop()

    asyncio.run(main())


def test_rotating_node_windows_answer_byte_identical_through_the_list_cache():
    """kube-scheduler's node sampling sends a moving window of the cluster each cycle. The
    native verbs cache the last 64 distinct lists (ids and token offsets), answer a fully
    fitting filter with the request's own list text, and resolve new windows through a per-
    thread name table. Every answer must still equal the Python verb's, across LRU evictions,
    nodes that do not fit, a node added (the ledger's node epoch moves) and an unknown name."""
    import random

    from nanogpu.extender.verbs import Extender
    from nanogpu.k8s.fake_apiserver import FakeKubeStore, InProcKube
    from nanogpu.state.cluster import ClusterState

    st = ClusterState()
    names = [f"node-{i:02d}" for i in range(30)]
    for n in names:
        st.register_node(pu.make_node(n, 8, synthetic_mi355x(8).to_json()))
    # some nodes nearly full: their FailedNodes entries interleave with the fitting ones
    for k, n in enumerate(names[::3]):
        nid = st.node_ids([n])[0]
        for dev in range(8):
            st.ledger.allocate_plan(nid, f"fill-{k}-{dev}", [(95, 0)], [[dev]], True)
    ext = Extender(st, InProcKube(FakeKubeStore()))
    fe = N.Frontend(st.ledger, "127.0.0.1", 0, 1)
    rnd = random.Random(4)
    try:
        fe.set_options(st.options, False, st.nominate, False, st.priority_lead)   # the Python verb's rules
        for step in range(160):
            if step == 100:   # a new node: every cached list re-checks its ids
                st.register_node(pu.make_node("node-new", 8, synthetic_mi355x(8).to_json()))
                names.append("node-new")
            start, size = rnd.randrange(len(names)), rnd.choice([5, 12, 25])
            window = [names[(start + j) % len(names)] for j in range(size)]
            pct = rnd.choice([10, 50])
            raw = json.dumps({"Pod": pu.make_pod(f"p{step}", [("c", pct)]), "NodeNames": window},
                             separators=(",", ":")).encode()
            for prio, verb in ((False, ext.filter), (True, ext.prioritize)):
                ok, _, out = fe.time_verb(raw, prio, 1)
                assert ok and out == _dumps(verb(json.loads(raw))), (step, prio)
        unknown = json.dumps({"Pod": pu.make_pod("u", [("c", 10)]), "NodeNames": names[:3] + ["ghost"]},
                             separators=(",", ":")).encode()
        assert fe.time_verb(unknown, False, 1)[0] is False     # Python registers or rejects it
        ok, _, out = fe.time_verb(json.dumps({"Pod": pu.make_pod("v", [("c", 10)]), "NodeNames": names[:3]},
                                             separators=(",", ":")).encode(), False, 1)
        assert ok and json.loads(out)["NodeNames"] == [n for n in names[:3] if n != "node-00"]
    finally:
        fe.stop()


def test_ambiguous_request_framing_is_refused():
    """`Content-Length: 12abc` (a numeric prefix), a second Content-Length that
    disagrees, or Content-Length together with chunked encoding would let the front door and a
    proxy in front of it frame the same bytes differently (request smuggling): each closes the
    connection without an answer. Well-framed requests, a repeated equal Content-Length
    included, are answered."""
    def send(port, data):
        s = socket.create_connection(("127.0.0.1", port))
        s.settimeout(2.0)
        try:
            s.sendall(data)
            s.shutdown(socket.SHUT_WR)
            out = b""
            while True:
                got = s.recv(65536)
                if not got:
                    return out
                out += got
        except (socket.timeout, ConnectionResetError):
            return b"<timeout>"
        finally:
            s.close()

    async def main():
        store, rt = await _runtime(2)
        loop = asyncio.get_running_loop()
        pod = store.create_pod(_pods(random.Random(1), 1)[0])
        body = _dumps({"Pod": pod, "NodeNames": ["n0"]})
        head = b"POST /scheduler/filter HTTP/1.1\r\nHost: x\r\n"
        n = str(len(body)).encode()
        try:
            for extra, answered in [(b"Content-Length: " + n + b"\r\n", True),
                                    (b"Content-Length: " + n + b"\r\nContent-Length: " + n + b"\r\n", True),
                                    (b"Content-Length: " + n + b"abc\r\n", False),
                                    (b"Content-Length: " + n + b", " + n + b"\r\n", False),
                                    (b"Content-Length: " + n + b"\r\nContent-Length: 3\r\n", False),
                                    (b"Content-Length: " + n + b"\r\nTransfer-Encoding: chunked\r\n", False)]:
                got = await loop.run_in_executor(None, send, rt.bound_port, head + extra + b"\r\n" + body)
                assert got.startswith(b"HTTP/1.1 200") == answered, (extra, got[:80])
                if not answered:
                    assert got == b"", (extra, got[:80])
        finally:
            await rt.stop()

    asyncio.run(main())


def test_io_tally_counts_the_front_door_calls_of_a_cycle():
    """bench.py --io-tally: with the tally on, one filter + priorities exchange shows up as
    recv / verb / cycle-send calls at their sites; off, nothing is counted."""
    async def main():
        store, rt = await _runtime(2)
        loop = asyncio.get_running_loop()
        try:
            pod = store.create_pod(pu.make_pod("t0", [("c0", 25, 0)]))
            raw = _dumps({"Pod": pod, "Nodes": None, "NodeNames": ["n0", "n1"]})
            reqs = [("POST", "/scheduler/filter", raw), ("POST", "/scheduler/priorities", raw)]
            N.io_tally_reset()
            await loop.run_in_executor(None, _http, rt.bound_port, reqs)
            assert N.io_tally() == {}
            N.io_tally_enable(True)
            try:
                got = await loop.run_in_executor(None, _http, rt.bound_port, reqs)
            finally:
                N.io_tally_enable(False)
            assert [s for s, _ in got] == [200, 200]
            t = N.io_tally()
            assert t["fe_verb"][0] == 2 and t["fe_send_cycle"][0] == 2, t
            assert t["fe_recv"][0] >= 1 and all(sec >= 0.0 for _, sec in t.values()), t
        finally:
            await rt.stop()

    asyncio.run(main())


def test_compact_args_layout_and_general_layout_answer_alike():
    """The verbs' fast framing (kube-scheduler's exact {"Pod":..,"Nodes":null,"NodeNames":[..]}
    layout, the pod found by comparison with the last one or parsed in place) and the general
    path (any other layout: spaces, member order) give the same answers, and a body that only
    looks framed (trailing members, a list that is not one) still gets the general path's
    verdict."""
    async def main():
        store, rt = await _runtime(4)
        fe = rt.native.fe
        ext = rt.extender
        names = [f"n{i}" for i in range(4)]
        rng = random.Random(3)
        try:
            for pod in _pods(rng, 12):
                pod = store.create_pod(pod)
                compact = _dumps({"Pod": pod, "Nodes": None, "NodeNames": names})
                spaced = json.dumps({"NodeNames": names, "Pod": pod, "Nodes": None}).encode()
                for prio in (False, True):
                    want = _dumps(ext.prioritize(json.loads(compact)) if prio else ext.filter(json.loads(compact)))
                    for body in (compact, spaced, compact):   # framed + parsed, general, framed + reused
                        ok, got = fe.verb(body, prio)
                        assert ok and got == want.decode(), (prio, body[:40], got)
            pod = _pods(rng, 1)[0]
            pod["metadata"]["name"] = "framing-edge"
            pod = store.create_pod(pod)
            base = _dumps({"Pod": pod, "Nodes": None, "NodeNames": names})
            want = _dumps(ext.filter(json.loads(base))).decode()
            assert fe.verb(base, False) == (True, want)
            # valid JSON with a member after the list: not the framed layout, answered alike
            for extra in (base[:-1] + b',"x":["y"]}', base[:-1] + b',"x":1}'):
                assert fe.verb(extra, False) == (True, want), extra[-20:]
            # not JSON (a stray bracket after the list): never answered natively
            assert fe.verb(base[:-1] + b']}', False)[0] is False
            assert fe.verb(base.replace(b'"NodeNames":["n0"', b'"NodeNames":["n0"]]', 1), False)[0] is False
        finally:
            await rt.stop()

    asyncio.run(main())


def test_filter_to_bind_pod_cache_stays_bounded_and_evicted_pods_still_bind():
    """The filter -> bind pod cache is 4-way buckets of fixed size: filtering more pods than it
    holds keeps it at its size, a recent pod's bind stays native, and a pod whose entry was
    given up still binds (Python reads the pod itself)."""
    async def main():
        store, rt = await _runtime(4)
        fe = rt.native.fe
        ext = rt.extender
        loop = asyncio.get_running_loop()
        try:
            first = store.create_pod(pu.make_pod("evict-first", [("c0", 10, 0)]))
            fe.verb(_dumps({"Pod": first, "Nodes": None, "NodeNames": ["n0"]}), False)
            for i in range(17000):   # more pods than the cache holds (16384)
                p = pu.make_pod(f"f{i}", [("c0", 10, 0)])
                assert fe.verb(_dumps({"Pod": p, "Nodes": None, "NodeNames": ["n1"]}), False)[0]
            assert fe.pod_cache_size() <= 16384
            last = store.create_pod(pu.make_pod("evict-last", [("c0", 10, 0)]))
            fe.verb(_dumps({"Pod": last, "Nodes": None, "NodeNames": ["n2"]}), False)
            for pod, node in ((last, "n2"), (first, "n0")):
                m = pu.meta(pod)
                body = _dumps({"PodName": m["name"], "PodNamespace": m["namespace"], "PodUID": m["uid"], "Node": node})
                got = await loop.run_in_executor(None, _http, rt.bound_port, [("POST", "/scheduler/bind", body)])
                assert got[0] == (200, b'{"Error":""}'), got
                assert rt.state.ledger.lookup(m["uid"]) is not None
        finally:
            await rt.stop()

    asyncio.run(main())
