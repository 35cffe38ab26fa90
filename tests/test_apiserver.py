"""The native API server (native/src/apiserver.cpp) against the Python HTTP fake
(nanogpu/k8s/fake_apiserver.py): one behaviour suite, run over the REST client against both,
so the bench's shared API server answers exactly what the tests' fake answers (codes, Status
bodies, merge-patch, binding conflicts, selectors, watch resume, 410 Gone)."""
import asyncio
import json

import pytest

from nanogpu import _native as N
from nanogpu.k8s import podutil as pu
from nanogpu.k8s.client import ApiError, KubeClient, KubeConfig
from nanogpu.k8s.fake_apiserver import FakeKubeStore, serve


class PyServer:
    async def start(self):
        self.store = FakeKubeStore(history=64)
        self.runner, port = await serve(self.store)
        return f"http://127.0.0.1:{port}"

    def compact(self):
        self.store.compact("pods")

    async def stop(self):
        await self.runner.cleanup()


class NativeServer:
    async def start(self):
        self.srv = N.ApiServer("127.0.0.1", 0, 2, 64)
        return f"http://127.0.0.1:{self.srv.port}"

    def compact(self):
        self.srv.compact("pods")

    async def stop(self):
        self.srv.stop()


def run(kind, body):
    async def main():
        srv = PyServer() if kind == "python" else NativeServer()
        url = await srv.start()
        api = KubeClient(KubeConfig(server=url))
        try:
            await body(api, srv)
        finally:
            await api.close()
            await srv.stop()

    asyncio.run(main())


KINDS = ["python", "native"]


@pytest.mark.parametrize("kind", KINDS)
def test_pod_lifecycle_codes_and_bodies(kind):
    async def body(api, srv):
        await api.request("POST", "/api/v1/nodes", pu.make_node("n0", 8, "{}"))
        p = await api.create_pod(pu.make_pod("a", [("main", 20)], namespace="ns1"))
        m = pu.meta(p)
        assert m["namespace"] == "ns1" and m["uid"] and m["resourceVersion"] and p["status"]["phase"] == "Pending"
        with pytest.raises(ApiError) as e:
            await api.create_pod(pu.make_pod("a", [("main", 20)], namespace="ns1"))
        assert e.value.status == 409 and e.value.reason == "AlreadyExists"
        q = await api.patch_pod("ns1", "a", {"metadata": {"annotations": {"x": "1"}, "labels": {"l": "v"}}})
        assert q["metadata"]["annotations"]["x"] == "1" and int(q["metadata"]["resourceVersion"]) > int(m["resourceVersion"])
        q = await api.patch_pod("ns1", "a", {"metadata": {"annotations": {"x": None}}})
        assert "x" not in q["metadata"]["annotations"] and q["metadata"]["labels"]["l"] == "v"
        with pytest.raises(ApiError) as e:
            await api.bind_pod("ns1", "a", "wrong-uid", "n0")
        assert e.value.status == 409
        with pytest.raises(ApiError) as e:
            await api.bind_pod("ns1", "a", m["uid"], "nope")
        assert e.value.status == 404
        await api.bind_pod("ns1", "a", m["uid"], "n0", annotations={"nano-gpu/container-main": "3", "l": "v2"})
        got = await api.get_pod("ns1", "a")
        assert got["spec"]["nodeName"] == "n0" and got["status"]["phase"] == "Running"
        # the Binding's annotations land with the node (kube-apiserver setPodHostAndAnnotations)
        assert got["metadata"]["annotations"]["nano-gpu/container-main"] == "3"
        with pytest.raises(ApiError) as e:
            await api.bind_pod("ns1", "a", m["uid"], "n0")
        assert e.value.status == 409 and "already assigned" in e.value.message
        await api.delete_pod("ns1", "a")
        with pytest.raises(ApiError) as e:
            await api.get_pod("ns1", "a")
        assert e.value.status == 404 and e.value.reason == "NotFound"
        with pytest.raises(ApiError) as e:
            await api.delete_pod("ns1", "a")
        assert e.value.status == 404

    run(kind, body)


@pytest.mark.parametrize("kind", KINDS)
def test_selectors_and_listing(kind):
    async def body(api, srv):
        await api.request("POST", "/api/v1/nodes", pu.make_node("n0", 8, "{}", {"gpu": "yes"}))
        await api.request("POST", "/api/v1/nodes", pu.make_node("n1", 8, "{}"))
        for i in range(4):
            p = await api.create_pod(pu.make_pod(f"p{i}", [("main", 10)]))
            if i % 2:
                await api.patch_pod("default", f"p{i}", {"metadata": {"labels": {"nano-gpu/assume": "true"}}})
                await api.bind_pod("default", f"p{i}", pu.pod_uid(p), "n0")
        items, rv = await api.list_pods(label_selector="nano-gpu/assume=true", field_selector="spec.nodeName=n0")
        assert sorted(pu.meta(p)["name"] for p in items) == ["p1", "p3"] and int(rv) > 0
        items, _ = await api.list_pods(label_selector="nano-gpu/assume!=true")
        assert sorted(pu.meta(p)["name"] for p in items) == ["p0", "p2"]
        items, _ = await api.list_pods(namespace="other")
        assert items == []
        nodes, _ = await api.list_nodes(label_selector="gpu")
        assert [pu.meta(n)["name"] for n in nodes] == ["n0"]
        n = await api.patch_node_status("n1", {"status": {"capacity": {"nano-gpu/gpu-percent": "800"}}})
        assert n["status"]["capacity"]["nano-gpu/gpu-percent"] == "800"

    run(kind, body)


@pytest.mark.parametrize("kind", KINDS)
def test_watch_resume_and_gone(kind):
    async def body(api, srv):
        await api.create_pod(pu.make_pod("a", [("main", 10)]))
        _, rv = await api.list_pods()
        await api.create_pod(pu.make_pod("b", [("main", 10)]))
        await api.patch_pod("default", "b", {"metadata": {"annotations": {"k": "v"}}})
        await api.delete_pod("default", "a")
        seen = []

        async def consume():
            async for batch in api.watch_batches("pods", rv, timeout_s=1):
                seen.extend((ev["type"], pu.meta(ev["object"])["name"]) for ev in batch)
                if len(seen) >= 3:
                    return

        await asyncio.wait_for(consume(), 5)
        assert seen == [("ADDED", "b"), ("MODIFIED", "b"), ("DELETED", "a")]
        # live events reach an open watch
        _, rv2 = await api.list_pods()
        got = []

        async def live():
            async for ev in api.watch("pods", rv2, timeout_s=2):
                got.append(ev["type"])
                return

        task = asyncio.ensure_future(live())
        await asyncio.sleep(0.1)
        await api.create_pod(pu.make_pod("c", [("main", 10)]))
        await asyncio.wait_for(task, 5)
        assert got == ["ADDED"]
        # the watch cache forgets: a resume from an old version is 410 Gone (HTTP or in-stream)
        srv.compact()
        gone = None
        try:
            async for ev in api.watch("pods", rv, timeout_s=1):
                gone = ev
                break
        except ApiError as e:
            gone = {"type": "ERROR", "object": {"code": e.status}}
        assert gone["type"] == "ERROR" and gone["object"]["code"] == 410

    run(kind, body)


@pytest.mark.parametrize("kind", KINDS)
def test_watch_label_selector_filters_and_no_selector_sees_all(kind):
    async def body(api, srv):
        await api.create_pod(pu.make_pod("seed", [("main", 10)]))
        _, rv = await api.list_pods()
        await api.create_pod(pu.make_pod("plain", [("main", 10)]))
        tagged = pu.make_pod("tagged", [("main", 10)])
        pu.meta(tagged).setdefault("labels", {})["team"] = "a"
        await api.create_pod(tagged)
        await api.delete_pod("default", "plain")
        await api.delete_pod("default", "tagged")

        async def take(n, sel):
            seen = []
            async for batch in api.watch_batches("pods", rv, timeout_s=1, label_selector=sel):
                seen.extend((ev["type"], pu.meta(ev["object"])["name"]) for ev in batch)
                if len(seen) >= n:
                    return seen
            return seen

        assert await asyncio.wait_for(take(4, None), 5) == [
            ("ADDED", "plain"), ("ADDED", "tagged"), ("DELETED", "plain"), ("DELETED", "tagged")]
        assert await asyncio.wait_for(take(2, "team=a"), 5) == [("ADDED", "tagged"), ("DELETED", "tagged")]

    run(kind, body)


@pytest.mark.parametrize("kind", KINDS)
def test_leases_and_events(kind):
    async def body(api, srv):
        lease = {"apiVersion": "coordination.k8s.io/v1", "kind": "Lease", "metadata": {"name": "x"},
                 "spec": {"holderIdentity": "a"}}
        le = await api.create_lease("kube-system", lease)
        with pytest.raises(ApiError) as e:
            await api.create_lease("kube-system", lease)
        assert e.value.status == 409
        le["spec"]["holderIdentity"] = "b"
        le2 = await api.update_lease("kube-system", "x", le)
        assert le2["spec"]["holderIdentity"] == "b"
        with pytest.raises(ApiError) as e:
            await api.update_lease("kube-system", "x", le)            # stale resourceVersion
        assert e.value.status == 409
        assert (await api.get_lease("kube-system", "x"))["spec"]["holderIdentity"] == "b"
        await api.create_event("default", {"kind": "Pod", "name": "p"}, "FailedBinding", "m")

    run(kind, body)


def test_native_bulk_create_delete_and_timeout_ends_the_stream():
    srv = N.ApiServer("127.0.0.1", 0, 2, 1000)
    try:
        pods = [json.dumps(pu.make_pod(f"p{i}", [("main", 10)], namespace="b")) for i in range(50)]
        assert srv.create_pods(pods) == [201] * 50
        assert srv.create_pods(pods[:1]) == [409]
        code, body = srv.call("GET", "/api/v1/namespaces/b/pods")
        assert code == 200 and len(json.loads(body)["items"]) == 50
        assert srv.delete_pods([("b", f"p{i}") for i in range(60)]) == 50
        st = json.loads(srv.stats())
        assert st["pods"] == 0 and st["calls"]["create_pod"] == 50

        async def main():
            api = KubeClient(KubeConfig(server=f"http://127.0.0.1:{srv.port}"))
            try:
                _, rv = await api.list_pods()
                t0 = asyncio.get_running_loop().time()
                async for _ in api.watch("pods", rv, timeout_s=1):
                    pass                                   # nothing happens; the stream ends cleanly
                assert 0.8 < asyncio.get_running_loop().time() - t0 < 3.0
            finally:
                await api.close()

        asyncio.run(main())
    finally:
        srv.stop()


def test_native_bulk_writes_in_chunks_keep_every_pod_and_event():
    """Bulk create / delete take the store's lock 128 pods at a time (a bind waits for one
    chunk): a 300-pod burst still lands whole, a watcher sees each pod's ADDED and DELETED once,
    in resourceVersion order, and a small watch cache evicting under them loses nothing live."""
    import socket
    import threading

    srv = N.ApiServer("127.0.0.1", 0, 2, 256)
    got = bytearray()
    s = socket.create_connection(("127.0.0.1", srv.port))
    try:
        s.sendall(b"GET /api/v1/pods?watch=true&resourceVersion=0 HTTP/1.1\r\nHost: x\r\n\r\n")

        def reader():
            while True:
                b = s.recv(1 << 20)
                if not b:
                    return
                got.extend(b)

        threading.Thread(target=reader, daemon=True).start()
        pods = [json.dumps(pu.make_pod(f"c{i}", [("main", 10)], namespace="k")) for i in range(300)]
        assert srv.create_pods(pods) == [201] * 300
        code, body = srv.call("GET", "/api/v1/namespaces/k/pods")
        assert code == 200 and len(json.loads(body)["items"]) == 300
        assert srv.delete_pods([("k", f"c{i}") for i in range(300)]) == 300
        import time

        end = time.time() + 5
        while got.count(b'"type":"DELETED"') < 300 and time.time() < end:
            time.sleep(0.02)
        assert got.count(b'"type":"ADDED"') == 300 and got.count(b'"type":"DELETED"') == 300
        rvs = [int(x) for x in __import__("re").findall(rb'"resourceVersion":"(\d+)"', bytes(got))]
        assert rvs == sorted(rvs)
        assert json.loads(srv.stats())["pods"] == 0
    finally:
        s.close()
        srv.stop()


def test_native_spinning_io_threads_still_answer_and_stop():
    """set_spin (bench --apiserver-spin-us, a diagnostic): IO threads poll for a window after
    their last event instead of sleeping; requests over HTTP are answered, timeouts and watch
    deadlines still fire, and stop() returns while they spin."""
    import time

    srv = N.ApiServer("127.0.0.1", 0, 2, 1000)
    srv.set_spin(0.05)
    try:
        async def main():
            api = KubeClient(KubeConfig(server=f"http://127.0.0.1:{srv.port}"))
            try:
                for i in range(20):
                    await api.create_pod(pu.make_pod(f"s{i}", [("main", 10)], namespace="s"))
                items, rv = await api.list_pods()
                assert len(items) == 20
                t0 = asyncio.get_running_loop().time()
                async for _ in api.watch("pods", rv, timeout_s=1):
                    pass
                assert 0.8 < asyncio.get_running_loop().time() - t0 < 3.0
            finally:
                await api.close()

        asyncio.run(main())
    finally:
        t0 = time.perf_counter()
        srv.stop()
        assert time.perf_counter() - t0 < 2.0


def test_slim_pod_decoding_keeps_what_the_controllers_read():
    """decode_pod_watch (the pod informer's native decoder) drops everything but identity,
    labels, nano-gpu/* annotations and resources, nodeName and phase; every podutil reading
    the controllers do gives the same answer on the slim object as on the full one."""
    from hypothesis import given, settings, strategies as st

    @settings(max_examples=60, deadline=None)
    @given(st.lists(st.tuples(st.integers(0, 300), st.integers(0, 1 << 20)), min_size=1, max_size=6),
           st.booleans(), st.sampled_from(["Pending", "Running", "Succeeded", "Failed"]), st.booleans())
    def check(conts, assumed, phase, deleting):
        pod = pu.make_pod("p", [(f"c{i}", p, m) for i, (p, m) in enumerate(conts)], namespace="x")
        pod["metadata"]["annotations"]["other/huge"] = "y" * 500
        pod["spec"]["containers"][0]["env"] = [{"name": "A", "value": "1"}]
        pod["spec"]["nodeName"] = "n1"
        pod["status"]["phase"] = phase
        if assumed:
            pod["metadata"]["annotations"]["nano-gpu/assume"] = "true"
            for i in range(len(conts)):
                pod["metadata"]["annotations"][f"nano-gpu/container-c{i}"] = str(i % 8)
        if deleting:
            pod["metadata"]["deletionTimestamp"] = "2026-01-01T00:00:00Z"
        line = json.dumps({"type": "MODIFIED", "object": pod}).encode() + b"\n"
        (ev,) = N.decode_pod_watch(line)
        slim = ev["object"]
        assert ev["type"] == "MODIFIED" and "other/huge" not in slim["metadata"]["annotations"]
        for f in (pu.plan_from_pod, pu.pod_demand, pu.is_completed, pu.is_assumed, pu.node_name_of, pu.pod_uid,
                  pu.is_gpu_sharing):
            assert f(slim) == f(pod), f.__name__

    check()
    err = N.decode_pod_watch(b'{"type":"ERROR","object":{"kind":"Status","code":410,"message":"gone"}}\n')
    assert err[0]["object"]["code"] == 410


def test_watch_filter_does_the_controllers_ledger_only_work():
    """PodWatchFilter: pending pods and bound pods the ledger holds never reach Python; a
    deletion of a pod Python never saw is released natively; a pod once handed to Python
    (foreign, completed) keeps going to Python so the informer's store stays current."""
    from nanogpu.state.cluster import ClusterState
    from nanogpu.topology.model import synthetic_mi355x

    st = ClusterState()
    st.register_node(pu.make_node("n0", 8, synthetic_mi355x(8).to_json()))
    nid = st.node_ids(["n0"])[0]
    known = pu.make_pod("known", [("main", 20)])
    done = pu.make_pod("done", [("main", 20)])
    for p in (known, done):
        assert st.ledger.reserve(nid, pu.pod_uid(p), [(20, 0)], st.options)[0] == N.OK

    def ev(etype, pod, node="", phase="Running", rv="1"):
        p = json.loads(json.dumps(pod))
        p["metadata"]["resourceVersion"] = rv
        if node:
            p["spec"]["nodeName"] = node
        p["status"]["phase"] = phase
        return json.dumps({"type": etype, "object": p}).encode() + b"\n"

    pending = pu.make_pod("pending", [("main", 10)])
    foreign = pu.make_pod("foreign", [("main", 10)])
    f = N.PodWatchFilter(st.ledger)
    data = (ev("ADDED", pending, rv="10") + ev("MODIFIED", known, "n0", rv="11") +
            ev("MODIFIED", foreign, "n0", rv="12") + ev("MODIFIED", done, "n0", "Succeeded", rv="13") +
            ev("DELETED", known, "n0", rv="14") + ev("MODIFIED", foreign, "n0", rv="15") +
            ev("DELETED", pending, rv="16"))
    out = f.decode(data)
    got = [(e["type"], e["object"]["metadata"].get("name"), e["object"]["metadata"]["resourceVersion"]) for e in out]
    assert got == [("MODIFIED", "foreign", "12"), ("MODIFIED", "done", "13"), ("MODIFIED", "foreign", "15"),
                   ("BOOKMARK", None, "16")]
    assert st.ledger.lookup(pu.pod_uid(known)) is None             # released natively
    assert st.ledger.lookup(pu.pod_uid(done)) is not None          # Python's to release (completed)
    assert f.released == 1 and f.dropped == 4 and f.forwarded == 2
    out = f.decode(ev("DELETED", done, "n0", "Succeeded", rv="17") + ev("DELETED", foreign, "n0", rv="18"))
    assert [e["type"] for e in out] == ["DELETED", "DELETED"] and f.forwarded == 0
    f.reset(["default/x"])
    assert f.forwarded == 1
    assert [e["type"] for e in N.decode_pod_watch(data)] == ["ADDED", "MODIFIED", "MODIFIED", "MODIFIED", "DELETED",
                                                            "MODIFIED", "DELETED"]


def test_watch_filter_shallow_parse_skips_deep_fields_exactly():
    """The filter parses events only down to metadata's fields; deeper objects are skipped
    as text. Tricky text in skipped parts (escaped quotes, brackets inside strings, nested
    arrays) must neither end a skip early nor hide a malformed event; a kept event still
    carries its deep fields (labels, container limits) to Python."""
    from nanogpu.state.cluster import ClusterState
    from nanogpu.topology.model import synthetic_mi355x

    st = ClusterState()
    st.register_node(pu.make_node("n0", 8, synthetic_mi355x(8).to_json()))
    tricky = {"a": 'x"}]{[\\', "b": "\\u005d]", "nested": "[[{}]]"}
    pending = pu.make_pod("pending", [("main", 10)])
    pending["metadata"]["labels"] = dict(tricky)
    pending["spec"]["extra"] = [[1, [2, {"k": "}"}]], {"q": ["]"]}]
    kept = pu.make_pod("kept", [("main", 30)])
    kept["metadata"]["labels"] = dict(tricky)
    kept["spec"]["nodeName"] = "n0"
    kept["status"]["phase"] = "Running"
    f = N.PodWatchFilter(st.ledger)
    data = b"".join(json.dumps({"type": t, "object": p}).encode() + b"\n"
                    for t, p in (("ADDED", pending), ("MODIFIED", kept)))
    out = f.decode(data)
    assert [(e["type"], e["object"]["metadata"]["name"]) for e in out] == [("MODIFIED", "kept")]
    assert out[0]["object"]["metadata"]["labels"] == tricky
    assert out[0]["object"]["spec"]["containers"][0]["resources"]["limits"] == kept["spec"]["containers"][0]["resources"]["limits"]
    assert f.dropped == 1
    # a skipped part is checked for structure only (strings, bracket balance): a broken one
    # still fails the event
    unbalanced = json.dumps({"type": "ADDED", "object": pending}).replace('"labels": {', '"labels": {[').encode() + b"\n"
    with pytest.raises(ValueError):
        f.decode(unbalanced)
    unterminated = b'{"type":"ADDED","object":{"metadata":{"labels":{"a":"x\\"}}}}\n'
    with pytest.raises(ValueError):
        f.decode(unterminated)


def test_shallow_skip_agrees_with_the_full_parser_at_every_alignment():
    """The shallow parser skips deep containers sixteen bytes at a time (json.cpp
    skip_container): quotes, escapes, brackets and control characters inside skipped text
    must be seen wherever they fall in a 16-byte block. Random label text around those bytes,
    at every offset: an event the filter keeps decodes exactly as the full parser decodes it,
    and a corrupted one fails in both."""
    import random

    from nanogpu.state.cluster import ClusterState
    from nanogpu.topology.model import synthetic_mi355x

    st = ClusterState()
    st.register_node(pu.make_node("n0", 8, synthetic_mi355x(8).to_json()))
    rnd = random.Random(7)
    alphabet = ['"', "\\", "[", "]", "{", "}", "a", "b", " ", ",", ":", "é", "\t", "\n"]
    for i in range(400):
        pod = pu.make_pod(f"p{i}", [("main", 10)])
        pod["spec"]["nodeName"] = "n0"              # foreign bound pod: the filter keeps it
        pod["metadata"]["labels"] = {f"k{j}": "x" * rnd.randrange(0, 17) + "".join(
            rnd.choice(alphabet) for _ in range(rnd.randrange(0, 6))) for j in range(rnd.randrange(1, 4))}
        pod["spec"]["extra"] = [["y" * rnd.randrange(0, 33), {"z": "[" * rnd.randrange(0, 3)}]]
        line = json.dumps({"type": "ADDED", "object": pod}).encode() + b"\n"
        f = N.PodWatchFilter(st.ledger)
        assert f.decode(line) == N.decode_pod_watch(line)
        # corrupt one byte inside the skipped part: both parsers must agree on failing or not
        at = line.index(b'"extra"') + rnd.randrange(8, 30)
        bad = line[:at] + rnd.choice([b'"', b"]", b"}", b"\x01"]) + line[at + 1:]
        outcomes = []
        for decode in (N.PodWatchFilter(st.ledger).decode, N.decode_pod_watch):
            try:
                decode(bad)
                outcomes.append(True)
            except ValueError:
                outcomes.append(False)
        if not outcomes[1]:
            assert not outcomes[0], bad      # what the full parser rejects, the skip rejects


def test_native_json_strings_match_python_at_every_alignment():
    """json.cpp scans strings sixteen bytes at a time for the first quote, backslash or control
    character: escapes and multi-byte UTF-8 at every offset of a 16-byte block decode exactly
    as Python's json does, in plain and ensure_ascii encodings, and a raw control character
    inside a string is rejected wherever it falls."""
    import random

    rnd = random.Random(11)
    pieces = ['"', "\\", "/", "\n", "\t", "é", "€", "😀", "a", "b", " ", "\u0001"]
    for i in range(300):
        labels = {f"k{j}": "x" * rnd.randrange(0, 18) + "".join(rnd.choice(pieces) for _ in range(rnd.randrange(0, 12)))
                  + "y" * rnd.randrange(0, 18) for j in range(rnd.randrange(1, 4))}
        pod = pu.make_pod(f"p{i}", [("main", 10)])
        pod["metadata"]["labels"] = labels
        for ascii_only in (False, True):
            line = json.dumps({"type": "MODIFIED", "object": pod}, ensure_ascii=ascii_only).encode() + b"\n"
            got = N.decode_pod_watch(line)
            assert got[0]["object"]["metadata"]["labels"] == labels
    # a raw control byte inside a string, at each offset of a block
    for k in range(20):
        pod = pu.make_pod("c", [("main", 10)])
        pod["metadata"]["labels"] = {"k": "z" * k + "CTL" + "w" * 20}
        line = json.dumps({"type": "ADDED", "object": pod}).encode().replace(b"CTL", b"\x01") + b"\n"
        with pytest.raises(ValueError):
            N.decode_pod_watch(line)
