"""The filtered pod watch read by a native thread (native/src/podwatch.cpp via
nanogpu/k8s/client.py::KubeClient._native_watch) against the aiohttp path it replaces: the same
events and resume point from a chunked stream cut at arbitrary points, the same errors (an HTTP
error answer, a transport failure, a bad line), a clean end, and a stop in mid-stream."""
from __future__ import annotations

import asyncio
import json
import random
import time

import pytest

from nanogpu import _native as N
from nanogpu.k8s import podutil as pu
from nanogpu.k8s.client import ApiError, KubeClient, KubeConfig
from nanogpu.state.cluster import ClusterState
from nanogpu.topology.model import synthetic_mi355x


def _state():
    st = ClusterState()
    st.register_node(pu.make_node("n0", 8, synthetic_mi355x(8).to_json()))
    return st


def _events(st, n=120, seed=3):
    """A mix the filter sorts every way: pending pods (dropped), bound pods the ledger holds
    (dropped), foreign bound pods (kept), deletions of both kinds, a bookmark."""
    rnd = random.Random(seed)
    nid = st.node_ids(["n0"])[0]
    lines, rv = [], 100
    held = []
    for i in range(n):
        rv += 1
        kind = rnd.choice(["pending", "held", "foreign", "delete", "bookmark"])
        p = pu.make_pod(f"p{i}", [("main", 5)])
        p["metadata"]["resourceVersion"] = str(rv)
        p["metadata"]["labels"] = {"app": "x" * rnd.randint(0, 300)}   # varied line lengths
        et = "ADDED"
        if kind == "held":
            assert st.ledger.reserve(nid, pu.pod_uid(p), [(5, 0)], st.options)[0] == N.OK
            p["spec"]["nodeName"] = "n0"
            held.append(p)
        elif kind == "foreign":
            p["spec"]["nodeName"] = "n0"
            p["status"]["phase"] = "Running"
        elif kind == "delete" and held:
            p = held.pop()
            p["metadata"]["resourceVersion"] = str(rv)
            et = "DELETED"
        elif kind == "bookmark":
            lines.append(json.dumps({"type": "BOOKMARK", "object": {"kind": "Pod", "metadata": {
                "resourceVersion": str(rv)}}}).encode())
            continue
        lines.append(json.dumps({"type": et, "object": p}).encode())
    rv += 1
    tail = pu.make_pod("tail", [("main", 5)])      # a dropped event last: the resume point
    tail["metadata"]["resourceVersion"] = str(rv)
    lines.append(json.dumps({"type": "ADDED", "object": tail}).encode())
    return b"\n".join(lines) + b"\n", str(rv)


async def _serve(handler, host="127.0.0.1", heads=None):
    async def conn(reader, writer):
        head = await reader.readuntil(b"\r\n\r\n")
        if heads is not None:
            heads.append(head.decode())
        try:
            await handler(writer)
        finally:
            writer.close()

    srv = await asyncio.start_server(conn, host, 0)
    return srv, srv.sockets[0].getsockname()[1]


def _chunked(data: bytes, seed=5, pause=0.0):
    async def handler(w):
        w.write(b"HTTP/1.1 200 OK\r\nContent-Type: application/json\r\nTransfer-Encoding: chunked\r\n\r\n")
        rnd = random.Random(seed)
        p = 0
        while p < len(data):
            n = rnd.randint(1, 900)
            part = data[p:p + n]
            p += n
            # chunk headers and bodies split across writes too
            frame = b"%x\r\n" % len(part) + part + b"\r\n"
            cut = rnd.randint(0, len(frame))
            w.write(frame[:cut])
            await w.drain()
            if pause:
                await asyncio.sleep(pause)
            w.write(frame[cut:])
            await w.drain()
        w.write(b"0\r\n\r\n")
        await w.drain()
    return handler


async def _collect(api, wf):
    out = []
    async for batch in api.watch_batches("pods", "100", slim=True, watch_filter=wf):
        out.extend(batch)
    return out


def _shape(events):
    kept = [(e["type"], e["object"]["metadata"].get("name"), e["object"]["metadata"].get("resourceVersion"))
            for e in events if e["type"] != "BOOKMARK" or e["object"].get("kind") == "Pod"]
    last = events[-1]["object"]["metadata"]["resourceVersion"] if events else None
    return kept, last


@pytest.mark.parametrize("pause", [0.0, 0.001])
def test_native_watch_matches_the_aiohttp_path(pause):
    async def main():
        shapes, counts = [], []
        for native in (False, True):
            st = _state()
            data, last_rv = _events(st)
            srv, port = await _serve(_chunked(data, pause=pause))
            api = KubeClient(KubeConfig(server=f"http://127.0.0.1:{port}"), native_watch=native)
            assert api.native_watch is native
            wf = N.PodWatchFilter(st.ledger)
            try:
                evs = await asyncio.wait_for(_collect(api, wf), 20)
            finally:
                await api.close()
                srv.close()
            kept, last = _shape(evs)
            assert last == last_rv                       # the resume point covers the dropped tail
            shapes.append(kept)
            counts.append((wf.dropped, wf.released, wf.forwarded))
        assert shapes[0] == shapes[1] and counts[0] == counts[1]
        assert counts[1][0] > 0 and counts[1][1] > 0 and shapes[1]

    asyncio.run(main())


def test_native_watch_errors_end_and_stop():
    async def answer(w, head, body=b""):
        w.write(head + b"Content-Length: %d\r\n\r\n" % len(body) + body)
        await w.drain()

    async def main():
        st = _state()
        wf = N.PodWatchFilter(st.ledger)

        async def gone(w):
            await answer(w, b"HTTP/1.1 410 Gone\r\nContent-Type: application/json\r\n",
                         b'{"kind":"Status","code":410,"message":"too old"}')

        async def bad_line(w):
            w.write(b"HTTP/1.1 200 OK\r\nTransfer-Encoding: chunked\r\n\r\n")
            w.write(b"6\r\n{nope\n\r\n")
            await w.drain()
            await asyncio.sleep(5)

        async def cut(w):
            w.write(b"HTTP/1.1 200 OK\r\nTransfer-Encoding: chunked\r\n\r\n" + b"40\r\n{\"type\":")
            await w.drain()

        async def unframed_end(w):   # no length, no chunking: the body ends with the connection
            p = pu.make_pod("f", [("main", 5)])
            p["spec"]["nodeName"] = "n0"
            p["metadata"]["resourceVersion"] = "7"
            w.write(b"HTTP/1.1 200 OK\r\nConnection: close\r\n\r\n" +
                    json.dumps({"type": "ADDED", "object": p}).encode() + b"\n")
            await w.drain()

        async def endless(w):
            w.write(b"HTTP/1.1 200 OK\r\nTransfer-Encoding: chunked\r\n\r\n")
            p = pu.make_pod("e", [("main", 5)])
            p["spec"]["nodeName"] = "n0"
            line = json.dumps({"type": "ADDED", "object": p}).encode() + b"\n"
            w.write(b"%x\r\n" % len(line) + line + b"\r\n")
            await w.drain()
            await asyncio.sleep(30)

        for handler, check in ((gone, "410"), (bad_line, "transport"), (cut, "transport"),
                               (unframed_end, "end"), (endless, "stop")):
            srv, port = await _serve(handler)
            api = KubeClient(KubeConfig(server=f"http://127.0.0.1:{port}"))
            try:
                if check == "410":
                    with pytest.raises(ApiError) as ei:
                        await asyncio.wait_for(_collect(api, wf), 10)
                    assert ei.value.status == 410 and "too old" in str(ei.value)
                elif check == "transport":
                    with pytest.raises(ConnectionError):
                        await asyncio.wait_for(_collect(api, wf), 10)
                elif check == "end":
                    evs = await asyncio.wait_for(_collect(api, wf), 10)
                    assert [(e["type"], e["object"]["metadata"]["name"]) for e in evs] == [("ADDED", "f")]
                else:
                    stream = api.watch_batches("pods", "1", slim=True, watch_filter=wf)
                    first = await asyncio.wait_for(stream.__anext__(), 10)
                    assert first[0]["object"]["metadata"]["name"] == "e"
                    t0 = time.monotonic()
                    await stream.aclose()                 # shuts the socket down, joins the thread
                    assert time.monotonic() - t0 < 2.0
            finally:
                await api.close()
                srv.close()

    asyncio.run(main())


def test_native_watch_over_ipv6_sends_a_bracketed_host_header():
    async def main():
        st = _state()
        data, last_rv = _events(st, n=20)
        heads = []
        try:
            srv, port = await _serve(_chunked(data), host="::1", heads=heads)
        except OSError:
            pytest.skip("no IPv6 loopback")
        api = KubeClient(KubeConfig(server=f"http://[::1]:{port}", token="t0k"))
        try:
            evs = await asyncio.wait_for(_collect(api, N.PodWatchFilter(st.ledger)), 20)
        finally:
            await api.close()
            srv.close()
        assert _shape(evs)[1] == last_rv
        (head,) = heads
        assert f"\r\nHost: [::1]:{port}\r\n" in head and "\r\nAuthorization: Bearer t0k\r\n" in head
        assert head.startswith("GET /api/v1/pods?watch=1&resourceVersion=100&")

    asyncio.run(main())


def test_a_held_pod_the_node_agent_reconciled_goes_on_to_the_controller():
    """A bound pod the ledger holds is dropped natively, unless the node agent rewrote its
    placement (`nano-gpu/reconciled` annotation, agent/plugin.py): then the controller must
    re-account it. The annotation can sit anywhere in a long event line."""
    st = _state()
    nid = st.node_ids(["n0"])[0]
    wf = N.PodWatchFilter(st.ledger)
    lines = []
    for i, reconciled in enumerate([False, True, False, True]):
        p = pu.make_pod(f"h{i}", [("main", 5)])
        assert st.ledger.reserve(nid, pu.pod_uid(p), [(5, 0)], st.options)[0] == N.OK
        p["spec"]["nodeName"] = "n0"
        p["metadata"]["resourceVersion"] = str(200 + i)
        p["metadata"]["labels"] = {"k\"q": "\"" * 200}            # many quotes before the annotations
        p["metadata"]["annotations"] = {"a": "nano-gpu/reconciled-not"}
        if reconciled:
            p["metadata"]["annotations"]["nano-gpu/reconciled"] = "1"
        lines.append(json.dumps({"type": "MODIFIED", "object": p}).encode())
    kept = [e["object"]["metadata"]["name"] for e in wf.decode(b"\n".join(lines) + b"\n") if e["type"] == "MODIFIED"]
    assert kept == ["h1", "h3"] and wf.dropped == 2
