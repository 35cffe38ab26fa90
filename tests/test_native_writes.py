"""Native bind writes (native/src/kubewriter.cpp): the front door's C++ threads do the
bind's PATCH + binding POST + ledger commit. Same contract as the Python path
(nanogpu/extender/verbs.py::Extender._write, the reference's Bind at dealer.go:155-203 with
D1/D2 fixed): transient 5xx retried, a failed binding rolls the reservation back and records a
FailedBinding event; kube-scheduler gets {"Error": ...}. The Binding carries the placement
annotations and the label PATCH is guarded by spec.nodeName, so a refused bind writes nothing
on the pod. Each test runs with the writer on and off and expects the same outcome."""
import asyncio
import json

import aiohttp
import pytest

from nanogpu import types as T
from nanogpu.app import Config, Runtime
from nanogpu.k8s import podutil as pu
from nanogpu.k8s.client import ApiError
from nanogpu.k8s.fake_apiserver import Faults, FakeKubeStore, serve
from nanogpu.topology.model import synthetic_mi355x


async def _stack(store, native, batch_labels=False):
    """native: "inline" / "evented" / "threads" (the C++ writer in that mode) or False (Python
    writes); batch_labels: the evented driver's batched label PATCHes instead of pipelined ones."""
    runner, port = await serve(store)
    rt = Runtime(Config(kube_api=f"http://127.0.0.1:{port}", port=0, host="127.0.0.1",
                        policy_config_path="/nonexistent", native_bind_writes=bool(native),
                        bind_writer_mode=native or "evented", batch_labels=batch_labels))
    await rt.start()
    return runner, rt


async def _schedule(base, pod, node):
    async with aiohttp.ClientSession() as s:
        args = {"Pod": pod, "NodeNames": [node]}
        async with s.post(f"{base}/scheduler/filter", json=args) as r:
            assert (await r.json())["NodeNames"] == [node]
        m = pu.meta(pod)
        async with s.post(f"{base}/scheduler/bind", json={"PodName": m["name"], "PodNamespace": m["namespace"],
                                                            "PodUID": m["uid"], "Node": node}) as r:
            return r.status, await r.json()


async def _metrics(base):
    async with aiohttp.ClientSession() as s:
        async with s.get(f"{base}/metrics") as r:
            return await r.text()


@pytest.mark.parametrize("native", ["inline", "evented", "frontdoor", "threads", False])
def test_bind_writes_retry_transient_errors(native):
    async def main():
        store = FakeKubeStore(faults=Faults(patch_error_rate=0.3, bind_error_rate=0.3, seed=11))
        store.add_node(pu.make_node("n0", 8, synthetic_mi355x(8).to_json()))
        runner, rt = await _stack(store, native)
        base = f"http://127.0.0.1:{rt.bound_port}"
        try:
            ok = 0
            for i in range(12):
                p = store.create_pod(pu.make_pod(f"p{i}", [("main", 10)]))
                status, res = await _schedule(base, p, "n0")
                ok += res["Error"] == ""
            assert ok >= 10                     # 3 retries through 30 % 5xx
            assert rt.state.ledger.n_pods == ok
            text = await _metrics(base)
            if native:
                assert 'nanogpu_native_binds_total{result="ok"} ' + str(ok) in text
                assert "nanogpu_native_api_retries_total" in text
            else:
                assert "nanogpu_native_binds_total" not in text
        finally:
            await rt.stop()
            await runner.cleanup()

    asyncio.run(main())


@pytest.mark.parametrize("native", ["inline", "evented", "frontdoor", "threads", False])
def test_failed_binding_rolls_back_and_writes_nothing(native):
    async def main():
        store = FakeKubeStore(faults=Faults(bind_error_rate=1.0))
        store.add_node(pu.make_node("n0", 8, synthetic_mi355x(8).to_json()))
        runner, rt = await _stack(store, native)
        base = f"http://127.0.0.1:{rt.bound_port}"
        try:
            p = store.create_pod(pu.make_pod("doomed", [("main", 40)]))
            status, res = await _schedule(base, p, "n0")
            assert status == 500 and "500" in res["Error"] and "injected binding failure" in res["Error"]
            assert rt.state.status()["n0"]["GPUs"][0]["Percent"] == 100      # D2: rolled back
            assert rt.state.ledger.lookup(pu.pod_uid(p)) is None

            def clean():
                ann = store.get_pod("default", "doomed")["metadata"].get("annotations") or {}
                return T.ANNOTATION_GPU_ASSUME not in ann and T.container_annotation("main") not in ann

            for _ in range(200):
                if clean() and any(e["reason"] == "FailedBinding" for e in store.events):
                    break
                await asyncio.sleep(0.01)
            assert clean()
            ev = next(e for e in store.events if e["reason"] == "FailedBinding")
            assert ev["involvedObject"]["name"] == "doomed" and ev["message"].startswith("nano-gpu bind failed: ")
        finally:
            await rt.stop()
            await runner.cleanup()

    asyncio.run(main())


@pytest.mark.parametrize("native", ["inline", "evented", "frontdoor", "threads", False])
def test_binding_conflict_on_the_same_node_is_success(native):
    """A retried binding POST whose first attempt landed answers 409; the pod already sits on
    the requested node, so the bind succeeded."""
    async def main():
        store = FakeKubeStore()
        store.add_node(pu.make_node("n0", 8, synthetic_mi355x(8).to_json()))
        runner, rt = await _stack(store, native)
        base = f"http://127.0.0.1:{rt.bound_port}"
        try:
            p = store.create_pod(pu.make_pod("a", [("main", 30)]))
            orig = store.bind_pod

            def bind_then_conflict(ns, name, uid, node, annotations=None):
                orig(ns, name, uid, node, annotations)
                raise ApiError(409, "already assigned", "Conflict")

            store.bind_pod = bind_then_conflict
            status, res = await _schedule(base, p, "n0")
            assert status == 200 and res == {"Error": ""}
            assert store.get_pod("default", "a")["spec"]["nodeName"] == "n0"
            assert rt.state.status()["n0"]["GPUs"][0]["Percent"] == 70
            ann = store.get_pod("default", "a")["metadata"]["annotations"]
            assert ann[T.container_annotation("main")] == "0" and float(ann[T.ANNOTATION_ASSUME_TIME]) > 0
        finally:
            await rt.stop()
            await runner.cleanup()

    asyncio.run(main())


@pytest.mark.parametrize("mode", ["inline", "evented", "frontdoor", "threads"])
def test_native_writer_speaks_tls_with_a_bearer_token(tmp_path, mode):
    """https + token (how an in-cluster extender reaches kube-apiserver): a TLS proxy with a
    self-signed certificate in front of the fake API server checks the Authorization header.
    The certificate names the server the way kube-apiserver's does (CN kube-apiserver, the
    service IP as an IP SAN), so the writer must verify the IP against the IP SANs."""
    import shutil
    import ssl
    import subprocess

    if shutil.which("openssl") is None:
        pytest.skip("openssl CLI not available")
    key, crt = tmp_path / "k.pem", tmp_path / "c.pem"
    subprocess.run(["openssl", "req", "-x509", "-newkey", "rsa:2048", "-nodes", "-keyout", str(key), "-out", str(crt),
                    "-days", "1", "-subj", "/CN=kube-apiserver",
                    "-addext", "subjectAltName=DNS:kubernetes.default.svc,IP:127.0.0.1"],
                   check=True, capture_output=True)
    tok = tmp_path / "token"
    tok.write_text("s3cret\n")

    async def main():
        from aiohttp import web

        from nanogpu.k8s.client import KubeConfig
        from nanogpu.k8s.fake_apiserver import make_app

        store = FakeKubeStore()
        store.add_node(pu.make_node("n0", 8, synthetic_mi355x(8).to_json()))
        seen = []

        @web.middleware
        async def auth(request, handler):
            seen.append(request.headers.get("Authorization"))
            if request.headers.get("Authorization") != "Bearer s3cret":
                return web.json_response({"kind": "Status", "code": 401, "message": "Unauthorized"}, status=401)
            return await handler(request)

        app = make_app(store)
        app.middlewares.append(auth)
        runner = web.AppRunner(app)
        await runner.setup()
        sctx = ssl.create_default_context(ssl.Purpose.CLIENT_AUTH)
        sctx.load_cert_chain(str(crt), str(key))
        site = web.TCPSite(runner, "127.0.0.1", 0, ssl_context=sctx)
        await site.start()
        port = site._server.sockets[0].getsockname()[1]
        from nanogpu.k8s.client import KubeClient

        api = KubeClient(KubeConfig(server=f"https://127.0.0.1:{port}", ca_file=str(crt), token_file=str(tok),
                                    token="s3cret"))
        rt = Runtime(Config(port=0, host="127.0.0.1", policy_config_path="/nonexistent", bind_writer_mode=mode),
                     api=api)
        await rt.start()
        try:
            assert rt.native.fe.kube_writer_stats() is not None
            base = f"http://127.0.0.1:{rt.bound_port}"
            p = store.create_pod(pu.make_pod("t", [("main", 20)]))
            status, res = await _schedule(base, p, "n0")
            assert status == 200 and res == {"Error": ""}, res
            assert store.get_pod("default", "t")["spec"]["nodeName"] == "n0"
            assert rt.native.fe.kube_writer_stats()["ok"] == 1
            # the pod watch over the same TLS endpoint (the native watch thread): the deletion
            # of a pod the filter kept from Python is released in that thread
            assert api.native_watch and rt.pod_informer.watch_filter is not None
            uid = pu.pod_uid(p)
            store.delete_pod("default", "t")
            for _ in range(500):
                if rt.state.ledger.lookup(uid) is None:
                    break
                await asyncio.sleep(0.01)
            assert rt.state.ledger.lookup(uid) is None
            assert rt.pod_informer.watch_filter.released == 1
        finally:
            await rt.stop()
            await runner.cleanup()

    asyncio.run(main())


@pytest.mark.parametrize("mode", ["inline", "evented", "frontdoor", "threads"])
def test_stop_with_binds_in_flight_answers_every_bind_and_leaves_the_ledger_clean(mode):
    """A bind is in flight to a slow API server (0.3 s per answer) when the extender stops:
    the writer finishes what it holds within its grace period, kube-scheduler gets an answer
    for every bind, and no reservation is left behind (each pod is committed or rolled back)."""
    from nanogpu import _native as NN

    async def main():
        srv = NN.ApiServer("127.0.0.1", 0, 2, 4096)
        n0 = pu.make_node("n0", 8, synthetic_mi355x(8).to_json())
        st, _ = srv.call("POST", "/api/v1/nodes", json.dumps(n0))
        assert st in (200, 201)
        url = f"http://127.0.0.1:{srv.port}"
        rt = Runtime(Config(kube_api=url, port=0, host="127.0.0.1", policy_config_path="/nonexistent",
                            bind_writer_mode=mode))
        await rt.start()
        base = f"http://127.0.0.1:{rt.bound_port}"
        pods = []
        for i in range(6):
            p = pu.make_pod(f"s{i}", [("main", 10)])
            st, _ = srv.call("POST", "/api/v1/namespaces/default/pods", json.dumps(p))
            assert st == 201
            pods.append(p)
        srv.set_latency(0.3)
        answers = []

        async def bind(p):
            m = pu.meta(p)
            async with aiohttp.ClientSession() as s:
                try:
                    async with s.post(f"{base}/scheduler/bind", json={
                            "PodName": m["name"], "PodNamespace": "default", "PodUID": m["uid"], "Node": "n0"},
                            timeout=aiohttp.ClientTimeout(total=20)) as r:
                        answers.append((r.status, await r.json()))
                except Exception as e:   # noqa: BLE001
                    answers.append((0, {"Error": repr(e)}))

        tasks = [asyncio.ensure_future(bind(p)) for p in pods]
        await asyncio.sleep(0.15)              # the writes are out, their answers not back yet
        stopping = asyncio.ensure_future(rt.stop())
        await asyncio.gather(*tasks)
        await stopping
        try:
            assert len(answers) == len(pods)
            assert all(st in (200, 500) for st, _ in answers), answers
            led = rt.state.ledger
            for p in pods:
                rec = led.lookup(pu.pod_uid(p))
                assert rec is None or rec["state"] == "committed", rec   # no reservation left
            committed = sum(1 for p in pods if led.lookup(pu.pod_uid(p)) is not None)
            assert committed == sum(1 for st, a in answers if st == 200 and a["Error"] == "")
        finally:
            srv.stop()

    asyncio.run(main())


@pytest.mark.parametrize("native_writes", [True, False])
def test_bind_on_another_worker_process_stays_native_through_the_ledger_handoff(native_writes):
    """Two extender workers on one shared ledger (what `--workers N` runs, and the bench's
    ranks): kube-scheduler's filter reaches one worker and its bind, sent on another
    connection, the other. The bind worker never saw the pod, so it takes the pod the filter
    parsed from the ledger (Ledger::take_pod_info) and binds natively; a bind whose pod no
    filter published goes to the Python path, which reads the pod from the API server."""
    import os

    async def main():
        store = FakeKubeStore()
        store.add_node(pu.make_node("n0", 8, synthetic_mi355x(8).to_json()))
        runner, port = await serve(store)
        path = f"/dev/shm/nanogpu-test-handoff-{os.getpid()}"
        rts = []
        try:
            for w in range(2):
                rt = Runtime(Config(kube_api=f"http://127.0.0.1:{port}", port=0, host="127.0.0.1",
                                    policy_config_path="/nonexistent", ledger_path=path,
                                    native_bind_writes=native_writes), worker=w)
                await rt.start()
                rts.append(rt)
            a, b = (f"http://127.0.0.1:{rt.bound_port}" for rt in rts)
            assert rts[0].state.ledger.attached >= 2
            p = store.create_pod(pu.make_pod("h", [("main", 30, 4096)]))
            m = pu.meta(p)
            bind = {"PodName": "h", "PodNamespace": m["namespace"], "PodUID": m["uid"], "Node": "n0"}
            async with aiohttp.ClientSession() as s:
                async with s.post(f"{a}/scheduler/filter", json={"Pod": p, "NodeNames": ["n0"]}) as r:
                    assert (await r.json())["NodeNames"] == ["n0"]
                async with s.post(f"{b}/scheduler/bind", json=bind) as r:
                    assert (await r.json()) == {"Error": ""}
                fa, fb = rts[0].native.fe.stats(), rts[1].native.fe.stats()
                assert fa["pods_published"] == 1 and fb["bind_handoffs"] == 1
                if native_writes:
                    assert rts[1].native.fe.kube_writer_stats()["ok"] == 1  # the native writer bound it
                got = store.get_pod("default", "h")
                assert got["spec"]["nodeName"] == "n0"
                assert got["metadata"]["annotations"]["nano-gpu/container-main"]
                rec = rts[0].state.ledger.lookup(m["uid"])
                assert rec["state"] == "committed" and rec["demand"] == [(30, 4096)]
                # no filter published this one: the Python path binds it from the API object
                q = store.create_pod(pu.make_pod("q", [("main", 20)]))
                mq = pu.meta(q)
                async with s.post(f"{b}/scheduler/bind", json={**bind, "PodName": "q", "PodUID": mq["uid"]}) as r:
                    assert (await r.json()) == {"Error": ""}
                assert rts[1].native.fe.stats()["bind_handoffs"] == 1
                assert store.get_pod("default", "q")["spec"]["nodeName"] == "n0"
        finally:
            for rt in rts:
                await rt.stop()
            await runner.cleanup()
            try:
                os.unlink(path)
            except FileNotFoundError:
                pass

    asyncio.run(main())


@pytest.mark.parametrize("native", ["inline", "evented", "frontdoor", "threads", False])
def test_no_assume_label_binds_with_one_api_write(native):
    """`--no-assume-label`: the binding alone (it carries the placement annotations, which
    kube-apiserver sets with spec.nodeName) — one API write per bind instead of two, no label."""
    async def main():
        store = FakeKubeStore()
        store.add_node(pu.make_node("n0", 8, synthetic_mi355x(8).to_json()))
        runner, port = await serve(store)
        rt = Runtime(Config(kube_api=f"http://127.0.0.1:{port}", port=0, host="127.0.0.1",
                            policy_config_path="/nonexistent", native_bind_writes=bool(native),
                            bind_writer_mode=native or "evented", assume_label=False))
        await rt.start()
        base = f"http://127.0.0.1:{rt.bound_port}"
        try:
            patches0 = store.counts.get("patch_pod", 0)
            for i in range(3):
                p = store.create_pod(pu.make_pod(f"p{i}", [("main", 20)]))
                status, res = await _schedule(base, p, "n0")
                assert status == 200 and res == {"Error": ""}, res
                got = store.get_pod("default", f"p{i}")
                assert got["spec"]["nodeName"] == "n0"
                ann = got["metadata"]["annotations"]
                assert ann["nano-gpu/assume"] == "true" and ann["nano-gpu/container-main"]
                assert T.LABEL_GPU_ASSUME not in (got["metadata"].get("labels") or {})
                assert rt.state.ledger.lookup(pu.pod_uid(p))["state"] == "committed"
            assert store.counts.get("bind_pod", 0) == 3
            assert store.counts.get("patch_pod", 0) == patches0     # no label PATCH
        finally:
            await rt.stop()
            await runner.cleanup()

    asyncio.run(main())


@pytest.mark.parametrize("faults", [dict(patch_error_rate=1.0), dict(close_after_binding=True),
                                    dict(patch_error_rate=0.5, seed=3)])
@pytest.mark.parametrize("mode", ["inline", "evented", "frontdoor"])
@pytest.mark.parametrize("batch", [False, True])
def test_pipelined_label_after_the_binding(faults, mode, batch):
    """The evented writer pipelines the label PATCH behind the binding on one connection (or,
    batched, sends the label PATCHes of bound pods together after their bindings) and
    answers kube-scheduler when the binding lands. A label PATCH that fails (5xx), or never gets
    an answer because the server closed the connection after the binding's, is retried on the
    slow path: the bind stays a success and is never rolled back; a lasting label failure is
    counted, never turned into a failed bind."""
    async def main():
        store = FakeKubeStore(faults=Faults(**faults))
        store.add_node(pu.make_node("n0", 8, synthetic_mi355x(8).to_json()))
        runner, rt = await _stack(store, mode, batch)
        base = f"http://127.0.0.1:{rt.bound_port}"
        try:
            for i in range(6):
                p = store.create_pod(pu.make_pod(f"p{i}", [("main", 10)]))
                status, res = await _schedule(base, p, "n0")
                assert status == 200 and res == {"Error": ""}, res
                got = store.get_pod("default", f"p{i}")
                assert got["spec"]["nodeName"] == "n0"
                assert got["metadata"]["annotations"][T.container_annotation("main")]
                assert rt.state.ledger.lookup(pu.pod_uid(p))["state"] == "committed"
            assert rt.state.status()["n0"]["GPUs"][0]["Percent"] == 40
            labelled = lambda: sum((store.get_pod("default", f"p{i}")["metadata"].get("labels") or {})
                                   .get(T.LABEL_GPU_ASSUME) == "true" for i in range(6))
            for _ in range(300):   # the label lands after the answer, through the slow path's retry
                if labelled() == 6 or rt.native.fe.kube_writer_stats()["inflight"] == 0:
                    break
                await asyncio.sleep(0.01)
            text = await _metrics(base)
            assert 'nanogpu_native_binds_total{result="ok"} 6' in text
            failures = int(next(ln.split()[1] for ln in text.splitlines()
                                if ln.startswith("nanogpu_native_label_failures_total ")))
            if faults.get("patch_error_rate") == 1.0:
                assert labelled() == 0 and failures == 6
                assert store.events == []                           # no rollback, no FailedBinding
            else:   # a 50 % 5xx rate can outlast the retries: every label lands or is counted
                assert labelled() + failures == 6
        finally:
            await rt.stop()
            await runner.cleanup()

    asyncio.run(main())


class _NativeServer:
    """The native API server (native/src/apiserver.cpp) behind the same calls the tests make
    on FakeKubeStore."""

    def __init__(self):
        from nanogpu import _native as NN

        self.srv = NN.ApiServer("127.0.0.1", 0, 2, 4096)
        self.url = f"http://127.0.0.1:{self.srv.port}"

    def call(self, method, path, body=None):
        st, text = self.srv.call(method, path, json.dumps(body) if body is not None else "")
        return st, (json.loads(text) if text else None)

    def stats(self):
        return json.loads(self.srv.stats())


def _bound_elsewhere_pod(name):
    """A pod another scheduler bound to a node this extender does not manage, with that
    scheduler's placement annotations and label."""
    p = pu.make_pod(name, [("main", 40)])
    p["spec"]["nodeName"] = "other-node"
    p["metadata"]["annotations"] = {T.container_annotation("main"): "5", T.ANNOTATION_GPU_ASSUME: "true",
                                    T.ANNOTATION_ASSUME_TIME: "1700000000.000001"}
    p["metadata"]["labels"] = {T.LABEL_GPU_ASSUME: "true", "app": "x"}
    return p


@pytest.mark.parametrize("server", ["python", "native"])
@pytest.mark.parametrize("native", ["inline", "evented", "frontdoor", "threads", False])
def test_binding_refused_for_a_pod_bound_elsewhere_leaves_its_placement_alone(native, server):
    """The pod is already bound to another node (with that placement's annotations) when this
    extender binds it to n0: the binding is refused (409, the GET shows the other node), the
    ledger holds nothing for n0, and the pod's annotations and labels are byte-identical."""
    async def main():
        runner = ns = None
        if server == "python":
            store = FakeKubeStore()
            store.add_node(pu.make_node("n0", 8, synthetic_mi355x(8).to_json()))
            runner, port = await serve(store)
            url = f"http://127.0.0.1:{port}"
            p = store.create_pod(_bound_elsewhere_pod("taken"))
            get = lambda: store.get_pod("default", "taken")
        else:
            ns = _NativeServer()
            url = ns.url
            assert ns.call("POST", "/api/v1/nodes", pu.make_node("n0", 8, synthetic_mi355x(8).to_json()))[0] in (200, 201)
            st, p = ns.call("POST", "/api/v1/namespaces/default/pods", _bound_elsewhere_pod("taken"))
            assert st == 201
            get = lambda: ns.call("GET", "/api/v1/namespaces/default/pods/taken")[1]
        before = json.dumps(get()["metadata"].get("annotations"), sort_keys=True), \
            json.dumps(get()["metadata"].get("labels"), sort_keys=True)
        rt = Runtime(Config(kube_api=url, port=0, host="127.0.0.1", policy_config_path="/nonexistent",
                            native_bind_writes=bool(native), bind_writer_mode=native or "evented"))
        await rt.start()
        base = f"http://127.0.0.1:{rt.bound_port}"
        try:
            status, res = await _schedule(base, p, "n0")
            assert status == 500 and "409" in res["Error"], res
            assert rt.state.ledger.lookup(pu.pod_uid(p)) is None
            assert rt.state.status()["n0"]["GPUs"][0]["Percent"] == 100
            if native:   # the writer made the reservation, and rolled it back
                assert rt.native.fe.kube_writer_stats()["rollbacks"] == 1
            await asyncio.sleep(0.2)   # anything still in flight would have landed by now
            got = get()
            assert got["spec"]["nodeName"] == "other-node"
            after = json.dumps(got["metadata"].get("annotations"), sort_keys=True), \
                json.dumps(got["metadata"].get("labels"), sort_keys=True)
            assert after == before
        finally:
            await rt.stop()
            if runner is not None:
                await runner.cleanup()
            if ns is not None:
                ns.srv.stop()

    asyncio.run(main())


@pytest.mark.parametrize("server", ["python", "native"])
@pytest.mark.parametrize("native", ["inline", "evented", "frontdoor", "threads", False])
def test_binding_refused_for_a_deleted_pod_sends_no_cleanup_patch(native, server):
    """The pod is deleted between filter and bind: the binding answers 404, the reservation is
    rolled back, and no PATCH follows (the evented writer's guarded label PATCH, pipelined
    behind the binding, is the only one that may go out; it finds no pod)."""
    async def main():
        runner = ns = None
        if server == "python":
            store = FakeKubeStore()
            store.add_node(pu.make_node("n0", 8, synthetic_mi355x(8).to_json()))
            runner, port = await serve(store)
            url = f"http://127.0.0.1:{port}"
            p = store.create_pod(pu.make_pod("gone", [("main", 30)]))
            patches = lambda: store.counts.get("patch_pod", 0)
            delete = lambda: store.delete_pod("default", "gone")
        else:
            ns = _NativeServer()
            url = ns.url
            assert ns.call("POST", "/api/v1/nodes", pu.make_node("n0", 8, synthetic_mi355x(8).to_json()))[0] in (200, 201)
            st, p = ns.call("POST", "/api/v1/namespaces/default/pods", pu.make_pod("gone", [("main", 30)]))
            assert st == 201
            patches = lambda: ns.stats()["calls"]["patch_pod"]
            delete = lambda: ns.call("DELETE", "/api/v1/namespaces/default/pods/gone")
        rt = Runtime(Config(kube_api=url, port=0, host="127.0.0.1", policy_config_path="/nonexistent",
                            native_bind_writes=bool(native), bind_writer_mode=native or "evented"))
        await rt.start()
        base = f"http://127.0.0.1:{rt.bound_port}"
        try:
            async with aiohttp.ClientSession() as s:
                async with s.post(f"{base}/scheduler/filter", json={"Pod": p, "NodeNames": ["n0"]}) as r:
                    assert (await r.json())["NodeNames"] == ["n0"]
                delete()
                p0 = patches()
                m = pu.meta(p)
                async with s.post(f"{base}/scheduler/bind", json={"PodName": "gone", "PodNamespace": "default",
                                                                    "PodUID": m["uid"], "Node": "n0"}) as r:
                    status, res = r.status, await r.json()
            assert status == 500 and "404" in res["Error"], res
            assert rt.state.ledger.lookup(pu.pod_uid(p)) is None
            await asyncio.sleep(0.2)
            assert patches() - p0 <= (1 if native in ("evented", "inline", "frontdoor") else 0)
        finally:
            await rt.stop()
            if runner is not None:
                await runner.cleanup()
            if ns is not None:
                ns.srv.stop()

    asyncio.run(main())


@pytest.mark.parametrize("mode", ["inline", "evented", "frontdoor", "threads"])
def test_an_api_server_that_never_answers_times_the_bind_out(mode):
    """A half-open API server (accepts, reads, never answers nor resets): every bind still gets
    an answer (an error) within a few writer timeouts, the reservation is rolled back, and the
    evented writer counts the timeouts (its requests had no deadline)."""
    import socket
    import threading
    import time as _time

    lsock = socket.socket()
    lsock.bind(("127.0.0.1", 0))
    lsock.listen(64)
    held, stop = [], threading.Event()

    def accept():
        lsock.settimeout(0.1)
        while not stop.is_set():
            try:
                c, _ = lsock.accept()
                held.append(c)   # read nothing back, answer nothing
            except OSError:
                pass

    th = threading.Thread(target=accept, daemon=True)
    th.start()

    async def main():
        from nanogpu.k8s.fake_apiserver import InProcKube

        store = FakeKubeStore()
        store.add_node(pu.make_node("n0", 8, synthetic_mi355x(8).to_json()))
        rt = Runtime(Config(port=0, host="127.0.0.1", policy_config_path="/nonexistent", bind_writer_mode=mode,
                            api_write_timeout_s=0.5), api=InProcKube(store))
        await rt.start()
        base = f"http://127.0.0.1:{rt.bound_port}"
        from nanogpu.k8s.client import KubeConfig

        # the bind writes go to the silent server (the informers stay on the in-process store)
        assert rt.native.enable_native_writes(KubeConfig(server=f"http://127.0.0.1:{lsock.getsockname()[1]}"),
                                              2, 1, False, mode != "threads", True, 0.5, mode == "inline")
        try:
            pods = [store.create_pod(pu.make_pod(f"h{i}", [("main", 10)])) for i in range(3)]
            t0 = _time.monotonic()
            res = await asyncio.gather(*(_schedule(base, p, "n0") for p in pods))
            took = _time.monotonic() - t0
            assert all(st == 500 and r["Error"] for st, r in res), res
            assert took < 15, took
            for p in pods:
                assert rt.state.ledger.lookup(pu.pod_uid(p)) is None
            if mode != "threads":
                assert rt.native.fe.kube_writer_stats()["timeouts"] >= 1
        finally:
            await rt.stop()

    try:
        asyncio.run(main())
    finally:
        stop.set()
        th.join(2)
        for c in held:
            c.close()
        lsock.close()


@pytest.mark.parametrize("lazy", [False, True])
@pytest.mark.parametrize("mode", ["evented", "inline", "frontdoor"])
def test_many_concurrent_binds_with_label_patches_all_complete(mode, lazy):
    """Driven by the native kube-scheduler stand-in (binds back to back, many in flight) against
    the native API server, every bind is answered once, every pod is bound with its label
    (pipelined behind its binding on a connection the writer keeps), and the writer ends with
    nothing in flight."""
    from nanogpu import _native as NN
    from nanogpu.sim.driver import NativeSchedulerDriver, node_capacities

    async def main():
        srv = NN.ApiServer("127.0.0.1", 0, 2, 8192)
        nodes = []
        for i in range(8):
            st, body = srv.call("POST", "/api/v1/nodes", json.dumps(pu.make_node(f"n{i}", 8, synthetic_mi355x(8).to_json())))
            nodes.append(json.loads(body))
        rt = Runtime(Config(kube_api=f"http://127.0.0.1:{srv.port}", port=0, host="127.0.0.1",
                            policy_config_path="/nonexistent", bind_writer_mode=mode, lazy_label_answers=lazy))
        await rt.start()
        loop = asyncio.get_running_loop()
        try:
            for rnd in range(3):
                pods = []
                for i in range(400):
                    p = pu.make_pod(f"r{rnd}-c{i}", [("main", 5)])
                    st, body = srv.call("POST", "/api/v1/namespaces/default/pods", json.dumps(p))
                    assert st == 201
                    pods.append(json.loads(body))
                drv = NativeSchedulerDriver("127.0.0.1", rt.bound_port, [n["metadata"]["name"] for n in nodes],
                                            node_capacities(nodes), bind_threads=16)
                res = await asyncio.wait_for(loop.run_in_executor(None, drv.run, pods), 60)
                assert res.scheduled == len(pods) and res.failed == 0, (res.scheduled, res.failed)
                for _ in range(300):   # the last label answers: read within a few milliseconds
                    if rt.native.fe.kube_writer_stats()["inflight"] == 0:
                        break
                    await asyncio.sleep(0.01)
                assert rt.native.fe.kube_writer_stats()["inflight"] == 0
                for p in pods:
                    st, body = srv.call("GET", f"/api/v1/namespaces/default/pods/{pu.meta(p)['name']}", "")
                    got = json.loads(body)
                    assert got["spec"].get("nodeName") and got["metadata"]["labels"].get(T.GPU_ASSUME) == "true", got
                for p in pods:   # room for the next round
                    srv.call("DELETE", f"/api/v1/namespaces/default/pods/{pu.meta(p)['name']}", "")
                for _ in range(300):
                    if rt.state.ledger.n_pods == 0:
                        break
                    await asyncio.sleep(0.01)
        finally:
            await rt.stop()
            srv.stop()

    asyncio.run(main())
