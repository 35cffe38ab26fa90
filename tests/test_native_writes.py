"""Native bind writes (native/src/kubewriter.cpp): the front door's C++ threads do the
bind's PATCH + binding POST + ledger commit. Same contract as the Python path
(nanogpu/extender/verbs.py::Extender._write, the reference's Bind at dealer.go:155-203 with
D1/D2 fixed): transient 5xx retried, a failed binding rolls the reservation back, takes the
placement annotations off again and records a FailedBinding event; kube-scheduler gets
{"Error": ...}. Each test runs with the writer on and off and expects the same outcome."""
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


async def _stack(store, native):
    """native: "evented" / "threads" (the C++ writer in that mode) or False (Python writes)."""
    runner, port = await serve(store)
    rt = Runtime(Config(kube_api=f"http://127.0.0.1:{port}", port=0, host="127.0.0.1",
                        policy_config_path="/nonexistent", native_bind_writes=bool(native),
                        bind_writer_mode=native or "evented"))
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


@pytest.mark.parametrize("native", ["evented", "threads", False])
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


@pytest.mark.parametrize("native", ["evented", "threads", False])
def test_failed_binding_rolls_back_and_unannotates(native):
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


@pytest.mark.parametrize("native", ["evented", "threads", False])
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


@pytest.mark.parametrize("mode", ["evented", "threads"])
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


@pytest.mark.parametrize("mode", ["evented", "threads"])
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


@pytest.mark.parametrize("native", ["evented", "threads", False])
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
def test_pipelined_label_after_the_binding(faults):
    """The evented writer pipelines the label PATCH behind the binding on one connection and
    answers kube-scheduler when the binding lands. A label PATCH that fails (5xx), or never gets
    an answer because the server closed the connection after the binding's, is retried on the
    slow path: the bind stays a success and is never rolled back; a lasting label failure is
    counted, never turned into a failed bind."""
    async def main():
        store = FakeKubeStore(faults=Faults(**faults))
        store.add_node(pu.make_node("n0", 8, synthetic_mi355x(8).to_json()))
        runner, rt = await _stack(store, "evented")
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
