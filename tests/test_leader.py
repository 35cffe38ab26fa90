"""Active/standby replicas on a coordination.k8s.io Lease (nanogpu/k8s/lease.py).

The reference has one replica and no HA (deploy yaml:73). Two extender replicas share one
fake API server: exactly one holds the Lease and serves; the standby answers 503 (and is
not ready) while its pod controller keeps its ledger equal to the leader's binds; when the
leader stops, the standby takes over and schedules on a warm, correct ledger."""
import asyncio
import json
import socket

from nanogpu.app import Config, Runtime
from nanogpu.k8s import podutil as pu
from nanogpu.k8s.fake_apiserver import FakeKubeStore, InProcKube
from nanogpu.topology.model import synthetic_mi355x


def _http(port, method, path, body=b""):
    s = socket.create_connection(("127.0.0.1", port))
    s.sendall(f"{method} {path} HTTP/1.1\r\nHost: x\r\nConnection: close\r\nContent-Length: {len(body)}\r\n\r\n"
              .encode() + body)
    out = b""
    while True:
        b = s.recv(65536)
        if not b:
            break
        out += b
    s.close()
    head, _, rest = out.partition(b"\r\n\r\n")
    return int(head.split(b" ")[1]), rest


async def wait_for(pred, timeout=5.0):
    end = asyncio.get_running_loop().time() + timeout
    while asyncio.get_running_loop().time() < end:
        if pred():
            return True
        await asyncio.sleep(0.01)
    return pred()


def test_leader_election_failover_with_warm_standby():
    async def main():
        store = FakeKubeStore()
        store.add_node(pu.make_node("n0", 8, synthetic_mi355x(8).to_json()))
        kw = dict(port=0, host="127.0.0.1", policy_config_path="/nonexistent", leader_elect=True,
                  lease_duration_s=1.0, lease_renew_deadline_s=0.6, lease_retry_s=0.05)
        a = Runtime(Config(identity="a", **kw), api=InProcKube(store))
        b = Runtime(Config(identity="b", **kw), api=InProcKube(store))
        await a.start()
        await b.start()
        loop = asyncio.get_running_loop()
        try:
            assert await wait_for(lambda: a.elector.leader or b.elector.leader)
            await asyncio.sleep(0.2)
            assert a.elector.leader != b.elector.leader
            lead, stand = (a, b) if a.elector.leader else (b, a)
            pod = store.create_pod(pu.make_pod("p", [("c", 30)]))
            body = json.dumps({"Pod": pod, "NodeNames": ["n0"]}).encode()
            st, _ = await loop.run_in_executor(None, _http, stand.bound_port, "POST", "/scheduler/filter", body)
            assert st == 503
            st, _ = await loop.run_in_executor(None, _http, stand.bound_port, "GET", "/readyz")
            assert st == 503
            st, out = await loop.run_in_executor(None, _http, lead.bound_port, "POST", "/scheduler/filter", body)
            assert st == 200 and json.loads(out)["NodeNames"] == ["n0"]
            m = pu.meta(pod)
            bind = json.dumps({"PodName": "p", "PodNamespace": "default", "PodUID": m["uid"], "Node": "n0"}).encode()
            st, _ = await loop.run_in_executor(None, _http, lead.bound_port, "POST", "/scheduler/bind", bind)
            assert st == 200
            # the standby's ledger follows the leader's bind through its pod informer
            assert await wait_for(lambda: stand.state.status()["n0"]["GPUs"][0]["Percent"] == 70)
            await lead.stop()
            assert await wait_for(lambda: stand.elector.leader, timeout=5)
            st, _ = await loop.run_in_executor(None, _http, stand.bound_port, "GET", "/readyz")
            assert st == 200
            pod2 = store.create_pod(pu.make_pod("q", [("c", 70)]))
            body2 = json.dumps({"Pod": pod2, "NodeNames": ["n0"]}).encode()
            st, out = await loop.run_in_executor(None, _http, stand.bound_port, "POST", "/scheduler/priorities", body2)
            assert st == 200
            m2 = pu.meta(pod2)
            bind2 = json.dumps({"PodName": "q", "PodNamespace": "default", "PodUID": m2["uid"], "Node": "n0"}).encode()
            st, _ = await loop.run_in_executor(None, _http, stand.bound_port, "POST", "/scheduler/bind", bind2)
            assert st == 200
            ann = store.get_pod("default", "q")["metadata"]["annotations"]
            assert ann["nano-gpu/container-c"] == "0"       # binpack onto the warm device 0 (30 % used)
            lease = store.get_lease("kube-system", "nano-gpu-scheduler")
            assert lease["spec"]["holderIdentity"] == stand.cfg.identity
        finally:
            for rt in (a, b):
                try:
                    await rt.stop()
                except Exception:
                    pass

    asyncio.run(main())
