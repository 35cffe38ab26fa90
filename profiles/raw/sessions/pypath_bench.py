"""CPU time of the extender's Python pod path per 1000 pods (create, bind_prepared, watch events,
delete + release) against the in-process API server, without sockets: min over 10 bursts."""
import sys, asyncio, time
sys.path.insert(0, __import__('os').path.dirname(__import__('os').path.dirname(__import__('os').path.abspath(__file__))))
import bench
from nanogpu.app import Config, Runtime
from nanogpu.k8s import podutil as pu
from nanogpu.k8s.fake_apiserver import FakeKubeStore, InProcKube
from nanogpu.topology.model import synthetic_mi355x
from nanogpu import _native as N

async def main():
    store = FakeKubeStore(history=8192)
    topo = synthetic_mi355x(8, "SPX")
    for i in range(64): store.add_node(pu.make_node(f"mi355x-{i:03d}", 8, topo.to_json()))
    rt = Runtime(Config(port=0, host="127.0.0.1", policy_config_path="/nonexistent", ledger_path=f"/dev/shm/bb-{id(store)}"), api=InProcKube(store))
    await rt.start()
    api = InProcKube(store); ext = rt.extender
    out = {"create": [], "bind": [], "events": [], "release": []}
    for step in range(12):
        pods = bench.burst(0, 1, 1000, step, 7)
        c0 = time.thread_time()
        for p in pods: await api.create_pod(p)
        await asyncio.sleep(0); await asyncio.sleep(0)
        c1 = time.thread_time()
        preps = []
        for j, p in enumerate(pods):
            node = f"mi355x-{j % 64:03d}"
            nid = rt.state.ledger.find_node(node)
            rc, plan = rt.state.ledger.reserve(nid, pu.pod_uid(p), pu.pod_demand(p), rt.state.options)
            preps.append({"rc": rc, "ns": pu.pod_ns_name(p)[0], "name": pu.pod_ns_name(p)[1], "uid": pu.pod_uid(p),
                          "node": node, "containers": ["main"], "plan": plan, "demand": list(pu.pod_demand(p))})
        c2 = time.thread_time()
        for pr in preps:
            co = ext.bind_prepared(pr)
            try:
                co.send(None)
            except StopIteration:
                pass
        c3 = time.thread_time()
        await asyncio.sleep(0); await asyncio.sleep(0)
        c4 = time.thread_time()
        for p in pods: store.delete_pod(*pu.pod_ns_name(p))
        await asyncio.sleep(0); await asyncio.sleep(0)
        c5 = time.thread_time()
        if step >= 2:
            out["create"].append(c1 - c0); out["bind"].append(c3 - c2); out["events"].append(c4 - c3); out["release"].append(c5 - c4)
    print({k: round(1e3 * min(v), 2) for k, v in out.items()}, "ms per 1000 pods (min of 10)")
    await rt.stop()
asyncio.run(main())
