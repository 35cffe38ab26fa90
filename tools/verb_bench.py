import sys, json, asyncio
sys.path.insert(0, __import__('os').path.dirname(__import__('os').path.dirname(__import__('os').path.abspath(__file__))))
from nanogpu.sim import benchlib
from nanogpu.app import Config, Runtime
from nanogpu.k8s import podutil as pu
from nanogpu.k8s.fake_apiserver import FakeKubeStore, InProcKube
from nanogpu.topology.model import synthetic_mi355x

async def scan():
    store = FakeKubeStore()
    topo = synthetic_mi355x(8, "SPX")
    nodes = [pu.make_node(f"mi355x-{i:03d}", 8, topo.to_json()) for i in range(64)]
    for n in nodes: store.add_node(n)
    rt = Runtime(Config(port=0, host="127.0.0.1", policy_config_path="/nonexistent", ledger_path=f"/dev/shm/vb3-{id(store)}", nominate=False), api=InProcKube(store))
    await rt.start()
    fe = rt.native.fe
    p = benchlib.burst(0, 1, 12, 0, 7)[0]
    for k in (1, 64):
        names = [f"mi355x-{i:03d}" for i in range(k)]
        body = json.dumps({"Pod": p, "Nodes": None, "NodeNames": names}, separators=(",", ":")).encode()
        tf = min(fe.time_verb(body, False, 3000)[1] for _ in range(15))
        tp = min(fe.time_verb(body, True, 3000)[1] for _ in range(15))
        print(f"k={k} filter {tf*1e6:.2f} us  prio {tp*1e6:.2f} us")
    await rt.stop()
asyncio.run(scan())
