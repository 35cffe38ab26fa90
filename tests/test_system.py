"""System test: every component together over real sockets.

fake API server (HTTP)  <-  node agents (topology + device plugin, gRPC to a fake kubelet)
                        <-  extender (native front door, real REST client + watches)
                        <-  kube-scheduler stand-in (HTTP)
then the fake kubelets admit the bound pods through the device plugins. Checks the whole
chain: published MI355X topology -> placement -> annotations -> Allocate answers the same
device with disjoint XCD-symmetric CU masks -> delete releases both the extender's ledger
and the agent's CU grants."""
import asyncio
import os

from nanogpu import types as T
from nanogpu.agent import cumask
from nanogpu.agent.node import NodeAgent, discover
from nanogpu.app import Config, Runtime
from nanogpu.k8s import podutil as pu
from nanogpu.k8s.client import KubeClient, KubeConfig
from nanogpu.k8s.fake_apiserver import FakeKubeStore, InProcKube, serve
from nanogpu.sim.driver import FastExtenderClient, SchedulerDriver, node_capacities
from nanogpu.sim.kubelet import FakeKubelet, admission_order
from nanogpu.topology.fixtures import write_mi355x_sysfs


async def wait_for(pred, timeout=10.0):
    end = asyncio.get_running_loop().time() + timeout
    while asyncio.get_running_loop().time() < end:
        if pred():
            return True
        await asyncio.sleep(0.01)
    return pred()


def test_full_stack_agent_extender_kubelet(tmp_path):
    async def main():
        store = FakeKubeStore()
        runner, port = await serve(store)
        url = f"http://127.0.0.1:{port}"
        names = ["gpu-node-0", "gpu-node-1"]
        agents, kubelets, clients = [], [], []
        try:
            for i, n in enumerate(names):
                store.add_node({"apiVersion": "v1", "kind": "Node", "metadata": {"name": n, "labels": {},
                                                                                 "annotations": {}}, "status": {}})
                root = write_mi355x_sysfs(tmp_path / f"sys{i}", 8, "SPX")
                topo, host = discover(str(root), use_amdsmi=False)
                pdir = tmp_path / f"dp{i}"
                pdir.mkdir()
                api = KubeClient(KubeConfig(server=url))
                clients.append(api)
                kl = FakeKubelet(api, n, str(pdir))
                await kl.start()
                ag = NodeAgent(api, n, topo, host, device_plugin=True, plugin_dir=str(pdir), health_period_s=0)
                await ag.start()
                await asyncio.wait_for(kl.ready.wait(), 10)
                agents.append(ag)
                kubelets.append(kl)
            # what the agents + kubelets published
            for n in names:
                node = store.get_node(n)
                assert node["status"]["capacity"][T.RESOURCE_GPU_PERCENT] == "800"
                assert T.ANNOTATION_TOPOLOGY in node["metadata"]["annotations"]
                assert node["metadata"]["labels"]["amd.com/gpu.present"] == "true"
            rt = Runtime(Config(kube_api=url, port=0, host="127.0.0.1", policy_config_path="/nonexistent"))
            await rt.start()
            client = FastExtenderClient("127.0.0.1", rt.bound_port)
            try:
                assert await wait_for(lambda: all(n in rt.state.status() for n in names))
                pods = [pu.make_pod(f"job-{k}", [("main", 25, 16 * 1024)]) for k in range(6)] + \
                       [pu.make_pod("tp2", [("r0", 100), ("r1", 100)])]
                nodes_now = [store.get_node(n) for n in names]
                drv = SchedulerDriver(client, InProcKube(store), names, node_capacities(nodes_now))
                stats = await drv.run(pods)
                assert stats.scheduled == 7, stats.summary()
                # kubelet admits each bound pod on its node through the device plugin
                masks: dict[tuple[str, str], list[int]] = {}
                bound = [store.get_pod("default", pu.meta(p)["name"]) for p in pods]
                for cur in admission_order(bound):     # kubelet admits in bind order
                    node = pu.node_name_of(cur)
                    kl = kubelets[names.index(node)]
                    spec = await kl.admit(cur)
                    for c in pu.containers(cur):
                        dev = pu.container_assignment(cur, c["name"])
                        s = spec[c["name"]]
                        assert s["envs"]["NANO_GPU_DEVICES"] == ",".join(map(str, dev))
                        assert "/dev/kfd" in s["devices"]
                        if "HSA_CU_MASK" in s["envs"]:
                            bits = cumask.parse_ranges(s["envs"]["HSA_CU_MASK"].split(":")[1])
                            assert len(bits) == 64                      # 25 % of 256 CUs
                            masks.setdefault((node, dev[0]), []).extend(bits)
                for (node, dev), bits in masks.items():
                    assert len(bits) == len(set(bits)), (node, dev)    # co-located tenants disjoint
                # tear down: ledger and CU grants both released
                for p in pods:
                    store.delete_pod("default", pu.meta(p)["name"])
                assert await wait_for(lambda: all(g["Percent"] == 100 for n in names
                                                  for g in rt.state.status()[n]["GPUs"]))
                assert await wait_for(lambda: all(not d.used for ag in agents for d in ag.plugin.cus))
            finally:
                await client.close()
                await rt.stop()
        finally:
            for ag in agents:
                await ag.stop()
            for kl in kubelets:
                await kl.stop()
            for c in clients:
                await c.close()
            await runner.cleanup()

    asyncio.run(main())


def test_agent_re_registers_after_kubelet_restart(tmp_path):
    """kubelet restarts wipe the device-plugin directory and serve a new kubelet.sock: the
    agent notices, serves its socket again and re-registers, and the new kubelet sees the
    devices through ListAndWatch."""
    import os

    async def main():
        store = FakeKubeStore()
        runner, port = await serve(store)
        api = KubeClient(KubeConfig(server=f"http://127.0.0.1:{port}"))
        n = "gpu-node-r"
        store.add_node({"apiVersion": "v1", "kind": "Node", "metadata": {"name": n, "labels": {},
                                                                         "annotations": {}}, "status": {}})
        topo, host = discover(str(write_mi355x_sysfs(tmp_path / "sys", 8, "SPX")), use_amdsmi=False)
        pdir = tmp_path / "dp"
        pdir.mkdir()
        kl = FakeKubelet(api, n, str(pdir))
        await kl.start()
        ag = NodeAgent(api, n, topo, host, device_plugin=True, plugin_dir=str(pdir), health_period_s=0,
                       kubelet_check_s=0.05)
        kl2 = None
        try:
            await ag.start()
            await asyncio.wait_for(kl.ready.wait(), 10)
            assert ag.registrations == 1
            # kubelet restarts: stops, removes every socket in the directory, comes back
            await kl.stop()
            for f in os.listdir(pdir):
                os.unlink(pdir / f)
            kl2 = FakeKubelet(api, n, str(pdir))
            await kl2.start()
            await asyncio.wait_for(kl2.ready.wait(), 10)
            assert kl2.registered and kl2.registered[0][2] == T.RESOURCE_GPU_PERCENT
            assert len(kl2.devices) == 800 and ag.registrations == 2
            assert os.path.exists(ag.socket_path)
        finally:
            await ag.stop()
            if kl2 is not None:
                await kl2.stop()
            await api.close()
            await runner.cleanup()

    asyncio.run(main())
