"""A fake kubelet for system tests: the device-plugin side of a node, without a cluster.

It serves the kubelet `Registration` service on `<dir>/kubelet.sock`; when the node agent's
plugin registers, it connects back, reads ListAndWatch, and advertises the plugin's device
count as the node's `nano-gpu/gpu-percent` capacity (what kubelet does for extended
resources). `admit(pod)` then plays kubelet's part of starting a pod that the scheduler
bound to this node: per container, GetPreferredAllocation + Allocate with as many virtual
IDs as the container's gpu-percent limit, returning the container runtime spec (env,
device nodes) the plugin answered with.
"""
from __future__ import annotations

import asyncio
import os

from .. import types as T
from ..agent import dpapi as D
from ..k8s import podutil as pu


def admission_order(pods: list[dict]) -> list[dict]:
    """Pods bound to one node in the order a kubelet admits them: as they reach the node
    (bind order), ties by creation time. The device plugin's Matcher relies on it."""
    from ..agent.plugin import admission_key

    return sorted(pods, key=admission_key)


class FakeKubelet:
    def __init__(self, api, node_name: str, plugin_dir: str):
        self.api = api
        self.node = node_name
        self.dir = plugin_dir
        self.server = None
        self.registered: list[tuple[str, str, str]] = []
        self.devices: list[str] = []
        self.healthy: set[str] = set()
        self.allocated: set[str] = set()
        # what kubelet's pod-resources API lists: (namespace, pod, container) -> device IDs
        self.assigned: dict[tuple[str, str, str], list[str]] = {}
        self.resource = T.RESOURCE_GPU_PERCENT
        self._plugin_ch = None
        self._stub = None
        self._watch: asyncio.Task | None = None
        self.ready = asyncio.Event()

    async def start(self) -> None:
        import grpc

        from ..agent import podresources as PR

        self.server = grpc.aio.server()
        self.server.add_generic_rpc_handlers((D.generic_handler("Registration", self),
                                              PR.generic_handler(self)))
        self.server.add_insecure_port(f"unix://{os.path.join(self.dir, 'kubelet.sock')}")
        self.server.add_insecure_port(f"unix://{self.pod_resources_socket}")
        await self.server.start()

    @property
    def pod_resources_socket(self) -> str:
        return os.path.join(self.dir, "pod-resources.sock")

    async def List(self, request, context):
        """PodResourcesLister.List: the device IDs every admitted container holds."""
        from ..agent import podresources as PR

        resp = PR.ListPodResourcesResponse()
        pods: dict[tuple[str, str], object] = {}
        for (ns, name, cn), ids in self.assigned.items():
            p = pods.get((ns, name))
            if p is None:
                p = pods[(ns, name)] = resp.pod_resources.add(name=name, namespace=ns)
            c = p.containers.add(name=cn)
            c.devices.add(resource_name=self.resource, device_ids=ids)
        return resp

    async def Register(self, request, context):
        self.registered.append((request.version, request.endpoint, request.resource_name))
        self._watch = asyncio.ensure_future(self._connect(request.endpoint, request.resource_name))
        return D.Empty()

    async def _connect(self, endpoint: str, resource: str) -> None:
        import grpc

        self._plugin_ch = grpc.aio.insecure_channel(f"unix://{os.path.join(self.dir, endpoint)}")
        self._stub = D.Stub(self._plugin_ch, "DevicePlugin")
        async for resp in self._stub.ListAndWatch(D.Empty()):
            self.devices = [d.ID for d in resp.devices]
            self.healthy = {d.ID for d in resp.devices if d.health == D.HEALTHY}
            n = len(self.healthy)
            await self.api.patch_node_status(self.node, {"status": {"capacity": {resource: str(len(self.devices))},
                                                                    "allocatable": {resource: str(n)}}})
            self.ready.set()

    async def admit(self, pod: dict) -> dict[str, dict]:
        """Allocates every GPU container of a pod bound to this node; returns name -> spec."""
        out = {}
        for c in pu.containers(pod):
            pct = pu.container_percent(c)
            if pct <= 0:
                continue
            free = [i for i in self.devices if i in self.healthy and i not in self.allocated]
            pref = await self._stub.GetPreferredAllocation(D.PreferredAllocationRequest(container_requests=[
                D.ContainerPreferredAllocationRequest(available_deviceIDs=free, allocation_size=pct)]))
            ids = list(pref.container_responses[0].deviceIDs)
            resp = await self._stub.Allocate(D.AllocateRequest(container_requests=[
                D.ContainerAllocateRequest(devices_ids=ids)]))
            self.allocated.update(ids)
            ns, name = pu.pod_ns_name(pod)
            self.assigned[(ns, name, c.get("name", ""))] = ids
            r = resp.container_responses[0]
            out[c.get("name", "")] = {"ids": ids, "envs": dict(r.envs),
                                      "devices": [d.host_path for d in r.devices],
                                      "annotations": dict(r.annotations)}
        return out

    def release(self, ids: list[str]) -> None:
        self.allocated.difference_update(ids)

    async def stop(self) -> None:
        if self._watch is not None:
            self._watch.cancel()
        if self._plugin_ch is not None:
            await self._plugin_ch.close()
        if self.server is not None:
            await self.server.stop(None)


__all__ = ["FakeKubelet", "T"]
