"""Kubelet pod-resources API (k8s.io/kubelet/pkg/apis/podresources/v1) without protoc, built like
nanogpu.agent.dpapi: the List call that tells which pod and container kubelet gave each device
ID. The device-plugin API gives Allocate no pod identity (dpapi), so this is how the agent checks
afterwards that every container got the device its own pod was placed on.

  service PodResourcesLister { List(ListPodResourcesRequest) returns (ListPodResourcesResponse) }
"""
from __future__ import annotations

from . import dpapi

PACKAGE = "v1"
SOCKET = "/var/lib/kubelet/pod-resources/kubelet.sock"

_MESSAGES = {
    "ListPodResourcesRequest": [],
    "ListPodResourcesResponse": [("pod_resources", 1, ".PodResources", True)],
    "PodResources": [("name", 1, "string", False), ("namespace", 2, "string", False),
                     ("containers", 3, ".ContainerResources", True)],
    "ContainerResources": [("name", 1, "string", False), ("devices", 2, ".ContainerDevices", True),
                           ("cpu_ids", 3, "int64", True)],
    "ContainerDevices": [("resource_name", 1, "string", False), ("device_ids", 2, "string", True),
                         ("topology", 3, ".TopologyInfo", False)],
    "TopologyInfo": [("nodes", 1, ".NUMANode", True)],
    "NUMANode": [("ID", 1, "int64", False)],
}
_SERVICES = {"PodResourcesLister": [("List", "ListPodResourcesRequest", "ListPodResourcesResponse", False)]}

M = dpapi._build(PACKAGE, "nanogpu/podresources_v1.proto", _MESSAGES, _SERVICES)
globals().update(M)


def generic_handler(impl):
    return dpapi.generic_handler("PodResourcesLister", impl, PACKAGE, _SERVICES, M)


def stub(channel):
    return dpapi.Stub(channel, "PodResourcesLister", PACKAGE, _SERVICES, M)


async def list_devices(socket_path: str, resource: str) -> dict[tuple[str, str, str], list[str]]:
    """(namespace, pod, container) -> device IDs of `resource` kubelet allocated to it."""
    import grpc

    async with grpc.aio.insecure_channel(f"unix://{socket_path}") as ch:
        resp = await stub(ch).List(ListPodResourcesRequest(), timeout=5.0)
    out = {}
    for p in resp.pod_resources:
        for c in p.containers:
            ids = [i for d in c.devices if d.resource_name == resource for i in d.device_ids]
            if ids:
                out[(p.namespace, p.name, c.name)] = ids
    return out
