"""nano-gpu device plugin for MI355X: kubelet side of the scheduler's placement.

The reference scheduler writes `nano-gpu/container-<c>=<device>` on the pod and relies on
an external NVIDIA device plugin (nano-gpu-agent, reference README.md:9, 30-34) to turn it
into a device inside the container. This is the AMD equivalent:

* advertises `nano-gpu/gpu-percent` as 100 virtual IDs per schedulable device (an SPX
  GPU or a DPX/QPX/CPX partition), each carrying the device's NUMA node;
* on Allocate, kubelet hands over N arbitrary virtual IDs for one container; the plugin
  finds the container the extender placed on this node (assumed pod, not yet allocated,
  a container whose gpu-percent == N, oldest `nano-gpu/assume-time` first) and reads its
  device index from the annotation;
* answers with the device nodes (`/dev/kfd` + the partition's `/dev/dri/renderD*`), a
  spatial CU mask for fractional grants (`HSA_CU_MASK`, XCD-symmetric, see cumask.py),
  and the HBM budget (`NANO_GPU_MEMORY_MIB`, enforced in-process by nanogpu.agent.guest);
* records the CU grant as `nano-gpu/cu-mask-<c>` on the pod, so an agent restart
  rebuilds its CU map from the API server (the same checkpoint contract as the
  extender's, reference dealer.go:58-72);
* reconciles against kubelet's pod-resources API (`reconcile`): Allocate has no pod identity,
  so if kubelet admits two same-size containers out of bind order, each gets the other's
  device and grant. kubelet's List says which pod holds which IDs; the agent then moves the
  grants to the containers that really run with them, rewrites both pods' placement and
  CU-mask annotations (marked `nano-gpu/reconciled`, which the extender's pod controller
  re-accounts), and records a Warning Event on each pod.
"""
from __future__ import annotations

import asyncio
import logging
import os
import time
from dataclasses import dataclass

from .. import types as T
from ..k8s import podutil as pu
from ..topology.model import NodeTopology
from . import cumask
from . import dpapi as D

log = logging.getLogger(__name__)


def virtual_ids(topo: NodeTopology) -> list[tuple[str, int]]:
    """(ID, numa) for every percent unit of every schedulable device: "d<dev>-<k>"."""
    numa = {g.index: g.numa for g in topo.gpus}
    return [(f"d{i}-{k}", numa.get(d.gpu, -1)) for i, d in enumerate(topo.devices)
            for k in range(T.GPU_PERCENT_EACH_CARD)]


@dataclass
class Assignment:
    pod_key: str
    container: str
    devices: list[int]
    percent: int
    mib: int
    cus: int = 0          # CUs granted by the mask (0: whole devices, no mask)


class Matcher:
    """Finds which container an Allocate call is for (no pod identity in the request)."""

    def __init__(self, api, node_name: str):
        self.api = api
        self.node = node_name
        self.claimed: dict[tuple[str, str], float] = {}   # (pod uid, container) -> time

    async def candidates(self) -> list[dict]:
        # by node and annotation, not by the assume label: the placement annotations land
        # with the binding itself, the label in a PATCH that may arrive a moment later
        pods, _ = await self.api.list_pods(field_selector=f"{T.NODE_NAME_FIELD}={self.node}")
        return [p for p in pods if pu.is_assumed(p) and not pu.is_completed(p)]

    async def match(self, percent: int, claim: bool = True) -> tuple[dict, dict] | None:
        """The container kubelet is admitting: kubelet admits pods in the order they reach the
        node (bind order; HandlePodAdditions sorts one batch by creation time) and allocates
        a pod's containers in spec order. So: the first not-yet-allocated container asking
        for `percent` of the earliest-bound pod (assume time, then creation time, then name).
        An AllocateRequest carries no pod identity (device plugin v1beta1), so this order is
        the contract; `nanogpu.sim.kubelet.admission_order` is the same order."""
        best = None
        for p in await self.candidates():
            ann = pu.meta(p).get("annotations") or {}
            for c in pu.containers(p):
                name = c.get("name", "")
                if (pu.pod_uid(p), name) in self.claimed or T.ANNOTATION_CU_MASK_FMT.format(name) in ann:
                    continue
                if pu.container_percent(c) != percent or pu.container_assignment(p, name) is None:
                    continue
                key = admission_key(p)
                if best is None or key < best[0]:
                    best = (key, p, c)
                break
        if best is None:
            return None
        if claim:
            self.claimed[(pu.pod_uid(best[1]), best[2].get("name", ""))] = time.time()
        return best[1], best[2]


def admission_key(pod: dict) -> tuple:
    """kubelet's admission order for pods bound to one node (see Matcher.match)."""
    m = pu.meta(pod)
    ann = m.get("annotations") or {}
    return (float(ann.get(T.ANNOTATION_ASSUME_TIME, "0") or 0), m.get("creationTimestamp") or "",
            m.get("namespace") or "", m.get("name") or "")


class NanoGpuPlugin:
    """DevicePlugin service implementation (grpc.aio generic handlers)."""

    def __init__(self, topo: NodeTopology, api, node_name: str, render_minors: list[int] | None = None,
                 dev_root: str = "/dev"):
        self.topo = topo
        self.api = api
        self.node = node_name
        self.matcher = Matcher(api, node_name)
        self.render = render_minors or [128 + 8 * i for i in range(len(topo.devices))]
        self.dev_root = dev_root
        self.cus = [cumask.DeviceCUs(d.cus, d.xcds) for d in topo.devices]
        self.health = [bool(d.healthy) for d in topo.devices]
        self._changed = asyncio.Event()
        # live grants by (pod uid, container): what the agent's /metrics reports per container
        self.grants: dict[tuple[str, str], Assignment] = {}
        self.id_mismatches = 0   # Allocate IDs on another device than the placement (see Allocate)
        self.swaps_fixed = 0     # containers whose grant was moved after a pod-resources check

    # ---------------------------------------------------------------- restart rebuild
    async def rebuild(self, pods: list[dict] | None = None) -> int:
        n = 0
        if pods is None:
            pods = await self.matcher.candidates()
        for p in pods:
            # terminating pods still hold their CUs: restore their grants too
            if pu.node_name_of(p) != self.node or not pu.is_assumed(p) or pu.is_terminated(p):
                continue
            ann = pu.meta(p).get("annotations") or {}
            for c in pu.containers(p):
                name = c.get("name", "")
                mask = ann.get(T.ANNOTATION_CU_MASK_FMT.format(name))
                idx = pu.container_assignment(p, name)
                if mask is None or not idx:
                    continue
                self.matcher.claimed[(pu.pod_uid(p), name)] = 0.0
                cus = 0
                if mask not in ("", "full") and 0 <= idx[0] < len(self.cus):
                    bits = cumask.parse_ranges(mask.split(":")[-1])
                    self.cus[idx[0]].restore(f"{pu.pod_uid(p)}/{name}", bits)
                    cus = len(bits)
                self.grants[(pu.pod_uid(p), name)] = Assignment(pu.pod_key(p), name, list(idx),
                                                                pu.container_percent(c), pu.container_mib(c), cus)
                n += 1
        return n

    def release_pod(self, uid: str) -> None:
        for d in self.cus:
            for owner in [o for o in d.used if o.startswith(uid + "/")]:
                d.release(owner)
        for k in [k for k in self.matcher.claimed if k[0] == uid]:
            del self.matcher.claimed[k]
        for k in [k for k in self.grants if k[0] == uid]:
            del self.grants[k]

    async def reconcile(self, listed: dict[tuple[str, str, str], list[str]]) -> list[tuple[str, str]]:
        """Checks the grants against kubelet's record of which container got which device IDs
        (pod-resources List: (namespace, pod, container) -> IDs of nano-gpu/gpu-percent).

        A container kubelet lists on other devices than the grant recorded for it ran with
        another container's Allocate answer: kubelet admitted same-size containers out of bind
        order, and the matcher gave each the other's placement. Each such container is paired
        with the mis-recorded grant of the same size whose devices it really holds; the grant
        (CU bits included) moves to it, both pods' annotations are rewritten to what runs, and
        a Warning Event says so. Returns the (pod uid, container) keys that moved."""
        uid_of = {a.pod_key: uid for (uid, _), a in self.grants.items()}
        actual: dict[tuple[str, str], list[int]] = {}
        for (ns, pod, cn), ids in listed.items():
            uid = uid_of.get(f"{ns}/{pod}")
            if uid is None or (uid, cn) not in self.grants:
                continue
            try:
                actual[(uid, cn)] = sorted({int(i[1:i.index("-")]) for i in ids})
            except ValueError:
                continue
        wrong = [(k, devs) for k, devs in actual.items() if devs != sorted(self.grants[k].devices)]
        if not wrong:
            return []
        pool = {k: self.grants[k] for k, _ in wrong}
        moves = []          # (container that runs it, grant it runs under)
        for k, devs in wrong:
            want = self.grants[k].percent
            src = next((g for g, a in pool.items() if sorted(a.devices) == devs and a.percent == want), None)
            if src is None:
                log.warning("reconcile: %s/%s holds devices %s, no matching grant", *k, devs)
                continue
            del pool[src]
            moves.append((k, src))
        old = dict(self.grants)
        bits = {}           # grant key -> (device, CU bits) before the moves
        for k, src in moves:
            a = old[src]
            if len(a.devices) == 1 and f"{src[0]}/{src[1]}" in self.cus[a.devices[0]].used:
                bits[src] = (a.devices[0], self.cus[a.devices[0]].bits(f"{src[0]}/{src[1]}"))
        for _, src in moves:
            if src in bits:
                self.cus[bits[src][0]].release(f"{src[0]}/{src[1]}")
        moved = []
        for k, src in moves:
            a = old[src]
            mine = old[k]
            self.grants[k] = Assignment(mine.pod_key, k[1], list(a.devices), a.percent, mine.mib, a.cus)
            mask_ann = "full"
            if src in bits:
                dev, b = bits[src]
                self.cus[dev].restore(f"{k[0]}/{k[1]}", b)
                mask_ann = cumask.hsa_cu_mask(0, b)
            ns, name = mine.pod_key.split("/", 1)
            placed = ",".join(map(str, mine.devices))
            runs = ",".join(map(str, a.devices))
            try:
                await self.api.patch_pod(ns, name, {"metadata": {"annotations": {
                    T.container_annotation(k[1]): runs, T.ANNOTATION_CU_MASK_FMT.format(k[1]): mask_ann,
                    T.ANNOTATION_RECONCILED: str(time.time())}}})
            except Exception as e:   # the grant map is right either way; the next pass retries
                log.warning("reconcile: annotating %s failed: %s", mine.pod_key, e)
            try:
                await self.api.create_event(ns, {"kind": "Pod", "namespace": ns, "name": name, "uid": k[0]},
                                            "NanoGpuAllocationSwapped",
                                            f"container {k[1]} runs on device {runs} (placed on {placed}): kubelet "
                                            f"admitted same-size containers out of bind order; placement and "
                                            f"CU-mask annotations now follow what runs", "Warning")
            except Exception as e:
                log.debug("reconcile: event for %s failed: %s", mine.pod_key, e)
            moved.append(k)
        self.swaps_fixed += len(moved)
        return moved

    def set_health(self, dev: int, healthy: bool) -> None:
        if self.health[dev] != healthy:
            self.health[dev] = healthy
            self._changed.set()

    # ---------------------------------------------------------------- gRPC methods
    async def GetDevicePluginOptions(self, request, context):
        return D.DevicePluginOptions(pre_start_required=False, get_preferred_allocation_available=True)

    def _device_list(self):
        resp = D.ListAndWatchResponse()
        for vid, numa in virtual_ids(self.topo):
            dev = int(vid[1:vid.index("-")])
            d = resp.devices.add(ID=vid, health=D.HEALTHY if self.health[dev] else D.UNHEALTHY)
            if numa >= 0:
                d.topology.nodes.add(ID=numa)
        return resp

    async def ListAndWatch(self, request, context):
        yield self._device_list()
        while True:
            await self._changed.wait()
            self._changed.clear()
            yield self._device_list()

    async def GetPreferredAllocation(self, request, context):
        """Prefers IDs of the device the container about to be admitted was placed on (the
        Matcher's next pick for this size, not yet claimed), else of one device: kubelet's
        own per-ID accounting then mirrors the real share, and Allocate can check that the
        IDs it is handed name the device it answers with (`id_mismatches`)."""
        resp = D.PreferredAllocationResponse()
        for cr in request.container_requests:
            by_dev: dict[str, list[str]] = {}
            for vid in cr.available_deviceIDs:
                by_dev.setdefault(vid.split("-")[0], []).append(vid)
            chosen = list(cr.must_include_deviceIDs)
            nxt = await self.matcher.match(cr.allocation_size, claim=False)
            idx = pu.container_assignment(nxt[0], nxt[1].get("name", "")) if nxt else None
            want = by_dev.get(f"d{idx[0]}") if idx and len(idx) == 1 and idx[0] >= 0 else None
            if want and len(want) >= cr.allocation_size - len(chosen):
                chosen += [i for i in want if i not in chosen][:cr.allocation_size - len(chosen)]
            for ids in sorted(by_dev.values(), key=len):
                if len(chosen) >= cr.allocation_size:
                    break
                if len(ids) >= cr.allocation_size - len(chosen):
                    chosen += [i for i in ids if i not in chosen][:cr.allocation_size - len(chosen)]
                    break
            if len(chosen) < cr.allocation_size:
                rest = [i for i in cr.available_deviceIDs if i not in chosen]
                chosen += rest[:cr.allocation_size - len(chosen)]
            resp.container_responses.add(deviceIDs=chosen)
        return resp

    async def PreStartContainer(self, request, context):
        return D.PreStartContainerResponse()

    async def Allocate(self, request, context):
        resp = D.AllocateResponse()
        for cr in request.container_requests:
            percent = len(cr.devices_ids)
            m = await self.matcher.match(percent)
            if m is None:
                msg = f"no assumed container with gpu-percent={percent} on node {self.node}"
                log.warning("Allocate: %s", msg)
                if context is not None:
                    await context.abort(_grpc_status("FAILED_PRECONDITION"), msg)
                raise RuntimeError(msg)
            pod, c = m
            idx = pu.container_assignment(pod, c.get("name", "")) or []
            got = {vid.split("-")[0] for vid in cr.devices_ids}
            if len(idx) == 1 and idx[0] >= 0 and got != {f"d{idx[0]}"}:
                # kubelet did not take our preferred IDs (or admitted out of order): the answer
                # still follows the placement; counted so an operator can see it happen
                self.id_mismatches += 1
                log.info("Allocate: IDs on %s for a container placed on device %d", sorted(got), idx[0])
            resp.container_responses.append(await self._container_response(pod, c, percent))
        return resp

    async def _container_response(self, pod: dict, c: dict, percent: int):
        name = c.get("name", "")
        devs = pu.container_assignment(pod, name) or []
        mib = pu.container_mib(c)
        r = D.ContainerAllocateResponse()
        r.devices.add(container_path="/dev/kfd", host_path=f"{self.dev_root}/kfd", permissions="rw")
        for d in devs:
            minor = self.render[d]
            r.devices.add(container_path=f"/dev/dri/renderD{minor}", host_path=f"{self.dev_root}/dri/renderD{minor}",
                          permissions="rw")
        r.envs["NANO_GPU_DEVICES"] = ",".join(map(str, devs))
        r.envs["NANO_GPU_PERCENT"] = str(percent)
        mask_ann = "full"
        cus = 0
        if percent < T.GPU_PERCENT_EACH_CARD and len(devs) == 1:
            bits = self.cus[devs[0]].grant(f"{pu.pod_uid(pod)}/{name}", percent)
            if bits is None:
                raise RuntimeError(f"device {devs[0]} has no free CUs for {percent}%")
            mask_ann = cumask.hsa_cu_mask(0, bits)   # the container sees its device as index 0
            r.envs["HSA_CU_MASK"] = mask_ann
            r.envs["NANO_GPU_CUS"] = str(len(bits))
            cus = len(bits)
        if mib:
            r.envs["NANO_GPU_MEMORY_MIB"] = str(mib)
            total = self.topo.devices[devs[0]].hbm_mib if devs else 0
            if total:
                r.envs["NANO_GPU_MEMORY_FRACTION"] = f"{min(1.0, mib / total):.6f}"
                if mib < total:
                    # the HIP runtime's own view (ROCclr): the device reports this share of its
                    # memory as its total (hipMemGetInfo, hipDeviceProp.totalGlobalMem) and
                    # refuses any single allocation above it, so programs that size themselves
                    # from the total fit the budget. Whole percents, rounded up: never below the
                    # grant; the exact budget is the allocator cap guest.apply sets. Measured on
                    # MI355X: the runtime does not cap the sum of allocations
                    # (profiles/gpu_calibration.md).
                    r.envs["GPU_MAX_HEAP_SIZE"] = str(min(100, -(-100 * mib // total)))
        r.annotations["nano-gpu/devices"] = r.envs["NANO_GPU_DEVICES"]
        ns, pname = pu.pod_ns_name(pod)
        try:
            await self.api.patch_pod(ns, pname, {"metadata": {"annotations": {
                T.ANNOTATION_CU_MASK_FMT.format(name): mask_ann}}})
        except Exception as e:  # the allocation stands; the annotation only speeds up rebuild
            log.warning("annotating %s/%s failed: %s", ns, pname, e)
        self.grants[(pu.pod_uid(pod), name)] = Assignment(pu.pod_key(pod), name, list(devs), percent, mib, cus)
        return r


def _grpc_status(name: str):
    import grpc

    return getattr(grpc.StatusCode, name)


# -------------------------------------------------------------------- serving / registration
async def serve(plugin: NanoGpuPlugin, plugin_dir: str = D.PLUGIN_DIR, socket_name: str = "nanogpu-percent.sock",
                kubelet_socket: str | None = None, resource: str = T.RESOURCE_GPU_PERCENT, register: bool = True):
    """Starts the plugin's gRPC server on a unix socket and registers with kubelet."""
    import grpc

    path = os.path.join(plugin_dir, socket_name)
    try:
        os.unlink(path)
    except FileNotFoundError:
        pass
    server = grpc.aio.server()
    server.add_generic_rpc_handlers((D.generic_handler("DevicePlugin", plugin),))
    server.add_insecure_port(f"unix://{path}")
    await server.start()
    if register:
        await register_with_kubelet(kubelet_socket or os.path.join(plugin_dir, "kubelet.sock"), socket_name, resource)
    return server, path


async def register_with_kubelet(kubelet_socket: str, endpoint: str, resource: str) -> None:
    import grpc

    async with grpc.aio.insecure_channel(f"unix://{kubelet_socket}") as ch:
        stub = D.Stub(ch, "Registration")
        await stub.Register(D.RegisterRequest(
            version=D.VERSION, endpoint=endpoint, resource_name=resource,
            options=D.DevicePluginOptions(pre_start_required=False, get_preferred_allocation_available=True)),
            timeout=10)
