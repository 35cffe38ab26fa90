"""Node agent: discovers the node's MI355X devices, publishes them, runs the device plugin.

Reference counterpart: the node side is outside the reference repo (nano-gpu-agent,
reference README.md:9, 30-34); the scheduler only reads `capacity["nano-gpu/gpu-percent"]`
(reference pkg/utils/node.go:8-14). This agent publishes, per node:
  * annotation `nano-gpu/topology`: devices (GPU or partition), CUs, XCDs, HBM MiB, NUMA,
    xGMI link matrix, partition modes and optional probe calibration (topology.model);
  * label `amd.com/gpu.present=true` (the load-aware poller's node selector);
  * status capacity/allocatable `nano-gpu/gpu-memory` (HBM MiB) and, without the device
    plugin (`--advertise status`), `nano-gpu/gpu-percent` = 100 x devices;
and serves the kubelet device plugin (plugin.py) for `nano-gpu/gpu-percent`.
"""
from __future__ import annotations

import asyncio
import json
import logging
import os

from .. import types as T
from ..k8s import podutil as pu
from ..topology.model import NodeTopology, from_host_json

log = logging.getLogger(__name__)


def discover(sysfs_root: str = "", use_amdsmi: bool = True) -> tuple[NodeTopology, dict]:
    from ..native import core

    host = json.loads(core().discover_topology(sysfs_root, use_amdsmi))
    return from_host_json(host), host


def calibrate(topo: NodeTopology, device: int = 0, host: dict | None = None, busy_s: float = 3.0) -> dict:
    """Measures what the annotation cannot read from sysfs, on the real devices (HIP probe):
    the HBM copy rate, and each GPU's own mem_busy_percent scale (GpuSpec.hbm_busy_cal) under
    the probe's stream at 25 % and 100 % of its CUs, which the extender's poller reads HBM
    activity through (telemetry.store.normalize_hbm_activity)."""
    from ..native import probe
    from ..probe.calibrate import hbm_bandwidth, hbm_busy_calibration, local_gpu_facts, mem_busy_files

    out: dict = {}
    facts = local_gpu_facts(device)
    props = facts.get("props") or {}
    if props:
        out["gcn_arch"] = props.get("gcn_arch")
        out["hbm_copy_gbs"] = round(hbm_bandwidth(device, 1 << 30, 10), 1)
        P = probe()
        h = host if host is not None else facts.get("host") or {}
        files = mem_busy_files(h)
        by_index = {g.index: g for g in topo.gpus}
        cals, seen = {}, set()
        # HIP ordinal k is the k-th device the reader lists (KFD order). Whole GPUs (SPX) only:
        # the probe's CU masks assume the full chip
        for k, hg in enumerate((h.get("gpus") or [])[:P.device_count()]):
            parent = int(hg.get("parent", k))
            g = by_index.get(parent)
            if g is None or parent in seen or (hg.get("compute_partition") or "SPX").upper() != "SPX":
                continue
            seen.add(parent)
            try:
                g.hbm_busy_cal = hbm_busy_calibration(P, k, files.get(parent), seconds=busy_s)
            except Exception:   # a probe failure leaves that GPU on the reference scale
                log.exception("mem_busy calibration of GPU %d failed", parent)
                g.hbm_busy_cal = []
            if g.hbm_busy_cal:
                cals[parent] = g.hbm_busy_cal
        out["hbm_busy_cal"] = cals
    topo.calibration.update(out)
    return out


def gpu_selftest(P, device: int) -> bool:
    """Active check of one HIP device with the probe's kernels: a bit-exact 16 MiB HBM copy
    and one bf16 MFMA tile (32x32x16, small integers, so the fp32 result is exact) against
    a host reference. A device that loads its driver and shows in sysfs can still compute
    wrong or fault; the agent then reports it Unhealthy (kubelet) and unschedulable (the
    extender). Runs on the calling thread (HIP's current device)."""
    try:
        if not P.copy_check(device, 1 << 22):
            return False
        a = [float((i * 7) % 7 - 3) for i in range(32 * 16)]
        b = [float((i * 5) % 5 - 2) for i in range(16 * 32)]
        c = P.gemm_tile(a, b)                  # on `device`: copy_check made it current
        for r in range(32):
            row = a[r * 16:(r + 1) * 16]
            for col in range(32):
                if c[r * 32 + col] != sum(row[k] * b[k * 32 + col] for k in range(16)):
                    return False
        return True
    except Exception:                          # a HIP error is a failed device
        log.exception("self-test of device %d raised", device)
        return False


def node_patch(topo: NodeTopology) -> dict:
    labels = {T.AMD_GPU_NODE_LABEL[0]: T.AMD_GPU_NODE_LABEL[1]}
    if topo.gpus:
        labels["nano-gpu/compute-partition"] = topo.gpus[0].compute_partition or "SPX"
    return {"metadata": {"annotations": {T.ANNOTATION_TOPOLOGY: topo.to_json()}, "labels": labels}}


def status_patch(topo: NodeTopology, advertise_percent: bool) -> dict:
    res = {T.RESOURCE_GPU_MEMORY: str(topo.hbm_capacity_mib())}
    if advertise_percent:
        res[T.RESOURCE_GPU_PERCENT] = str(T.GPU_PERCENT_EACH_CARD * len(topo.devices))
    return {"status": {"capacity": dict(res), "allocatable": dict(res)}}


async def publish(api, node_name: str, topo: NodeTopology, advertise_percent: bool) -> None:
    await api.patch_node(node_name, node_patch(topo))
    await api.patch_node_status(node_name, status_patch(topo, advertise_percent))


class NodeAgent:
    def __init__(self, api, node_name: str, topo: NodeTopology, host: dict | None = None,
                 device_plugin: bool = True, plugin_dir: str = "", health_period_s: float = 10.0,
                 sysfs_root: str = "", kubelet_check_s: float = 1.0, pod_resources_socket: str | None = None,
                 reconcile_period_s: float = 5.0):
        self.api = api
        self.node = node_name
        self.topo = topo
        self.host = host or {}
        self.device_plugin = device_plugin
        self.plugin_dir = plugin_dir
        self.health_period_s = health_period_s
        self.sysfs_root = sysfs_root
        self.kubelet_check_s = kubelet_check_s
        self.selftest_failed: set[int] = set()   # devices whose active self-test failed
        # kubelet's pod-resources API: which container got which device IDs (plugin.reconcile)
        from .podresources import SOCKET as _PR_SOCKET

        self.pod_resources_socket = pod_resources_socket if pod_resources_socket is not None else _PR_SOCKET
        self.reconcile_period_s = reconcile_period_s
        self.registrations = 0
        self._register = True
        self.plugin = None
        self.server = None
        self.socket_path = ""
        self.informer = None
        self.tasks: list[asyncio.Task] = []

    def render_minors(self) -> list[int]:
        gpus = self.host.get("gpus") or []
        if len(gpus) == len(self.topo.devices):
            return [int(g.get("render_minor", 0)) for g in gpus]
        return [128 + 8 * i for i in range(len(self.topo.devices))]

    async def start(self, register: bool = True) -> None:
        from ..k8s.informer import Informer
        from .plugin import NanoGpuPlugin

        await publish(self.api, self.node, self.topo, advertise_percent=not self.device_plugin)
        if not self.device_plugin:
            return
        self.plugin = NanoGpuPlugin(self.topo, self.api, self.node, self.render_minors())
        # pods on this node: CU grants are rebuilt from the synced informer's view (the API
        # server is the checkpoint), and released when pods finish or go away. Selected by node
        # (as kubelet watches), not by the assume label: each agent sees its own node's pods,
        # not every GPU pod of the cluster, and a label that lands after the binding is no gap
        self.informer = Informer(self.api, "pods", field_selector=f"{T.NODE_NAME_FIELD}={self.node}")
        self.informer.add_handler(self._on_pod)
        self.tasks.append(self.informer.start())
        await self.informer.synced.wait()
        restored = await self.plugin.rebuild(self.informer.list())
        log.info("agent %s: %d devices, %d CU grants restored", self.node, len(self.topo.devices), restored)
        self._register = register
        await self._serve()
        if register and self.kubelet_check_s > 0:
            self.tasks.append(asyncio.ensure_future(self._kubelet_watch()))
        if self.health_period_s > 0:
            self.tasks.append(asyncio.ensure_future(self._health_loop()))
        if self.reconcile_period_s > 0 and self.pod_resources_socket:
            self.tasks.append(asyncio.ensure_future(self._reconcile_loop()))

    async def reconcile_now(self) -> list[tuple[str, str]]:
        """One pass: kubelet's pod-resources List against the plugin's grants."""
        from .podresources import list_devices

        if self.plugin is None or not os.path.exists(self.pod_resources_socket):
            return []
        listed = await list_devices(self.pod_resources_socket, T.RESOURCE_GPU_PERCENT)
        moved = await self.plugin.reconcile(listed)
        if moved:
            log.warning("agent %s: %d containers ran with another container's grant; reconciled", self.node,
                        len(moved))
        return moved

    async def _reconcile_loop(self) -> None:
        while True:
            await asyncio.sleep(self.reconcile_period_s)
            try:
                await self.reconcile_now()
            except Exception as e:   # kubelet restarting, socket not served yet
                log.debug("agent %s: pod-resources check failed: %s", self.node, e)

    def _dir(self) -> str:
        return self.plugin_dir or "/var/lib/kubelet/device-plugins"

    async def _serve(self) -> None:
        from .plugin import serve

        self.server, self.socket_path = await serve(self.plugin, self._dir(), register=self._register)
        self.registrations += int(self._register)

    @staticmethod
    def _identity(path: str) -> tuple[int, int] | None:
        try:
            st = os.stat(path)
            return st.st_ino, st.st_mtime_ns
        except OSError:
            return None

    async def _kubelet_watch(self) -> None:
        """A restarted kubelet removes every plugin socket and serves a new kubelet.sock; a
        plugin has to notice, serve again and re-register (its devices are unknown to the new
        kubelet until it does). Both files are polled every `kubelet_check_s`."""
        kubelet_sock = os.path.join(self._dir(), "kubelet.sock")
        seen = self._identity(kubelet_sock)
        while True:
            await asyncio.sleep(self.kubelet_check_s)
            now = self._identity(kubelet_sock)
            if now is None:
                continue                                  # kubelet down: wait for it
            if now == seen and os.path.exists(self.socket_path):
                continue
            log.warning("agent %s: kubelet restarted (or our socket vanished): registering again", self.node)
            try:
                if self.server is not None:
                    await self.server.stop(grace=0.5)
                await self._serve()
                seen = now
            except Exception:
                log.exception("agent %s: re-registration failed; retrying", self.node)

    def _on_pod(self, etype: str, pod: dict, old: dict | None) -> None:
        if pu.node_name_of(pod) != self.node or self.plugin is None:
            return
        # a terminating pod's containers still run on their CUs through the grace period: the
        # grant goes back when they stop (Succeeded/Failed) or the pod object is gone
        if etype == "DELETED" or pu.is_terminated(pod):
            self.plugin.release_pod(pu.pod_uid(pod))

    async def _health_loop(self) -> None:
        while True:
            await asyncio.sleep(self.health_period_s)
            try:
                await self.check_health()
            except Exception:
                log.exception("health check failed")

    async def check_health(self) -> list[int]:
        """Re-reads KFD/DRM sysfs: a device whose render node vanished or whose GPU reports
        uncorrectable RAS errors becomes Unhealthy for kubelet and unschedulable for the
        extender (re-published topology annotation). Returns the devices that changed."""
        topo, host = discover(self.sysfs_root, use_amdsmi=False)
        present = {int(g["render_minor"]) for g in host.get("gpus", [])}
        ras_ok = [d.healthy for d in topo.devices] if len(topo.devices) == len(self.topo.devices) else None
        changed = []
        for i, minor in enumerate(self.render_minors()):
            ok = minor in present and (ras_ok is None or ras_ok[i]) and i not in self.selftest_failed
            if self.topo.devices[i].healthy != ok:
                self.topo.devices[i].healthy = ok
                changed.append(i)
            if self.plugin is not None:
                self.plugin.set_health(i, ok)
        if changed:
            log.warning("agent %s: devices %s health changed", self.node, changed)
            await self.api.patch_node(self.node, node_patch(self.topo))
        return changed

    def run_selftest(self, P=None) -> list[int] | None:
        """`gpu_selftest` on every HIP device; returns the failed device indices, or None when
        the probe is missing or its device count does not match the topology (HIP orders
        devices like the KFD nodes the topology is read from)."""
        if P is None:
            from ..native import probe

            P = probe(required=False)
        if P is None:
            return None
        n = P.device_count()
        if n != len(self.topo.devices):
            log.warning("agent %s: %d HIP devices vs %d topology devices: self-test skipped", self.node, n,
                        len(self.topo.devices))
            return None
        return [i for i in range(n) if not gpu_selftest(P, i)]

    async def selftest(self, P=None) -> list[int] | None:
        """Runs the self-test off the event loop and applies it: failed devices become
        Unhealthy for kubelet and unschedulable in the published topology."""
        failed = await asyncio.get_running_loop().run_in_executor(None, self.run_selftest, P)
        if failed is None:
            return None
        self.selftest_failed = set(failed)
        changed = False
        for i, d in enumerate(self.topo.devices):
            ok = i not in self.selftest_failed and d.healthy
            if i in self.selftest_failed and d.healthy:
                d.healthy = False
                changed = True
            if self.plugin is not None:
                self.plugin.set_health(i, ok)
        if changed:
            log.warning("agent %s: self-test failed on devices %s", self.node, sorted(self.selftest_failed))
            await self.api.patch_node(self.node, node_patch(self.topo))
        return failed

    async def stop(self) -> None:
        for t in self.tasks:
            t.cancel()
        if self.informer is not None:
            await self.informer.stop()
        if self.server is not None:
            await self.server.stop(grace=1.0)


def build_parser():
    import argparse

    ap = argparse.ArgumentParser(prog="nanogpu-agent", description="MI355X node agent for nano-gpu-scheduler")
    ap.add_argument("--node-name", default=os.environ.get("NODE_NAME", ""))
    ap.add_argument("--sysfs-root", default="")
    ap.add_argument("--no-amdsmi", action="store_true")
    ap.add_argument("--calibrate", action="store_true", help="run the HIP probe (HBM GB/s) before publishing")
    ap.add_argument("--advertise", choices=["device-plugin", "status"], default="device-plugin")
    ap.add_argument("--plugin-dir", default="/var/lib/kubelet/device-plugins")
    ap.add_argument("--kube-api", default=None)
    ap.add_argument("--kubeconfig", default=os.environ.get("KUBECONFIG"))
    ap.add_argument("--print", action="store_true", help="print the topology annotation and exit")
    ap.add_argument("--selftest", action="store_true",
                    help="run the HIP self-test (HBM copy + MFMA tile) on every device at start-up")
    ap.add_argument("--metrics-port", type=int, default=9410,
                    help="device / pod / container GPU metrics on :PORT/metrics (0: off)")
    ap.add_argument("--pod-resources-socket", default="/var/lib/kubelet/pod-resources/kubelet.sock",
                    help="kubelet's pod-resources API: the grants are checked against it ('' : off)")
    ap.add_argument("--reconcile-period", type=float, default=5.0,
                    help="seconds between pod-resources checks (0: off)")
    return ap


def main(argv: list[str] | None = None) -> int:
    ap = build_parser()
    a = ap.parse_args(argv)
    logging.basicConfig(level=logging.INFO, format="%(asctime)s %(levelname)s %(name)s: %(message)s")
    topo, host = discover(a.sysfs_root, not a.no_amdsmi)
    if a.calibrate:
        calibrate(topo, host=host)
    if a.print:
        print(json.dumps(topo.to_dict(), indent=1))
        return 0 if topo.devices else 1
    if not a.node_name:
        ap.error("--node-name (or NODE_NAME) is required")

    async def run() -> int:
        import signal

        from ..k8s.client import KubeClient, KubeConfig

        api = KubeClient(KubeConfig.auto(a.kubeconfig, a.kube_api))
        agent = NodeAgent(api, a.node_name, topo, host, device_plugin=a.advertise == "device-plugin",
                          plugin_dir=a.plugin_dir, sysfs_root=a.sysfs_root,
                          pod_resources_socket=a.pod_resources_socket, reconcile_period_s=a.reconcile_period)
        await agent.start()
        if a.selftest:
            failed = await agent.selftest()
            log.info("agent %s: self-test %s", a.node_name,
                     "skipped" if failed is None else f"failed on {failed}" if failed else "passed")
        metrics = None
        if a.metrics_port:
            from .metrics import serve_metrics

            metrics, _ = await serve_metrics(agent, port=a.metrics_port)
        stop = asyncio.Event()
        loop = asyncio.get_running_loop()
        for sig in (signal.SIGINT, signal.SIGTERM):
            loop.add_signal_handler(sig, stop.set)
        await stop.wait()
        if metrics is not None:
            await metrics.cleanup()
        await agent.stop()
        await api.close()
        return 0

    return asyncio.run(run())
