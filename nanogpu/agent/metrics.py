"""Node agent /metrics: GPU monitoring at device, pod and container level.

The reference lists "GPU monitor at pod and container level" on its roadmap
(README.md:93) and leaves device metrics to an external exporter queried through Prometheus
(pkg/prometheus/prometheus.go:68-83). This agent serves them itself, in the Prometheus text
format, joined with what it granted:

  per device (schedulable device = GPU or compute partition), read from amdgpu sysfs on scrape
    nanogpu_device_info{device,gpu,partition,part,numa,render}       1
    nanogpu_device_healthy{device}                                   1 | 0
    nanogpu_device_busy_percent{device}                              gpu_busy_percent
    nanogpu_device_mem_busy_percent{device}                          mem_busy_percent (HBM activity)
    nanogpu_device_vram_used_bytes{device} / _vram_total_bytes        mem_info_vram_{used,total}
    nanogpu_device_granted_percent{device}                           sum of container shares
    nanogpu_device_granted_cus{device} / nanogpu_device_cus{device}  CU-mask grants vs CUs
  per container (the grants the device plugin handed out)
    nanogpu_container_gpu_percent{namespace,pod,container,device}
    nanogpu_container_cus{...}                                       CUs in its HSA_CU_MASK
    nanogpu_container_hbm_budget_bytes{...}                          its HBM budget

A pod's utilisation is its share of its device's busy time: the container's CUs over the
device's CUs, times `nanogpu_device_busy_percent` (spatial sharing gives each tenant its own
CUs, which the co-location measurements in profiles/gpu_calibration.md confirm). A sysfs file
that this GPU or partition does not have is left out rather than reported as zero.
"""
from __future__ import annotations

from pathlib import Path


def _esc(v) -> str:
    return str(v).replace("\\", "\\\\").replace('"', '\\"').replace("\n", "\\n")


def _labels(**kv) -> str:
    return "{" + ",".join(f'{k}="{_esc(v)}"' for k, v in kv.items()) + "}"


def _read_int(p: Path) -> int | None:
    try:
        return int(p.read_text().strip())
    except (OSError, ValueError):
        return None


def render(topo, plugin=None, render_minors: list[int] | None = None, sysfs_root: str = "") -> str:
    """Prometheus text exposition of the node's devices and the plugin's live grants."""
    devs = topo.devices
    minors = render_minors or [128 + 8 * i for i in range(len(devs))]
    health = plugin.health if plugin is not None else [bool(d.healthy) for d in devs]
    grants = list(plugin.grants.values()) if plugin is not None else []
    g_pct = [0] * len(devs)
    g_cus = [0] * len(devs)

    def share(a, d):   # (percent, CUs) a grant holds on device d; no mask = the whole device
        whole = len(a.devices) > 1 or a.percent >= 100 or not a.cus
        return (100 if len(a.devices) > 1 else min(a.percent, 100)), (devs[d].cus if whole else a.cus)

    for a in grants:
        for d in a.devices:
            if 0 <= d < len(devs):
                p, c = share(a, d)
                g_pct[d] += p
                g_cus[d] += c
    out: list[str] = []

    def family(name: str, kind: str, help_: str, rows: list[tuple[str, float]]) -> None:
        if not rows:
            return
        out.append(f"# HELP {name} {help_}")
        out.append(f"# TYPE {name} {kind}")
        out.extend(f"{name}{lab} {val}" for lab, val in rows)

    root = Path(sysfs_root or "/")
    busy, mbusy, used, total = [], [], [], []
    for i, d in enumerate(devs):
        base = root / "sys/class/drm" / f"renderD{minors[i]}" / "device"
        for rows, f in ((busy, "gpu_busy_percent"), (mbusy, "mem_busy_percent"),
                        (used, "mem_info_vram_used"), (total, "mem_info_vram_total")):
            v = _read_int(base / f)
            if v is not None:
                rows.append((_labels(device=i), v))
    gpus = {g.index: g for g in topo.gpus}

    def info(i, d):
        g = gpus.get(d.gpu)
        return _labels(device=i, gpu=d.gpu, partition=g.compute_partition if g else "SPX", part=d.part,
                       numa=g.numa if g else -1, render=minors[i])

    family("nanogpu_device_info", "gauge", "schedulable device (GPU or compute partition) of this node",
           [(info(i, d), 1) for i, d in enumerate(devs)])
    family("nanogpu_device_healthy", "gauge", "1 if the device is advertised Healthy to kubelet",
           [(_labels(device=i), int(bool(health[i]))) for i in range(len(devs))])
    family("nanogpu_device_busy_percent", "gauge", "amdgpu gpu_busy_percent", busy)
    family("nanogpu_device_mem_busy_percent", "gauge", "amdgpu mem_busy_percent (HBM activity)", mbusy)
    family("nanogpu_device_vram_used_bytes", "gauge", "amdgpu mem_info_vram_used", used)
    family("nanogpu_device_vram_total_bytes", "gauge", "amdgpu mem_info_vram_total", total)
    family("nanogpu_device_granted_percent", "gauge", "gpu-percent granted to running containers",
           [(_labels(device=i), g_pct[i]) for i in range(len(devs))])
    family("nanogpu_device_cus", "gauge", "compute units of the device",
           [(_labels(device=i), d.cus) for i, d in enumerate(devs)])
    family("nanogpu_device_granted_cus", "gauge", "compute units held by containers' CU masks",
           [(_labels(device=i), g_cus[i]) for i in range(len(devs))])
    rows_p, rows_c, rows_m = [], [], []
    for a in sorted(grants, key=lambda a: (a.pod_key, a.container)):
        ns, _, pod = a.pod_key.partition("/")
        for d in a.devices:
            if not 0 <= d < len(devs):
                continue
            lab = _labels(namespace=ns, pod=pod, container=a.container, device=d)
            p, c = share(a, d)
            rows_p.append((lab, p))
            rows_c.append((lab, c))
            if a.mib:
                rows_m.append((lab, a.mib * (1 << 20) // max(1, len(a.devices))))
    family("nanogpu_container_gpu_percent", "gauge", "gpu-percent of the device granted to the container", rows_p)
    family("nanogpu_container_cus", "gauge", "compute units the container may use on the device", rows_c)
    family("nanogpu_container_hbm_budget_bytes", "gauge", "HBM budget of the container on the device", rows_m)
    if plugin is not None:
        family("nanogpu_plugin_swaps_fixed_total", "counter",
               "containers kubelet admitted with another container's grant, reconciled from pod-resources",
               [("", plugin.swaps_fixed)])
        family("nanogpu_plugin_id_mismatches_total", "counter",
               "Allocate calls whose kubelet IDs named another device than the container's placement",
               [("", plugin.id_mismatches)])
    return "\n".join(out) + "\n"


async def serve_metrics(agent, host: str = "0.0.0.0", port: int = 9410):
    """aiohttp server with /metrics and /healthz for a running NodeAgent."""
    from aiohttp import web

    async def metrics(_req):
        text = render(agent.topo, agent.plugin, agent.render_minors(), agent.sysfs_root)
        return web.Response(text=text, content_type="text/plain", charset="utf-8")

    async def healthz(_req):
        return web.Response(text="ok")

    app = web.Application()
    app.router.add_get("/metrics", metrics)
    app.router.add_get("/healthz", healthz)
    runner = web.AppRunner(app)
    await runner.setup()
    site = web.TCPSite(runner, host, port)
    await site.start()
    bound = site._server.sockets[0].getsockname()[1] if site._server and site._server.sockets else port
    return runner, bound
