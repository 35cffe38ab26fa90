"""Synthetic KFD/DRM sysfs trees of MI355X nodes, for testing the native topology reader
(native/src/topo.cpp) on topologies the single-GPU test box cannot show.

The property values are the ones captured from a real MI355X (gpurun box, KFD node 6 of
an 8-GPU hive: tests/fixtures/sysfs/mi355x_real): 1024 SIMDs (256 CUs), 8 XCCs, 160 KiB
LDS, gfx_target_version 90500, device_id 30115, 309,220,868,096 B of VRAM, and xGMI
io_links of type 11, weight 15, 76,000 MB/s to each of the 7 peers plus one PCIe link
(type 2, weight 52) to the CPU NUMA node.

Partition modes split a GPU into `parts` KFD nodes that share the PCI location and
unique_id (CPX: 8 nodes of 1 XCC / 32 CUs each); NPSx splits the VRAM between memory
partitions.
"""
from __future__ import annotations

from pathlib import Path

PARTS = {"SPX": 1, "DPX": 2, "QPX": 4, "CPX": 8}
NPS = {"NPS1": 1, "NPS2": 2, "NPS4": 4, "NPS8": 8}
VRAM = 309_220_868_096
XGMI_MBS = 76_000


def _w(p: Path, text: str) -> None:
    p.parent.mkdir(parents=True, exist_ok=True)
    p.write_text(text)


def _props(d: dict) -> str:
    return "".join(f"{k} {v}\n" for k, v in d.items())


def write_mi355x_sysfs(root: str | Path, n_gpus: int = 8, compute: str = "SPX", memory: str = "NPS1",
                       n_numa: int = 2, hidden: tuple[int, ...] = (), xgmi: bool = True,
                       degraded: dict | None = None, ras: dict | None = None) -> Path:
    """Writes /sys/class/{kfd,drm} for `n_gpus` MI355X under `root` and returns root.

    hidden:   physical GPUs whose KFD properties are unreadable (as for GPUs outside the
              container's cgroup on the real box: the node dirs and io_links exist, the
              properties file is empty);
    degraded: {(a, b): MB/s} overrides for individual xGMI links;
    ras:      {gpu: (ue, ce)} amdgpu RAS counters (written as umc_err_count).
    """
    root = Path(root)
    parts = PARTS[compute]
    nps = NPS[memory]
    kfd = root / "sys/class/kfd/kfd/topology/nodes"
    degraded = degraded or {}
    # CPU nodes first (KFD numbers CPUs 0..n_numa-1)
    for c in range(n_numa):
        _w(kfd / str(c) / "properties", _props({"cpu_cores_count": 128, "simd_count": 0, "mem_banks_count": 1,
                                                "io_links_count": 0, "location_id": 0, "drm_render_minor": 0}))
        _w(kfd / str(c) / "gpu_id", "0\n")
    node_of: dict[tuple[int, int], int] = {}
    nid = n_numa
    for g in range(n_gpus):
        for p in range(parts):
            node_of[(g, p)] = nid
            nid += 1
    gpu_per_numa = max(1, n_gpus // n_numa)
    for (g, p), n in node_of.items():
        numa = min(n_numa - 1, g // gpu_per_numa)
        render = 128 + 8 * (g * parts + p)
        loc = 0x0500 + 0x1000 * g  # bus 0x05 + 0x10*g, device 0, function 0
        props = {
            "cpu_cores_count": 0, "simd_count": 1024 // parts, "mem_banks_count": 1, "caches_count": 0,
            "io_links_count": 0, "p2p_links_count": 0, "max_waves_per_simd": 8, "lds_size_in_kb": 160,
            "wave_front_size": 64, "simd_per_cu": 4, "gfx_target_version": 90500, "vendor_id": 4098,
            "device_id": 30115, "location_id": loc, "domain": 0, "drm_render_minor": render,
            "hive_id": 8419846131476971335 if xgmi else 0, "num_sdma_xgmi_engines": 14,
            "max_engine_clk_fcompute": 2400, "local_mem_size": 0,
            "unique_id": 10461056751509885444 + g, "num_xcc": 8 // parts,
        }
        base = kfd / str(n)
        _w(base / "properties", "" if g in hidden else _props(props))
        _w(base / "gpu_id", "" if g in hidden else f"{8465 + 1000 * g + p}\n")
        _w(base / "name", "ip discovery\n")
        # VRAM: the memory partition a compute partition sees (NPS1: the whole pool)
        _w(base / "mem_banks/0/properties", _props({"heap_type": 1, "size_in_bytes": VRAM // nps, "flags": 0,
                                                     "width": 8192, "mem_clk_max": 2000}))
        links = [{"type": 2, "node_from": n, "node_to": numa, "weight": 52, "min_bandwidth": 0,
                  "max_bandwidth": 64000}]
        if xgmi:
            for (g2, p2), n2 in node_of.items():
                if n2 == n or (g2 == g):
                    continue
                if p2 != p and parts > 1:
                    continue  # partition k talks to partition k of each peer
                bw = degraded.get((min(g, g2), max(g, g2)), XGMI_MBS)
                links.append({"type": 11, "node_from": n, "node_to": n2, "weight": 15,
                              "min_bandwidth": bw, "max_bandwidth": bw})
        for i, lk in enumerate(links):
            _w(base / "io_links" / str(i) / "properties", _props(lk))
        drm = root / f"sys/class/drm/renderD{render}/device"
        _w(drm / "current_compute_partition", compute + "\n")
        _w(drm / "available_compute_partition", "SPX, DPX, QPX, CPX\n")
        _w(drm / "current_memory_partition", memory + "\n")
        _w(drm / "available_memory_partition", "NPS1, NPS2\n")
        _w(drm / "mem_info_vram_total", f"{VRAM // nps}\n")
        _w(drm / "numa_node", f"{numa}\n")
        _w(drm / "product_name", "AMD Instinct MI355 OAM\n")
        ue, ce = (ras or {}).get(g, (0, 0))
        _w(drm / "ras/umc_err_count", f"ue: {ue}\nce: {ce}\n")
        _w(drm / "ras/gfx_err_count", "ue: 0\nce: 0\n")
    return root
