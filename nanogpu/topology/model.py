"""Node GPU topology model: what the node agent publishes and the extender schedules on.

Reference: the reference knows only a GPU count, ⌊capacity/100⌋ (pkg/utils/node.go:8-14),
and every device is a 100% slot (pkg/dealer/node.go:25-42). Here a node carries a
`nano-gpu/topology` annotation (JSON, schema below) written by the node agent from the
native reader (native/src/topo.cpp). The schedulable *device* is a compute partition
(SPX: the whole MI355X; DPX/QPX/CPX: 2/4/8 partitions of its 8 XCDs); every device still
counts 100 gpu-percent, so node capacity stays `100 x devices` and the reference
annotation contract (`nano-gpu/container-<c>=<device index>`) is unchanged.

Schema (version 1):
{
  "version": 1, "model": "AMD Instinct MI355X", "gfx": "gfx950",
  "virtualization": "BAREMETAL",
  "gpus":    [{"index": 0, "numa": 0, "cus": 256, "xcds": 8, "hbm_mib": 294912,
               "compute_partition": "SPX", "memory_partition": "NPS1", "bdf": "0000:05:00.0",
               "hbm_busy_cal": [[25, 20.7], [100, 28.7]]}],   # optional (agent --calibrate)
  "devices": [{"gpu": 0, "part": 0, "cus": 256, "xcds": 8, "hbm_mib": 294912}],
  "link_bw": [[0.0, 153.0, ...], ...],     # GB/s between physical GPUs (0 = no direct link)
  "calibration": {...}                      # optional probe results (HBM GB/s, CU map)
}
"""
from __future__ import annotations

import json
from dataclasses import dataclass, field
from typing import Any

from .. import types as T

PARTITIONS = {"SPX": 1, "DPX": 2, "TPX": 3, "QPX": 4, "CPX": 8}


@dataclass
class GpuSpec:
    index: int
    numa: int = -1
    cus: int = T.MI355X_CUS
    xcds: int = T.MI355X_XCDS
    hbm_mib: int = 0
    compute_partition: str = "SPX"
    memory_partition: str = "NPS1"
    bdf: str = ""
    ras_ue: int = 0              # uncorrectable / correctable RAS errors (amdgpu ras/*_err_count)
    ras_ce: int = 0
    xgmi_peers: int = 0          # xGMI links of this GPU (visible or not from the agent's cgroup)
    xgmi_link_gbs: float = 0.0   # slowest of them, GB/s (KFD io_link max_bandwidth)
    # this GPU's own mem_busy_percent scale: [[CU share %, mem_busy %], ...] of the agent's
    # streaming probe alone on it (agent --calibrate, probe.calibrate.hbm_busy_calibration);
    # the poller maps readings through it onto types.HBM_STREAMING_CURVE (telemetry.store
    # normalize_hbm_activity). Empty: readings are taken as they are.
    hbm_busy_cal: list = field(default_factory=list)


@dataclass
class DeviceSpec:
    gpu: int
    part: int = 0
    cus: int = T.MI355X_CUS
    xcds: int = T.MI355X_XCDS
    hbm_mib: int = 0             # HBM this device can draw from (its pool's size when pooled)
    healthy: bool = True         # False: never chosen (uncorrectable RAS errors, device gone)
    pool: int = -1               # shared HBM pool (memory partition) id within the node, -1 = own HBM
    mib_share: int = 0           # HBM a whole-device grant takes from the pool (pool / members)


@dataclass
class NodeTopology:
    gpus: list[GpuSpec]
    devices: list[DeviceSpec]
    link_bw: list[list[float]] = field(default_factory=list)
    model: str = "AMD Instinct MI355X"
    gfx: str = "gfx950"
    virtualization: str = "UNKNOWN"
    calibration: dict = field(default_factory=dict)
    version: int = 1

    # --- serialisation -------------------------------------------------------------
    def to_dict(self) -> dict:
        return {
            "version": self.version, "model": self.model, "gfx": self.gfx,
            "virtualization": self.virtualization,
            "gpus": [g.__dict__ for g in self.gpus],
            "devices": [d.__dict__ for d in self.devices],
            "link_bw": self.link_bw,
            "calibration": self.calibration,
        }

    def to_json(self) -> str:
        return json.dumps(self.to_dict(), separators=(",", ":"), sort_keys=True)

    @classmethod
    def from_dict(cls, d: dict) -> "NodeTopology":
        gpus = [GpuSpec(**{k: v for k, v in g.items() if k in GpuSpec.__dataclass_fields__})
                for g in d.get("gpus", [])]
        devs = [DeviceSpec(**{k: v for k, v in x.items() if k in DeviceSpec.__dataclass_fields__})
                for x in d.get("devices", [])]
        if not devs:
            devs = [DeviceSpec(gpu=g.index, cus=g.cus, xcds=g.xcds, hbm_mib=g.hbm_mib) for g in gpus]
        return cls(gpus=gpus, devices=devs, link_bw=[list(map(float, r)) for r in d.get("link_bw", [])],
                   model=d.get("model", ""), gfx=d.get("gfx", ""),
                   virtualization=d.get("virtualization", "UNKNOWN"),
                   calibration=d.get("calibration") or {}, version=int(d.get("version", 1)))

    @classmethod
    def from_json(cls, s: str) -> "NodeTopology":
        return cls.from_dict(json.loads(s))

    # --- ledger views ----------------------------------------------------------------
    @property
    def n_gpus(self) -> int:
        return len(self.gpus)

    def ledger_devices(self, track_hbm: bool = True) -> list[dict]:
        numa = {g.index: g.numa for g in self.gpus}
        return [{"pct_total": T.GPU_PERCENT_EACH_CARD, "mib_total": d.hbm_mib if track_hbm else 0,
                 "gpu": d.gpu, "part": d.part, "numa": numa.get(d.gpu, -1), "healthy": bool(d.healthy),
                 "xcds": d.xcds, "cus": d.cus, "pool": d.pool if track_hbm else -1,
                 "mib_share": d.mib_share or d.hbm_mib} for d in self.devices]

    def hbm_capacity_mib(self) -> int:
        """Node HBM: every pool once plus every device with its own HBM."""
        pools = {d.pool: d.hbm_mib for d in self.devices if d.pool >= 0}
        return sum(pools.values()) + sum(d.hbm_mib for d in self.devices if d.pool < 0)

    def ledger_topo(self) -> dict:
        return {"n_gpus": self.n_gpus, "numa": [g.numa for g in self.gpus], "link_bw": self.link_bw}


def fallback_topology(n_devices: int) -> NodeTopology:
    """Reference behaviour (node.go:25-42): N anonymous 100% devices, no HBM, no links."""
    gpus = [GpuSpec(index=i, hbm_mib=0) for i in range(n_devices)]
    return NodeTopology(gpus=gpus, devices=[DeviceSpec(gpu=i, hbm_mib=0) for i in range(n_devices)],
                        link_bw=[[0.0] * n_devices for _ in range(n_devices)], model="", gfx="")


def synthetic_mi355x(n_gpus: int = 8, compute: str = "SPX", memory: str = "NPS1",
                     hbm_mib: int = 288 * 1024, link_gbs: float = 153.0,
                     gpus_per_numa: int = 4, link_matrix: list[list[float]] | None = None) -> NodeTopology:
    """An 8x MI355X platform (full xGMI mesh, 4 GPUs per socket) for tests and benches.

    `link_gbs` is a placeholder until the probe measures it; the agent overwrites it with
    what KFD/amdsmi or the peer-copy probe report. `link_matrix` (n_gpus x n_gpus GB/s, as
    measured by `probe.calibrate.link_matrix`) replaces the uniform mesh when given.
    """
    parts = PARTITIONS[compute]
    nps = _nps(memory)
    gpus, devs = [], []
    for g in range(n_gpus):
        gpus.append(GpuSpec(index=g, numa=g // max(1, gpus_per_numa), hbm_mib=hbm_mib,
                            compute_partition=compute, memory_partition=memory,
                            bdf=f"0000:{0x05 + 0x10 * g:02x}:00.0"))
        for p in range(parts):
            devs.append(DeviceSpec(gpu=g, part=p, cus=T.MI355X_CUS // parts,
                                   xcds=max(1, T.MI355X_XCDS // parts)))
        _assign_pools([d for d in devs if d.gpu == g], hbm_mib // nps, nps)
    if link_matrix is not None and len(link_matrix) == n_gpus:
        # a link's weight is the slower of its two directions
        bw = [[0.0 if a == b else min(link_matrix[a][b], link_matrix[b][a]) for b in range(n_gpus)]
              for a in range(n_gpus)]
    else:
        bw = [[0.0 if a == b else link_gbs for b in range(n_gpus)] for a in range(n_gpus)]
    return NodeTopology(gpus=gpus, devices=devs, link_bw=bw, virtualization="BAREMETAL")


def synthetic_sriov_guest(n_vfs: int = 4, hbm_mib: int = 288 * 1024) -> NodeTopology:
    """A VM on an MI355X host in SR-IOV (MxGPU) mode: `n_vfs` virtual functions passed
    through, one whole GPU each. From inside the guest amd-smi reports virtualization mode
    GUEST, the VFs' VRAM is their own, and neither the xGMI links between the physical GPUs
    nor the host's NUMA layout are visible (link matrix all zero, NUMA unknown), so the
    topology term stays neutral and placement follows the policy and HBM alone."""
    gpus = [GpuSpec(index=g, numa=-1, hbm_mib=hbm_mib, bdf=f"0000:{0x10 + g:02x}:00.0") for g in range(n_vfs)]
    devs = [DeviceSpec(gpu=g, hbm_mib=hbm_mib) for g in range(n_vfs)]
    return NodeTopology(gpus=gpus, devices=devs, link_bw=[[0.0] * n_vfs for _ in range(n_vfs)],
                        virtualization="GUEST")


def _assign_pools(ds: list, pool_mib: int, nps: int) -> None:
    """Partitions of one GPU: `nps` memory partitions of `pool_mib` each, len(ds)/nps
    compute partitions per memory partition. One member per pool = the device's own HBM."""
    members = max(1, len(ds) // max(1, nps))
    for k, d in enumerate(ds):
        d.hbm_mib = pool_mib
        if members > 1:
            d.pool = d.gpu * 8 + k // members
            d.mib_share = pool_mib // members
        else:
            d.pool, d.mib_share = -1, pool_mib


def _nps(mode: str) -> int:
    m = (mode or "").upper()
    return int(m[3:]) if m.startswith("NPS") and m[3:].isdigit() else 1


def from_host_json(host: str | dict, max_ue: int = 0) -> NodeTopology:
    """Converts the native reader's JSON (nanogpu-topo / _native.discover_topology).
    Devices with more than `max_ue` uncorrectable RAS errors are published unhealthy."""
    h = json.loads(host) if isinstance(host, str) else host
    gpus_by_parent: dict[int, GpuSpec] = {}
    devices: list[DeviceSpec] = []
    kfd_parent: dict[int, int] = {}
    for g in h.get("gpus", []):
        parent = int(g.get("parent", 0))
        kfd_parent[int(g.get("kfd_node", -1))] = parent
        part = int(g.get("partition", 0))
        cp = (g.get("compute_partition") or "SPX").upper() or "SPX"
        mib = int(g.get("vram_bytes", 0)) // (1 << 20)
        if parent not in gpus_by_parent:
            loc = int(g.get("location_id", 0))
            gpus_by_parent[parent] = GpuSpec(
                index=parent, numa=int(g.get("numa", -1)), cus=0, xcds=0, hbm_mib=0,
                compute_partition=cp, memory_partition=(g.get("memory_partition") or "").upper(),
                xgmi_peers=int(g.get("xgmi_peers", 0)), xgmi_link_gbs=float(g.get("xgmi_min_bw_mbs", 0)) / 1000.0,
                ras_ue=int(g.get("ras_ue", 0)), ras_ce=int(g.get("ras_ce", 0)),
                bdf=f"{int(g.get('domain', 0)):04x}:{(loc >> 8) & 0xff:02x}:{(loc >> 3) & 0x1f:02x}.{loc & 7}")
        gs = gpus_by_parent[parent]
        gs.cus += int(g.get("cus", 0))
        gs.xcds += int(g.get("num_xcc", 1))
        devices.append(DeviceSpec(gpu=parent, part=part, cus=int(g.get("cus", 0)),
                                  xcds=int(g.get("num_xcc", 1)), hbm_mib=mib,
                                  healthy=int(g.get("ras_ue", 0)) <= max_ue))
    # HBM: a compute partition reports the memory partition it lives in (NPS1: the whole
    # pool; NPSn: 1/n of it); the parts/n compute partitions of one memory partition draw
    # from it as a shared pool (mirrored in the ledger).
    for parent, gs in gpus_by_parent.items():
        ds = [d for d in devices if d.gpu == parent]
        reported = max((d.hbm_mib for d in ds), default=0)
        if ds and len(ds) > 1 and all(d.hbm_mib == reported for d in ds):
            nps = _nps(gs.memory_partition)
            _assign_pools(ds, reported, nps if len(ds) % nps == 0 else 1)
            gs.hbm_mib = reported * (nps if len(ds) % nps == 0 else 1)
        else:
            gs.hbm_mib = sum(d.hbm_mib for d in ds)
    n = len(gpus_by_parent)
    bw = [[0.0] * n for _ in range(n)]
    for lk in h.get("links", []):
        a, b = kfd_parent.get(int(lk.get("from", -1))), kfd_parent.get(int(lk.get("to", -1)))
        if a is None or b is None or a == b:
            continue
        gbs = float(lk.get("max_bw_mbs", 0)) / 1000.0
        if gbs <= 0 and int(lk.get("weight", 0)) > 0:
            gbs = 1000.0 / float(lk["weight"])  # relative weight when bandwidth is not exposed
        bw[a][b] = max(bw[a][b], gbs)
    gpus = [gpus_by_parent[i] for i in sorted(gpus_by_parent)]
    gfx = ""
    if h.get("gpus"):
        v = int(h["gpus"][0].get("gfx_target_version", 0))
        if v:
            gfx = f"gfx{v // 10000}{(v // 100) % 100:x}{v % 100:x}" if v >= 90000 else f"gfx{v}"
    return NodeTopology(gpus=gpus, devices=devices, link_bw=bw, virtualization=h.get("virtualization", "UNKNOWN"),
                        model="AMD Instinct MI355X" if gfx == "gfx950" else (gfx or "unknown"), gfx=gfx)


def from_node(node: dict) -> NodeTopology:
    """Topology annotation if present and consistent, else the reference fallback."""
    from ..k8s.podutil import meta, node_gpu_count

    ann = (meta(node).get("annotations") or {}).get(T.ANNOTATION_TOPOLOGY)
    count = node_gpu_count(node)
    if ann:
        try:
            t = NodeTopology.from_json(ann)
            if t.devices and (count == 0 or len(t.devices) == count):
                return t
        except (ValueError, TypeError, KeyError):
            pass
    return fallback_topology(count)


def describe(t: NodeTopology) -> dict[str, Any]:
    return {"gpus": t.n_gpus, "devices": len(t.devices),
            "partition": t.gpus[0].compute_partition if t.gpus else "",
            "hbm_mib_total": sum(d.hbm_mib for d in t.devices), "gfx": t.gfx}
