"""Topology reader (native/src/topo.cpp) + node model (nanogpu/topology/model.py).

Fixtures: the trimmed KFD/DRM sysfs capture of a real MI355X box
(tests/fixtures/sysfs/mi355x_real: one visible GPU of an 8-GPU xGMI hive) and synthetic
8-GPU trees in every compute-partition mode (nanogpu/topology/fixtures.py), which is how
8-GPU and CPX topologies are tested without 8 GPUs.
"""
import json
import subprocess
from pathlib import Path

import pytest

from nanogpu import _native as N
from nanogpu.topology.fixtures import VRAM, write_mi355x_sysfs
from nanogpu.topology.model import NodeTopology, from_host_json, from_node, synthetic_mi355x

ROOT = Path(__file__).resolve().parent.parent
REAL = ROOT / "tests/fixtures/sysfs/mi355x_real"


def discover(root) -> dict:
    return json.loads(N.discover_topology(str(root), False))


def test_real_capture_single_visible_gpu_of_8_hive():
    h = discover(REAL)
    assert h["n_physical"] == 1 and len(h["gpus"]) == 1 and h["links"] == []
    g = h["gpus"][0]
    assert (g["cus"], g["num_xcc"], g["lds_size_kib"]) == (256, 8, 160)
    assert g["gfx_target_version"] == 90500 and g["device_id"] == 30115
    assert g["vram_bytes"] == 309220868096
    assert (g["compute_partition"], g["memory_partition"]) == ("SPX", "NPS1")
    assert g["numa"] == 1
    # the other 7 GPUs are hidden from the container, but their xGMI links are not
    assert g["xgmi_peers"] == 7 and g["xgmi_min_bw_mbs"] == g["xgmi_max_bw_mbs"] == 76000
    t = from_host_json(h)
    assert t.gfx == "gfx950" and t.model == "AMD Instinct MI355X"
    assert t.gpus[0].xgmi_peers == 7 and t.gpus[0].xgmi_link_gbs == 76.0
    assert t.devices[0].hbm_mib == 309220868096 >> 20


@pytest.mark.parametrize("mode,parts", [("SPX", 1), ("DPX", 2), ("QPX", 4), ("CPX", 8)])
def test_synthetic_8gpu_partition_modes(tmp_path, mode, parts):
    write_mi355x_sysfs(tmp_path, 8, mode)
    h = discover(tmp_path)
    assert h["n_physical"] == 8 and len(h["gpus"]) == 8 * parts
    t = from_host_json(h)
    assert len(t.gpus) == 8 and len(t.devices) == 8 * parts
    for d in t.devices:
        assert d.cus == 256 // parts and d.xcds == 8 // parts
        # NPS1: every partition draws from its GPU's one 288 GB pool
        assert d.hbm_mib == VRAM >> 20
        if parts == 1:
            assert d.pool == -1
        else:
            assert (d.pool, d.mib_share) == (d.gpu * 8, (VRAM >> 20) // parts)
    assert [d.part for d in t.devices[:parts]] == list(range(parts))
    assert {g.numa for g in t.gpus} == {0, 1}
    # full xGMI mesh between physical GPUs, 76 GB/s per link
    for a in range(8):
        for b in range(8):
            assert t.link_bw[a][b] == (0.0 if a == b else 76.0)
    assert all(g.xgmi_peers == 7 for g in t.gpus)


def test_cpx_nps2_hbm_pools(tmp_path):
    write_mi355x_sysfs(tmp_path, 2, "CPX", "NPS2")
    t = from_host_json(discover(tmp_path))
    # each CPX partition reports its NPS2 half; 4 partitions share each half as one pool
    half = (VRAM // 2) >> 20
    assert all(d.hbm_mib == half and d.mib_share == half // 4 for d in t.devices)
    assert [d.pool for d in t.devices[:8]] == [0, 0, 0, 0, 1, 1, 1, 1]
    assert t.gpus[0].hbm_mib == 2 * half and t.hbm_capacity_mib() == 4 * half
    write_mi355x_sysfs(tmp_path / "dpx", 1, "DPX", "NPS2")     # one compute partition per memory partition
    t2 = from_host_json(discover(tmp_path / "dpx"))
    assert [(d.pool, d.hbm_mib) for d in t2.devices] == [(-1, half), (-1, half)]


def test_hidden_gpus_and_degraded_link(tmp_path):
    write_mi355x_sysfs(tmp_path, 8, "SPX", hidden=(1, 2, 3, 4, 5, 6, 7))
    h = discover(tmp_path)
    assert len(h["gpus"]) == 1 and h["gpus"][0]["xgmi_peers"] == 7
    d2 = tmp_path / "deg"
    write_mi355x_sysfs(d2, 4, "SPX", degraded={(0, 3): 19000})
    t = from_host_json(discover(d2))
    assert t.link_bw[0][3] == t.link_bw[3][0] == 19.0 and t.link_bw[0][1] == 76.0
    assert t.gpus[0].xgmi_link_gbs == 19.0


def test_no_xgmi_pcie_only(tmp_path):
    write_mi355x_sysfs(tmp_path, 2, "SPX", xgmi=False)
    t = from_host_json(discover(tmp_path))
    assert t.link_bw == [[0.0, 0.0], [0.0, 0.0]] and t.gpus[0].xgmi_peers == 0


def test_empty_root_warns(tmp_path):
    h = discover(tmp_path)
    assert h["gpus"] == [] and h["warnings"]


def test_cli_matches_module(tmp_path):
    write_mi355x_sysfs(tmp_path, 8, "QPX")
    exe = ROOT / "native/bin/nanogpu-topo"
    r = subprocess.run([str(exe), "--root", str(tmp_path), "--no-amdsmi"], capture_output=True, text=True)
    assert r.returncode == 0
    assert json.loads(r.stdout) == discover(tmp_path)
    r = subprocess.run([str(exe), "--root", str(tmp_path / "nothing"), "--no-amdsmi"], capture_output=True)
    assert r.returncode == 1


def test_annotation_roundtrip_and_fallback():
    from nanogpu.k8s import podutil as pu

    t = synthetic_mi355x(8, "CPX")
    assert NodeTopology.from_json(t.to_json()).to_dict() == t.to_dict()
    node = pu.make_node("n", 64, t.to_json())
    assert len(from_node(node).devices) == 64
    # annotation inconsistent with capacity => reference fallback (capacity / 100 devices)
    bad = pu.make_node("n", 8, t.to_json())
    fb = from_node(bad)
    assert len(fb.devices) == 8 and fb.devices[0].hbm_mib == 0
    assert len(from_node(pu.make_node("n", 3)).devices) == 3


def test_properties_parser():
    m = N.parse_properties("simd_count 1024\n  location_id   61696 \nbad\n")
    assert m == {"simd_count": "1024", "location_id": "61696"}
