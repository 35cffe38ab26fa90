"""Real-MI355X tests (run on the GPU box with `pytest -m gpu`).

They exercise the native code that only a GPU host can run: the HIP gfx950 probe kernels
(numerics against fp32 torch references, HBM copy, CU-mask isolation), the KFD/amdsmi
topology reader on real sysfs, and the node-agent path that turns the discovered device
into the scheduler's node model. Multi-GPU parts (xGMI peer copies, RCCL link matrix) skip
when only one device is visible.
"""
import json

import pytest

pytestmark = pytest.mark.gpu


def record(key: str, value) -> None:
    """Measured facts for profiles/gpu_calibration.md (merged back from the GPU box)."""
    from pathlib import Path

    p = Path("gpurun_out/gpu_facts.json")
    p.parent.mkdir(exist_ok=True)
    d = json.loads(p.read_text()) if p.exists() else {}
    d[key] = value
    p.write_text(json.dumps(d, indent=1))


@pytest.fixture(scope="module")
def P():
    import torch

    if not torch.cuda.is_available():
        pytest.skip("no GPU visible")
    from nanogpu.native import probe

    return probe(required=True)  # fails loudly if the HIP extension is missing


@pytest.fixture(scope="module")
def host():
    from nanogpu.native import core

    return json.loads(core().discover_topology("", True))


def test_device_is_mi355x(P):
    props = P.device_props(0)
    assert props["gcn_arch"].startswith("gfx950")
    assert props["warp_size"] == 64
    assert props["cus"] == 256
    assert props["total_mem_bytes"] > 250 * (1 << 30)
    assert props["max_shared_per_cu_bytes"] == 160 * 1024


def test_mfma_tile_matches_fp32_reference(P):
    import torch

    g = torch.Generator().manual_seed(0)
    for _ in range(3):
        a = torch.randn(32, 16, generator=g).bfloat16().float()
        b = torch.randn(16, 32, generator=g).bfloat16().float()
        c = torch.tensor(P.gemm_tile(a.flatten().tolist(), b.flatten().tolist())).view(32, 32)
        ref = a.double() @ b.double()
        torch.testing.assert_close(c.double(), ref, rtol=1e-5, atol=1e-5)


def test_hbm_copy_bit_exact_and_fast(P):
    assert P.copy_check(0, (1 << 24) + 3)
    gbs = P.hbm_bandwidth(0, 1 << 30, 10)
    record("hbm_copy_gbs_1GiB", round(gbs, 1))
    # MI355X: 8 TB/s peak, ~6.3 TB/s achievable (MI355X_MICROARCH.md); catch gross regressions
    assert gbs > 3500, gbs


def test_cu_mask_spatial_share_scales(P):
    """A gpu-percent grant maps to an XCD-symmetric CU mask: TFLOP/s must track the CUs granted."""
    from nanogpu.probe.calibrate import cu_mask_isolation

    r = cu_mask_isolation(0, fractions=(1, 2, 4, 8), iters=1024)
    record("mfma_tflops_by_cus", {str(k): round(v, 1) for k, v in r.items()})
    full, quarter = r[256], r[64]
    assert 0.18 < quarter / full < 0.35, r


def test_cu_census_covers_all_xcds(P):
    recs = P.cu_census(0, [], 2048, 16)
    xccs = {x for x, _ in recs}
    assert xccs == set(range(8)), xccs


def test_topology_reader_on_real_sysfs(host, P):
    assert host["gpus"], host
    g = host["gpus"][0]
    assert g["cus"] == 256 and g["num_xcc"] == 8
    assert g["compute_partition"] in ("SPX", "DPX", "QPX", "CPX")
    record("live_topology", {k: g.get(k) for k in ("cus", "num_xcc", "vram_bytes", "numa", "compute_partition",
                                                    "memory_partition", "xgmi_peers", "xgmi_min_bw_mbs",
                                                    "ras_available", "ras_ue", "ras_ce")})
    props = P.device_props(0)
    # the reader's VRAM equals what HIP reports (both come from the same KFD heap)
    assert abs(g["vram_bytes"] - props["total_mem_bytes"]) < (1 << 30)


def test_agent_node_model_from_real_device(host):
    from nanogpu.topology.model import from_host_json

    topo = from_host_json(host)
    assert len(topo.devices) >= 1
    assert topo.devices[0].hbm_mib == host["gpus"][0]["vram_bytes"] >> 20


def test_peer_bandwidth_multi_gpu(P):
    # the deadline-bounded probe: a wedged transfer raises PeerTimeout (a TimeoutError)
    assert issubclass(P.PeerTimeout, TimeoutError)
    with pytest.raises(ValueError):
        P.peer_bandwidth(0, 0, 1 << 20, 1, 5.0)
    if P.device_count() < 2:
        pytest.skip("single visible GPU")
    r = P.peer_bandwidth(0, 1, 64 << 20, 3)
    assert r["gbs"] > 10 and r["dma_gbs"] > 0


def test_smoke_entry():
    import __graft_entry__ as g

    g.smoke()


def test_bench_one_step_on_gpu(tmp_path):
    import subprocess
    import sys
    from pathlib import Path

    root = Path(__file__).resolve().parent.parent
    out = tmp_path / "b.json"
    r = subprocess.run([sys.executable, str(root / "bench.py"), "--steps", "1", "--warmup", "0", "--pods", "200",
                        "--nodes", "8", "--json-out", str(out)], capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-2000:]
    line = json.loads(out.read_text())
    assert line["scheduled"] > 0 and line["gpu"]["gpu"]["cus"] == 256


def test_colocated_cu_grants_are_isolated(P):
    """Two tenants of one device with the agent's disjoint XCD-symmetric masks (25 % / 75 %)
    run concurrently; each gets throughput in proportion to its CUs."""
    from nanogpu.agent import cumask

    d = cumask.DeviceCUs(256, 8)
    a, b = d.grant("a", 25), d.grant("b", 75)
    alone = P.mfma_throughput(0, [], 2048, 1024)["tflops"]
    ta, tb = P.mfma_colocated(0, [cumask.mask_words(a), cumask.mask_words(b)], [len(a) * 8, len(b) * 8], 1024)
    record("colocated_25_75", {"alone_tflops": round(alone, 1), "tenant25_tflops": round(ta, 1),
                               "tenant75_tflops": round(tb, 1)})
    assert 0.17 < ta / alone < 0.34, (ta, tb, alone)
    assert 0.55 < tb / alone < 0.85, (ta, tb, alone)


def test_cu_grant_unit_is_one_cu_per_xcd(P):
    """The agent's grant unit (cumask.DeviceCUs: 8 consecutive mask bits) must enable exactly
    one CU on each of the 8 XCDs, i.e. mask bits are XCC-interleaved; two units -> two per
    XCD. (A mask leaving an XCC without CUs is not restrictive, so grants are >= 1 unit.)"""
    import json
    from pathlib import Path

    from nanogpu.agent import cumask

    out = {}
    for units in (1, 2, 4):
        d = cumask.DeviceCUs(256, 8)
        bits = d.grant("t", max(1, (units * 100 + 31) // 32))   # percent giving `units` units
        assert len(bits) == 8 * units, (units, bits)
        recs = P.cu_census(0, cumask.mask_words(bits), 512, 64)
        cus = {(x, (h >> 8) & 0xF, (h >> 12) & 1, (h >> 13) & 7) for x, h in recs}
        per_xcd = {x: sum(1 for c in cus if c[0] == x) for x in range(8)}
        out[units] = per_xcd
    record("cu_grant_census_cus_per_xcd", {str(k): v for k, v in out.items()})
    for units, per_xcd in out.items():
        assert all(v == units for v in per_xcd.values()), out


_CHILD = r'''
import json, os, sys
sys.path.insert(0, os.environ["REPO"])
from nanogpu.native import probe
P = probe(required=True)
r = P.mfma_throughput(0, [], 2048, 1024)
out = {"tflops": r["tflops"]}
from nanogpu.agent import guest
if guest.apply(0):
    import torch
    free, total = torch.cuda.mem_get_info(0)
    ok_small, ok_big = True, True
    try:
        a = torch.empty(int(0.05 * total), dtype=torch.uint8, device="cuda")
        del a
    except torch.OutOfMemoryError:
        ok_small = False
    try:
        b = torch.empty(int(0.30 * total), dtype=torch.uint8, device="cuda")
        del b
    except torch.OutOfMemoryError:
        ok_big = False
    out.update(small_ok=ok_small, big_ok=ok_big)
print(json.dumps(out))
'''


def _child(env_extra: dict) -> dict:
    import os
    import subprocess
    import sys
    from pathlib import Path

    root = Path(__file__).resolve().parent.parent
    env = dict(os.environ, REPO=str(root), **env_extra)
    r = subprocess.run([sys.executable, "-c", _CHILD], env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]
    return json.loads(r.stdout.strip().splitlines()[-1])


def test_device_plugin_env_is_honoured_by_rocr():
    """The container environment the device plugin returns (nanogpu/agent/plugin.py) really
    confines a process: HSA_CU_MASK in the plugin's "<dev>:<cu ranges>" format limits MFMA
    throughput to the granted CUs, and NANO_GPU_MEMORY_FRACTION (applied by
    nanogpu.agent.guest) caps what the PyTorch allocator can take."""
    from nanogpu.agent import cumask

    full = _child({})["tflops"]
    d = cumask.DeviceCUs(256, 8)
    mask = cumask.hsa_cu_mask(0, d.grant("pod/c", 25))
    part = _child({"HSA_CU_MASK": mask, "NANO_GPU_MEMORY_FRACTION": "0.10"})
    record("plugin_env_in_child", {"full_tflops": round(full, 1), "hsa_cu_mask": mask,
                                    "masked_tflops": round(part["tflops"], 1),
                                    "alloc_5pct_ok": part.get("small_ok"), "alloc_30pct_ok": part.get("big_ok")})
    assert 0.15 < part["tflops"] / full < 0.40, (full, part)
    assert part["small_ok"] is True and part["big_ok"] is False


_HEAP_CHILD = r'''
import json, os, sys
sys.path.insert(0, os.environ["REPO"])
import torch
from nanogpu.agent import guest
applied = guest.apply(0) if os.environ.get("APPLY") == "1" else False
free, total = torch.cuda.mem_get_info(0)
out = {"applied": applied, "total_mib": total >> 20}
def fits(mib):
    try:
        x = torch.empty(int(mib) << 20, dtype=torch.uint8, device="cuda")
        del x
        return True
    except RuntimeError:
        return False
    finally:
        torch.cuda.empty_cache()
for k, v in json.loads(os.environ["SIZES"]).items():
    out[k] = fits(v)
if os.environ.get("SUM"):
    blocks, got = [], 0
    try:
        while got < int(os.environ["SUM"]):
            blocks.append(torch.empty(1024 << 20, dtype=torch.uint8, device="cuda"))
            got += 1024
    except RuntimeError:
        pass
    out["sum_mib"] = got
print(json.dumps(out))
'''


def test_hbm_budget_reaches_the_hip_runtime():
    """The device plugin's HBM budget (nanogpu/agent/plugin.py): GPU_MAX_HEAP_SIZE makes the
    HIP runtime report the rounded-up budget as the device's total and refuse any single
    allocation above it, for any HIP program; guest.apply then caps PyTorch's allocator at the
    exact budget, relative to that reported total. What the runtime does NOT do is cap the sum
    of allocations (pinned here, so the README's claim stays true)."""
    import os
    import subprocess
    import sys
    from pathlib import Path

    root = Path(__file__).resolve().parent.parent

    def child(env_extra):
        env = dict(os.environ, REPO=str(root), **env_extra)
        env.pop("PYTORCH_HIP_ALLOC_CONF", None)
        r = subprocess.run([sys.executable, "-c", _HEAP_CHILD], env=env, capture_output=True, text=True, timeout=300)
        assert r.returncode == 0, r.stderr[-3000:]
        return json.loads(r.stdout.strip().splitlines()[-1])

    import torch

    device_mib = torch.cuda.get_device_properties(0).total_memory >> 20
    budget = 16384
    pct = -(-100 * budget // device_mib)
    cap = device_mib * pct // 100
    env = {"GPU_MAX_HEAP_SIZE": str(pct), "NANO_GPU_MEMORY_MIB": str(budget),
           "NANO_GPU_MEMORY_FRACTION": f"{budget / device_mib:.6f}", "APPLY": "1",
           "SIZES": json.dumps({"under_budget": budget * 0.85, "over_budget": budget * 1.05})}
    a = child(env)
    # runtime alone (no allocator cap, caching off: every tensor is its own hipMalloc)
    b = child({"GPU_MAX_HEAP_SIZE": str(pct), "PYTORCH_NO_HIP_MEMORY_CACHING": "1",
               "SIZES": json.dumps({"under_cap": cap * 0.9, "over_cap": cap * 1.1}), "SUM": str(int(1.5 * cap))})
    record("hbm_budget_runtime", {"device_mib": device_mib, "budget_mib": budget, "gpu_max_heap_size": pct,
                                  "reported_total_mib": a["total_mib"], "guest": a, "runtime_only": b})
    assert abs(a["total_mib"] - cap) <= 2 and a["applied"]
    assert a["under_budget"] and not a["over_budget"]            # the exact budget (allocator)
    assert b["under_cap"] and not b["over_cap"]                  # one allocation over the cap
    assert b["sum_mib"] > cap                                    # the sum is not capped


def test_agent_metrics_read_real_amdgpu_sysfs(host, P):
    """The node agent's /metrics reads gpu_busy_percent and VRAM use from the real device; VRAM
    used grows by what a process allocates and the busy counter is a percentage."""
    import re

    import torch

    from nanogpu.agent.metrics import render
    from nanogpu.topology.model import from_host_json

    topo = from_host_json(host)
    minors = [int(g["render_minor"]) for g in host["gpus"]]
    if len(minors) != len(topo.devices):
        pytest.skip("partitioned GPU: render nodes are per partition")

    def used() -> int:
        m = re.search(r'nanogpu_device_vram_used_bytes\{device="0"\} (\d+)', render(topo, None, minors))
        assert m, "mem_info_vram_used not read"
        return int(m.group(1))

    text = render(topo, None, minors)
    busy = re.search(r'nanogpu_device_busy_percent\{device="0"\} (\d+)', text)
    assert busy and 0 <= int(busy.group(1)) <= 100
    mbusy = re.search(r'nanogpu_device_mem_busy_percent\{device="0"\} (\d+)', text)
    print("mem_busy_percent:", mbusy.group(1) if mbusy else "not exposed by this device")
    assert mbusy is None or 0 <= int(mbusy.group(1)) <= 100
    assert f'nanogpu_device_vram_total_bytes{{device="0"}} {host["gpus"][0]["vram_bytes"]}' in text
    import time

    def settled() -> int:
        # device-wide counter: memory of processes that just exited (earlier tests' children)
        # drains asynchronously, so wait until two readings agree
        prev = used()
        for _ in range(50):
            time.sleep(0.1)
            cur = used()
            if abs(cur - prev) < (64 << 20):
                return cur
            prev = cur
        return prev

    # the counter is the whole device's: memory another process frees (or takes) during a
    # reading moves it too (one box run read -40 GB across our 4 GiB allocation). Our 4 GiB
    # must show as a rise on allocation or as a fall on free; up to 3 attempts
    deltas = []
    for _attempt in range(3):
        torch.cuda.synchronize()
        torch.cuda.empty_cache()
        before = settled()
        x = torch.empty(4 << 30, dtype=torch.uint8, device="cuda:0")
        x.fill_(1)
        torch.cuda.synchronize()
        during = settled()
        del x
        torch.cuda.empty_cache()
        torch.cuda.synchronize()
        after = settled()
        deltas.append((during - before, during - after))
        if max(deltas[-1]) >= (3 << 30):
            break
    record("agent_metrics_vram_delta_for_4GiB", deltas[-1][0])
    assert any(max(d) >= (3 << 30) for d in deltas), deltas


def test_hbm_bandwidth_under_cu_mask_sharing(P):
    """CU masks partition compute, not the memory system. Measures (and records for
    profiles/gpu_calibration.md) how HBM3E bandwidth splits between two memory-bound tenants
    holding the agent's 25 % / 75 % masks, and what a 25 % tenant reaches alone."""
    from nanogpu.agent import cumask

    d = cumask.DeviceCUs(256, 8)
    a, b = d.grant("a", 25), d.grant("b", 75)
    ma, mb = cumask.mask_words(a), cumask.mask_words(b)
    full = P.hbm_colocated(0, [[]], 1 << 30, 10)[0]
    alone25 = P.hbm_colocated(0, [ma], 1 << 30, 10)[0]
    ta, tb = P.hbm_colocated(0, [ma, mb], 1 << 30, 10)
    record("hbm_cu_mask_sharing", {"full_gbs": round(full, 1), "alone_25pct_gbs": round(alone25, 1),
                                   "colocated_25pct_gbs": round(ta, 1), "colocated_75pct_gbs": round(tb, 1)})
    assert full > 4000, full
    # every tenant moves data; the pair together cannot beat the device
    assert ta > 0.05 * full and tb > 0.05 * full, (ta, tb, full)
    assert min(ta, tb) < full * 1.05


def test_memory_bound_tenant_pairs_better_with_compute_bound_neighbour(P):
    """What kFlagMemBound buys: a streaming 25 % tenant measured entirely beside (a) a
    streaming 75 % neighbour and (b) an MFMA-bound 75 % neighbour, both neighbours outlasting
    it. Recorded for profiles/gpu_calibration.md."""
    from nanogpu.agent import cumask

    d = cumask.DeviceCUs(256, 8)
    a, b = d.grant("a", 25), d.grant("b", 75)
    ma, mb = cumask.mask_words(a), cumask.mask_words(b)
    alone = P.hbm_colocated(0, [ma], 1 << 30, 10)[0]
    beside_stream = P.hbm_colocated(0, [ma, mb], 1 << 30, 10, [10, 40])[0]
    beside_mfma, mfma_tf = P.mixed_colocated(0, ma, mb, 1 << 30, 10, len(b) * 8, 32768)
    mfma_alone = P.mfma_throughput(0, mb, len(b) * 8, 4096)["tflops"]
    record("memory_bound_pairing", {"stream25_alone_gbs": round(alone, 1),
                                    "stream25_beside_stream75_gbs": round(beside_stream, 1),
                                    "stream25_beside_mfma75_gbs": round(beside_mfma, 1),
                                    "mfma75_beside_stream25_tflops": round(mfma_tf, 1),
                                    "mfma75_alone_tflops": round(mfma_alone, 1)})
    assert beside_mfma > beside_stream, (alone, beside_stream, beside_mfma)


def test_agent_selftest_passes_on_the_real_device(host, P):
    """The node agent's active self-test (HBM copy bit-exact + one MFMA tile against a host
    reference) on the real MI355X."""
    import asyncio

    from nanogpu.agent.node import NodeAgent, gpu_selftest
    from nanogpu.topology.model import from_host_json

    assert gpu_selftest(P, 0)
    topo = from_host_json(host)
    agent = NodeAgent(api=None, node_name="box", topo=topo, device_plugin=False)
    failed = asyncio.run(agent.selftest(P)) if len(topo.devices) == P.device_count() else []
    assert failed == [], failed


@pytest.fixture(scope="module")
def busy(host, P):
    """mem_busy_percent, every 10 ms sample averaged (what avg_over_time computes), while one
    tenant runs alone for 6 s: the full chip streaming HBM and burning MFMA, and the shares the
    learner has to tell apart, a 25 % streamer and a 75 % MFMA tenant."""
    from nanogpu.probe import calibrate as C

    f = C.mem_busy_file(host)
    if f is None:
        pytest.skip("mem_busy_percent not exposed")
    runs = [(label, C.tenant_call(P, kind, C.cu_share_mask(share)))
            for label, kind, share in (("stream100", "stream", 100), ("mfma100", "mfma", 100),
                                       ("stream25", "stream", 25), ("mfma75", "mfma", 75))]
    res = {r["label"]: r for r in C.mem_busy_while(f, runs, seconds=6.0)}
    record("mem_busy_percent_by_tenant", res)
    print(json.dumps(res, indent=1))
    return res


def test_streaming_tenant_drives_mem_busy_percent_over_the_hot_threshold(busy):
    """The signal behind Device::mem_hot: while the HBM copy streams on the whole GPU, the mean
    of every sample of amdgpu's mem_busy_percent (exported by the agent as
    nanogpu_device_mem_busy_percent and polled as gpu_hbm_activity_avg), and the mean of
    samples 1 s apart like scrapes, are at or above types.HBM_HOT_THRESHOLD. (Samples 5 s
    apart are one reading in a 6 s run: a single instantaneous value, 19 % on one box whose
    mean was 33 %, says nothing about the average the poller reads.)"""
    from nanogpu import types as T

    s = busy["stream100"]
    assert s["rate"] > 1000, s                      # GB/s: the copy really streamed
    assert s["mean_all"] >= 100 * T.HBM_HOT_THRESHOLD, s
    assert s["mean_1s"] >= 100 * T.HBM_HOT_THRESHOLD, s


def test_compute_bound_tenant_stays_under_the_hot_threshold(busy):
    """The other side: an MFMA-bound tenant (bf16 burn, almost no HBM traffic) keeps the same
    averages below types.HBM_HOT_THRESHOLD, so a busy compute tenant is not mistaken for a
    streaming one."""
    from nanogpu import types as T

    m = busy["mfma100"]
    assert m["rate"] > 500, m                       # TFLOP/s: the burn really ran
    assert m["mean_all"] < 100 * T.HBM_HOT_THRESHOLD, m
    assert m["mean_1s"] < 100 * T.HBM_HOT_THRESHOLD, m


def test_share_aware_learner_learns_a_lone_25pct_streamer_not_a_lone_75pct_mfma_tenant(busy):
    """The learner's threshold depends on the lone pod's share (types.HBM_STREAMING_CURVE,
    PolicySpec.learn_curve): the measured averages of a 25 % streaming tenant and of a 75 %
    MFMA tenant, each alone on its device, are written to the ledger as the poller would, and
    only the streamer's owner is learned."""
    from nanogpu import _native as N
    from nanogpu.config.policy import PolicySpec
    from nanogpu.topology.model import synthetic_mi355x

    t = synthetic_mi355x(2)
    L = N.Ledger("", 4, 64, True)
    nid = L.upsert_node("n0", t.ledger_devices(True), t.ledger_topo())
    assert L.allocate_plan(nid, "streamer", [(25, 0)], [[0]], True) == N.OK
    assert L.allocate_plan(nid, "mfma", [(75, 0)], [[1]], True) == N.OK
    L.set_pod_owner("streamer", "rs-stream")
    L.set_pod_owner("mfma", "rs-mfma")
    L.set_mem_busy(nid, 0, int(round(busy["stream25"]["mean_all"])))
    L.set_mem_busy(nid, 1, int(round(busy["mfma75"]["mean_all"])))
    curve = PolicySpec().learn_curve()
    assert L.learn_stream_owners(True, N.mono_now(), 3, curve) == (1, 0)
    assert L.is_stream_owner("rs-stream") and not L.is_stream_owner("rs-mfma")


@pytest.fixture(scope="module")
def busy_cal(host, P):
    """This device's own mem_busy scale (the agent's --calibrate: the probe's stream alone at
    25 % and 100 % of the CUs, every 10 ms sample averaged), then a 25 % streamer and a 75 % MFMA
    tenant alone for 16 s each, sampled as the original assertion did (readings 5 s apart)."""
    from nanogpu.probe import calibrate as C

    f = C.mem_busy_file(host)
    if f is None:
        pytest.skip("mem_busy_percent not exposed")
    cal = C.hbm_busy_calibration(P, 0, f, seconds=3.0)
    runs = [(label, C.tenant_call(P, kind, C.cu_share_mask(share)))
            for label, kind, share in (("stream25", "stream", 25), ("mfma75", "mfma", 75))]
    res = {r["label"]: r for r in C.mem_busy_while(f, runs, seconds=16.0)}
    record("mem_busy_calibration", {"cal": cal, "tenants": res})
    print(json.dumps({"cal": cal, "tenants": res}, indent=1))
    return cal, res


def test_calibrated_hbm_classifier_on_5s_samples(busy_cal):
    """with this device's own calibration the classifier tells a quarter-GPU
    streamer (hot) from a 75 % MFMA tenant (not) on samples 5 s apart, on a box whose scale is
    not the calibration box's (one read 20.7 / 28.7 % where the constants' box read 30.1 / 54.4)."""
    from nanogpu import types as T
    from nanogpu.telemetry.store import normalize_hbm_activity as norm

    cal, res = busy_cal
    assert len(cal) == 2 and all(b > 0 for _, b in cal), cal
    assert cal[0][1] < cal[1][1], cal                 # a quarter of the CUs streams less than all
    s, m = res["stream25"], res["mfma75"]
    assert s["rate"] > 500 and m["rate"] > 300, (s, m)   # GB/s, TFLOP/s: both tenants really ran
    assert s["mean_5s"] is not None and m["mean_5s"] is not None, (s, m)
    assert norm(s["mean_5s"] / 100, cal) >= T.HBM_HOT_THRESHOLD, (cal, s)
    assert norm(m["mean_5s"] / 100, cal) < T.HBM_HOT_THRESHOLD, (cal, m)
    # and the averages the poller converges to
    assert norm(s["mean_all"] / 100, cal) >= T.HBM_HOT_THRESHOLD > norm(m["mean_all"] / 100, cal)


_RCCL_SCRIPT = r"""
import json, os, sys
import torch
import torch.distributed as dist
sys.path.insert(0, os.environ["NANOGPU_ROOT"])
from datetime import timedelta
from nanogpu.probe.calibrate import link_matrix, ring_busbw, ring_busbw_bounded
torch.cuda.set_device(0)
dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", 0))
out = {"backend": dist.get_backend()}
out["busbw"] = ring_busbw(dist, "cuda:0", nbytes=64 << 20, iters=3)   # one rank: 0 by definition
# the bench's calibration: a gloo group for agreement, the ring on a communicator of its own
cal = dist.new_group(backend="gloo", timeout=timedelta(seconds=60))
out["busbw_bounded"] = list(ring_busbw_bounded(dist, "cuda:0", cal, timeout_s=60, nbytes=64 << 20, iters=3))
t = torch.full((1 << 20,), 2.0, dtype=torch.bfloat16, device="cuda:0")
dist.all_reduce(t)
out["allreduce_ok"] = bool((t == 2.0).all().item())
out["matrix"] = link_matrix(1, dist=dist, rank=0, group=cal)           # the all-gathered rows
dist.barrier(device_ids=[0])
got = [None]
dist.all_gather_object(got, {"rank": 0})
lst = ["url"]
dist.broadcast_object_list(lst, src=0)
out["objects"] = [got[0]["rank"], lst[0]]
dist.destroy_process_group()
print(json.dumps(out))
"""


def test_rccl_paths_of_the_multi_rank_bench_run_on_the_device(tmp_path):
    """The collectives a driver N-GPU bench run uses (torch.distributed backend "nccl" = RCCL
    on ROCm): RCCL all-reduce (ring_busbw), the peer-matrix all-gather, the device barrier and
    the object collectives, on the box's one MI355X with a one-rank group. A 2-rank group
    needs two GPUs (RCCL refuses two ranks on one device)."""
    import os
    import subprocess
    import sys
    from pathlib import Path

    root = Path(__file__).resolve().parent.parent
    env = dict(os.environ, NANOGPU_ROOT=str(root), MASTER_ADDR="127.0.0.1", MASTER_PORT="29613",
               HSA_ENABLE_IPC_MODE_LEGACY="0")
    r = subprocess.run([sys.executable, "-c", _RCCL_SCRIPT], capture_output=True, text=True, timeout=180, env=env)
    assert r.returncode == 0, (r.stdout + r.stderr)[-3000:]
    out = json.loads(r.stdout.strip().splitlines()[-1])
    record("rccl_one_rank", out)
    assert out["backend"] == "nccl" and out["allreduce_ok"]
    assert out["busbw"] == 0.0 and out["matrix"] == [[0.0]] and out["objects"] == [0, "url"]
    assert out["busbw_bounded"] == [0.0, ""]
