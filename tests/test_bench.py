"""bench.py contract (single rank and 2- and 4-rank gloo jobs) and the BASELINE config harness."""
import asyncio
import json
import statistics
import os
import socket
import subprocess
import tempfile
import sys
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parent.parent
KEYS = {"metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better", "scaling",
        "vs_baseline", "dtype", "data", "config"}


def _free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _last_json(out: str) -> dict:
    lines = [ln for ln in out.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, out[-3000:]
    # the driver keeps the last 8 KB of stdout: the whole line fits, headline keys last
    assert len(lines[0]) < 4096, len(lines[0])
    d = json.loads(lines[0])
    assert list(d)[-4:] == ["p99_bind_ms", "p50_bind_ms", "pods_per_s_first_filter_to_last_bind", "value"]
    assert "frag_pct" in list(d)[-8:] and "extender_cpu_us_per_pod_rank0" in list(d)[-10:]
    assert "step_diag_rank0" not in d
    return d


def test_bench_single_rank_cpu(tmp_path, cpu_exclusive):
    full = tmp_path / "full.json"
    r = subprocess.run([sys.executable, str(ROOT / "bench.py"), "--no-gpu", "--steps", "2", "--warmup", "1",
                        "--pods", "200", "--nodes", "8", "--steady-variant-steps", "2", "--nodes-variant", "120",
                        "--nodes-variant-steps", "1", "--json-out", str(full)],
                       capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]
    d = _last_json(r.stdout)
    diag = json.loads(full.read_text())["diagnostics"]
    assert len(diag["step_diag_rank0"]) == 2
    assert KEYS <= set(d)
    assert d["n_gpus"] == 1 and d["steps"] == 2 and d["warmup"] == 1 and d["higher_is_better"] is True
    assert d["scheduled"] == 400 and d["failed"] == 0 and d["value"] > 0
    assert d["p50_bind_ms"] is not None and 0 <= d["frag_pct"] <= 100
    # steady-state churn pass: live frag next to the reference algorithm on the same stream
    assert d["value_steady"] > 0 and d["failed_steady"] == 0
    assert d["frag_pct_steady"] is not None and d["frag_pct_steady_reference_model"] is not None
    # 120 nodes behind kube-scheduler's sampling: 100 feasible nodes reach the extender
    assert d["value_nodes120"] > 0 and d["failed_nodes120"] == 0 and d["pods_per_burst_nodes120"] == 3000
    # (a pod that found no host in a cycle is retried over the nodes that were feasible then)
    # (binpack fills nodes to kube-scheduler's resource fit, so late in a burst fewer than 100
    # nodes are feasible in a cycle)
    assert 80.0 <= d["nodes_sent_per_filter_nodes120"] <= 100.0
    assert d["value_mode"] == "one kube-scheduler stand-in" and "value_independent_schedulers" not in d
    assert d["frag_pct_nodes120_reference_model"] is not None
    # extender CPU a pod: by thread group, and split into user / kernel time
    assert d["extender_cpu_us_per_pod_rank0"] > 0 and "ngpu-fe" in diag["extender_cpu_us_per_pod_by_thread_rank0"]
    user, kernel = diag["extender_cpu_us_per_pod_user_kernel_rank0"]
    assert user >= 0 and kernel >= 0 and user + kernel > 0
    # every native bind split by hop: p50 <= p99 per hop; the median binds' hops add up to about
    # the front door's median wall (each hop's median is taken alone, so only roughly)
    hops = d["bind_hops_us"]
    assert list(hops) == ["reserve", "handoff", "window", "send", "api", "commit", "reply"] and d["bind_tail_hop"] in hops
    assert all(len(v) == 3 and 0 <= v[0] <= v[1] for v in hops.values())
    assert 0.2 * d["p50_bind_frontdoor_ms"] <= sum(v[0] for v in hops.values()) / 1e3 <= 3 * d["p50_bind_frontdoor_ms"]


@pytest.mark.parametrize("binds", [False, True])
def test_bench_spin_recv_catches_requests_on_the_hot_connection(binds, tmp_path, cpu_exclusive):
    # a 500 us window: on this host too kube-scheduler's next request lands inside it
    full = tmp_path / "full.json"
    r = subprocess.run([sys.executable, str(ROOT / "bench.py"), "--no-gpu", "--steps", "2", "--warmup", "1",
                        "--pods", "200", "--nodes", "8", "--steady-variant-steps", "0", "--nodes-variant", "0",
                        "--rtt-variant-ms", "0", "--inproc-variant-steps", "0", "--busy-poll-us", "500",
                        "--spin-recv", "--io-tally", "--json-out", str(full)] + (["--spin-recv-binds"] if binds else []),
                       capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]
    d = _last_json(r.stdout)
    assert d["scheduled"] == 400 and d["failed"] == 0
    io = json.loads(full.read_text())["diagnostics"]["io_per_pod_rank0"]
    # probes ran, and requests found by them skipped the reader's recv (3 exchanges a pod)
    assert io["fe_spin_recv"][0] > 0
    assert io["fe_recv"][0] < 3.0


@pytest.mark.parametrize("ranks", [2, 4])
def test_bench_multi_rank_gloo(ranks, tmp_path, cpu_exclusive):
    full = tmp_path / "full.json"
    env = dict(os.environ, MASTER_ADDR="127.0.0.1")
    r = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", str(ranks),
                        "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), str(ROOT / "bench.py"),
                        "--gpus", str(ranks), "--no-gpu", "--steps", "2", "--warmup", "1", "--pods", "200",
                        "--nodes", "8", "--rtt-variant-steps", "1", "--steady-variant-steps", "2",
                        "--nodes-variant", "16", "--nodes-variant-steps", "1", "--independent-variant-steps", "1",
                        "--json-out", str(full)],
                       capture_output=True, text=True, timeout=400, env=env, cwd="/tmp")
    assert r.returncode == 0, r.stderr[-3000:]
    d = _last_json(r.stdout)
    diag = json.loads(full.read_text())["diagnostics"]
    assert d["n_gpus"] == ranks and d["scheduled"] == 400 and d["failed"] == 0
    assert f"{ranks} extender worker" in d["config"]["parallelism"]
    assert d["value_rtt2ms"] and d["p50_bind_ms"] is not None
    assert d["value_steady"] > 0 and d["failed_steady"] == 0
    # placement-quality passes run the deployment that exists: one kube-scheduler for the job
    assert diag["steady_config"].endswith("one kube-scheduler stand-in, binds over every rank's worker")
    assert d["schedulers_nodes16"].startswith("one kube-scheduler") and d["failed_nodes16"] == 0
    # the headline is the deployment that exists: one kube-scheduler, binds over N workers;
    # N independent stand-ins are a labelled side figure
    assert d["value_mode"] == f"one kube-scheduler stand-in, binds over all {ranks} extender workers"
    assert d["value_independent_schedulers"] > 0 and d["steps_independent_schedulers"] == 1
    # binds the cycle's worker did not see stay native on the other workers (ledger handoff)
    assert d["bind_handoffs"] > 0


def test_plain_gpus_n_starts_n_ranks_itself(tmp_path, cpu_exclusive):
    """`python bench.py --gpus 4` without torchrun must not measure one rank.
    The launcher starts torch.distributed.run as a child (no GPU touched with --no-gpu) and the
    line reports the 4-worker job."""
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "LOCAL_WORLD_SIZE")}
    r = subprocess.run([sys.executable, str(ROOT / "bench.py"), "--gpus", "4", "--no-gpu", "--steps", "1",
                        "--warmup", "1", "--pods", "200", "--nodes", "8", "--rtt-variant-ms", "0",
                        "--steady-variant-steps", "0", "--nodes-variant", "0", "--inproc-variant-steps", "0",
                        "--independent-variant-steps", "0"],
                       capture_output=True, text=True, timeout=400, env=env, cwd="/tmp")
    assert r.returncode == 0, r.stderr[-3000:]
    assert len(r.stdout.strip().splitlines()) == 1, r.stdout[:2000]   # the JSON line alone (gloo's chatter: stderr)
    d = _last_json(r.stdout)
    assert d["n_gpus"] == 4 and d["config"]["parallelism"].startswith("4 extender worker")
    assert d["value_mode"] == "one kube-scheduler stand-in, binds over all 4 extender workers"
    assert d["scheduled"] == 200 and d["failed"] == 0


def _host_steal() -> tuple[int, int]:
    """(steal, total) jiffies of the host's CPUs (/proc/stat): what the hypervisor took."""
    with open("/proc/stat") as f:
        v = [int(x) for x in f.readline().split()[1:9]]
    return v[7], sum(v)


@pytest.mark.parametrize("ranks", [2, 4])
def test_one_scheduler_over_n_workers_does_the_one_worker_cycle_work(ranks, cpu_exclusive):
    """one kube-scheduler's binds spread over N extender workers (the
    driver's N-GPU headline) leave the scheduling cycle's worker the work it has with one: the
    same verbs, sends, pod-cache puts, nominations and ledger scans / memo re-validations a pod
    (`--io-tally` counts, exact to the stream), no bind through Python, and binds answered by the
    other workers through the ledger's handoff. The cycle stays on rank 0's worker; the handoff
    is published after its filter answer (Frontend::run_deferred) and a bind adopts its
    nomination under the pod shard's lock only, so neither sits on the cycle.
    The rate itself, >= 0.9x the 1-worker rate at 4 workers, is asserted in the GPU tier
    (test_one_scheduler_over_four_workers_keeps_the_rate_on_the_box) because this container
    cannot time it: it is a VM whose hypervisor takes CPU time (steal) in proportion to the
    vCPUs a job keeps busy, 0.6-1.2 % during a 1-worker run and 4-9 % during a 4-worker one;
    single runs of one build swing 3x (4-13k pods/s) and interleaved 1/N pair ratios 0.56-1.84.
    Here the rate gets a floor only for gross breakage (0.5x, fastest steps)."""
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "LOCAL_WORLD_SIZE")}
    base = ["--no-gpu", "--steps", "8", "--warmup", "2", "--rtt-variant-ms", "0", "--io-tally",
            "--steady-variant-steps", "0", "--nodes-variant", "0", "--inproc-variant-steps", "0",
            "--independent-variant-steps", "0", "--decisive-variant-steps", "0"]
    io, rate = {}, {}
    with tempfile.TemporaryDirectory() as tmp:
        for n in (1, ranks):
            out = Path(tmp) / f"r{n}.json"
            r = subprocess.run([sys.executable, str(ROOT / "bench.py"), "--gpus", str(n), "--json-out", str(out)]
                               + base, capture_output=True, text=True, timeout=400, env=env, cwd="/tmp")
            assert r.returncode == 0, r.stderr[-3000:]
            d = _last_json(r.stdout)
            assert d["n_gpus"] == n and d["failed"] == 0 and d["scheduled"] == 8000
            diag = json.loads(out.read_text())["diagnostics"]
            assert diag["python_requests_per_pod_rank0"] == 0.0   # every bind stayed native
            if n > 1:
                assert d["bind_handoffs"] > 0 and d["value_mode"].startswith("one kube-scheduler stand-in")
            io[n] = {k: v[0] for k, v in diag["io_per_pod_rank0"].items()}
            spans = diag["schedule_ms_each_step_rank0"]
            rate[n] = 1e3 * d["scheduled"] / len(spans) / min(spans)
    one, many = io[1], io[ranks]
    for k in ("fe_verb", "fe_send_cycle", "fe_verb_assume", "fe_verb_pod"):
        assert one[k] == many[k] == 2.0, (k, one[k], many[k])
    assert one["fe_verb_cache"] == many["fe_verb_cache"] == 3.0   # filter put (+ handoff), 2 verb lookups
    assert one["fe_verb_nominate"] == pytest.approx(1.0, abs=0.01) and many["fe_verb_nominate"] == pytest.approx(1.0, abs=0.01)
    for k in ("ledger_scan", "ledger_revalidate"):   # the memo's work a pod: same stream, same placements
        assert many[k] == pytest.approx(one[k], rel=0.1), (k, one[k], many[k])
    assert many["fe_verb_names"] < 2.1   # node lists resolved from the per-list cache
    assert rate[ranks] >= 0.5 * rate[1], rate


@pytest.mark.gpu
def test_one_scheduler_over_four_workers_keeps_the_rate_on_the_box():
    """The 0.9x bar of the test above, read where the job owns its CPUs: the GPU box (16 CPUs
    of its own, an L3 domain a rank). It runs in the GPU tier for those CPUs, not for the GPU:
    the ranks are gloo ranks with --no-gpu, as in profiles/scaling_rehearsal.md (r06f: 1.03x)."""
    med, info = _rate_pairs(4, 0.9, max_pairs=5, steps=16)
    assert med >= 0.9, info


def _rate_pairs(ranks: int, floor: float, max_pairs: int, steps: int) -> tuple[float, dict]:
    """1-worker and `ranks`-worker bench runs in interleaved pairs until the median of the pairs'
    rate ratios reaches `floor` (3 pairs at least) or `max_pairs` ran: (median, the record)."""
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "LOCAL_WORLD_SIZE")}
    base = ["--no-gpu", "--steps", str(steps), "--warmup", "2", "--rtt-variant-ms", "0",
            "--steady-variant-steps", "0", "--nodes-variant", "0", "--inproc-variant-steps", "0",
            "--independent-variant-steps", "0", "--decisive-variant-steps", "0"]
    got = {1: [], ranks: []}
    steal = {1: [], ranks: []}
    ratios: list[float] = []
    with tempfile.TemporaryDirectory() as tmp:
        for rnd in range(max_pairs):
            for n in (1, ranks):
                out = Path(tmp) / f"r{n}_{rnd}.json"
                s0 = _host_steal()
                r = subprocess.run([sys.executable, str(ROOT / "bench.py"), "--gpus", str(n), "--json-out", str(out)]
                                   + base, capture_output=True, text=True, timeout=400, env=env, cwd="/tmp")
                s1 = _host_steal()
                assert r.returncode == 0, r.stderr[-3000:]
                d = _last_json(r.stdout)
                assert d["n_gpus"] == n and d["failed"] == 0
                if n > 1:
                    assert d["bind_handoffs"] > 0 and d["value_mode"].startswith("one kube-scheduler stand-in")
                diag = json.loads(out.read_text())["diagnostics"]
                assert diag["python_requests_per_pod_rank0"] == 0.0   # every bind stayed native
                spans = diag["schedule_ms_each_step_rank0"]
                got[n].append(round(1e3 * d["scheduled"] / len(spans) / min(spans), 1))
                steal[n].append(round(100 * (s1[0] - s0[0]) / max(1, s1[1] - s0[1]), 1))
            ratios.append(got[ranks][-1] / got[1][-1])
            if len(ratios) >= 3 and statistics.median(ratios) >= floor:
                break
    med = statistics.median(ratios)
    print(f"{ranks} workers: median ratio {med:.3f}", {"rates": got, "steal_pct": steal})
    return med, {"rates": got, "ratios": [round(x, 3) for x in ratios], "steal_pct": steal}


def test_plain_gpus_n_refuses_when_fewer_gpus_are_visible(tmp_path):
    """`--gpus 2` on the real box's one-GPU sysfs view exits non-zero before starting ranks."""
    env = {k: v for k, v in os.environ.items() if k != "WORLD_SIZE"}
    real = ROOT / "tests/fixtures/sysfs/mi355x_real"
    r = subprocess.run([sys.executable, str(ROOT / "bench.py"), "--gpus", "2", "--steps", "1", "--warmup", "0",
                        "--sysfs-root", str(real)],
                       capture_output=True, text=True, timeout=120, env=env, cwd="/tmp")
    assert r.returncode == 2, (r.returncode, r.stderr[-2000:])
    assert "needs 2 visible GPUs; 1 visible" in r.stderr and not r.stdout.strip()


def test_visible_gpu_count_applies_the_visibility_variables(tmp_path):
    from nanogpu.topology.fixtures import write_mi355x_sysfs
    from nanogpu.topology.visible import visible_gpu_count

    write_mi355x_sysfs(tmp_path / "spx", 8, "SPX")
    write_mi355x_sysfs(tmp_path / "cpx", 8, "CPX")
    spx, cpx = str(tmp_path / "spx"), str(tmp_path / "cpx")
    assert visible_gpu_count(spx, env={}) == 8
    assert visible_gpu_count(cpx, env={}) == 64          # HIP enumerates every partition
    assert visible_gpu_count(spx, env={"HIP_VISIBLE_DEVICES": "0,3"}) == 2
    assert visible_gpu_count(spx, env={"CUDA_VISIBLE_DEVICES": "5"}) == 1
    assert visible_gpu_count(spx, env={"ROCR_VISIBLE_DEVICES": "0,1,2", "HIP_VISIBLE_DEVICES": "0,1,2,3"}) == 3
    assert visible_gpu_count(spx, env={"HIP_VISIBLE_DEVICES": "1,9,2"}) == 1   # stops at an invalid ordinal
    assert visible_gpu_count(spx, env={"HIP_VISIBLE_DEVICES": ""}) == 8   # set but empty: unset
    assert visible_gpu_count(spx, env={"ROCR_VISIBLE_DEVICES": "GPU-aa,GPU-bb"}) == 2
    assert visible_gpu_count(str(ROOT / "tests/fixtures/sysfs/mi355x_real"), env={}) == 1
    assert visible_gpu_count(str(tmp_path / "none"), env={}) == 0


def test_hop_summary_names_the_hop_that_owns_the_tail():
    import importlib.util

    spec = importlib.util.spec_from_file_location("bench_mod", ROOT / "bench.py")
    bench = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(bench)
    assert bench.hop_summary([]) is None
    rows = [[1000, 2000, 0, 3000, 40000, 500, 4000]] * 990 + [[1000, 2000, 0, 3000, 40000, 500, 300000]] * 10
    h = bench.hop_summary(rows)
    assert h["n"] == 1000 and h["tail_hop"] == "reply"
    assert h["us"]["api"] == [40.0, 40.0, 40.0] and h["us"]["reply"] == [4.0, 300.0, 300.0]
    # binds held for room in the admission window (the API server's backpressure) own their tail
    rows = [[1000, 2000, 0, 3000, 40000, 500, 4000]] * 990 + [[1000, 2000, 900000, 3000, 40000, 500, 4000]] * 10
    assert bench.hop_summary(rows)["tail_hop"] == "window"


def test_link_weights_fall_back_to_the_reader_and_a_matrix_sets_the_mesh():
    import importlib.util

    spec = importlib.util.spec_from_file_location("bench_mod", ROOT / "bench.py")
    bench = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(bench)
    d = bench.Dist(1)                          # no GPU: no probe
    host = {"gpus": [{"xgmi_min_bw_mbs": 76000}]}
    link, m, src = bench.measured_links(d, host, 8)
    assert link == 76.0 and m is None and "kfd io_link" in src
    link, m, src = bench.measured_links(d, {"gpus": [{}]}, 8)
    assert link == 153.0 and src.startswith("placeholder")
    from nanogpu.topology.model import synthetic_mi355x

    mat = [[0.0, 70.0, 60.0], [50.0, 0.0, 65.0], [61.0, 64.0, 0.0]]
    t = synthetic_mi355x(3, link_matrix=mat)
    assert t.link_bw[0][1] == t.link_bw[1][0] == 50.0 and t.link_bw[1][2] == 64.0 and t.link_bw[0][0] == 0.0


def test_config_harness_plumbing_and_topology():
    from nanogpu.sim import configs as C

    async def main():
        c1 = await C._both(C.config1)()
        for k in ("ours", "reference_model"):
            assert c1[k]["scheduled"] == 1 and c1[k]["placement"] == "0" and c1[k]["status_free"] == 80
        c4 = await C._both(C.config4)()
        o, f = c4["ours"], c4["reference_model"]
        assert o["share_pod"]["distinct_gpus"] == 4
        # the reference ignores links: it can put two ranks across the degraded GPU0-GPU1 link
        assert o["share_pod"]["min_link_gbs"] >= f["share_pod"]["min_link_gbs"]
        assert o["share_pod"]["min_link_gbs"] > 38.0
        assert o["whole_gpu_group"]["scheduled"] == 1 and o["whole_gpu_group"]["min_link_gbs"] > 38.0
        assert o["cpx_share_pod"]["distinct_gpus"] == 4
        c2 = await C.config2(gpus=1)
        assert c2["burst"]["scheduled"] == 5 and c2["hbm_probe"]["overcommitted_gib"] == 0
        c2r = await C.config2(gpus=1, reference=True)
        assert c2r["hbm_probe"]["overcommitted_gib"] > 0

    asyncio.run(main())


def test_config5_sriov_guests_churn():
    """SR-IOV guest VMs (virtual functions, no xGMI or NUMA visible): churn schedules every
    pod and the HBM dimension keeps every VF within its VRAM."""
    from nanogpu.sim import configs as C
    from nanogpu.topology.model import NodeTopology, synthetic_sriov_guest

    t = synthetic_sriov_guest(4)
    assert t.virtualization == "GUEST" and NodeTopology.from_json(t.to_json()).virtualization == "GUEST"
    assert all(g.numa == -1 for g in t.gpus) and not any(any(row) for row in t.link_bw)
    r = asyncio.run(C.config5(rounds=5, pods_n=125, sriov=True))
    assert r["scheduled"] == 125 and r["max_hbm_overcommitted_gib"] == 0


def test_bench_steady_main_pass_two_ranks_share_placements(cpu_exclusive):
    """`--steady` as the main pass with 2 independent stand-ins: each stand-in's kube-scheduler
    cache gets the other rank's placements after every step (bench.py one_step_steady)."""
    env = dict(os.environ, MASTER_ADDR="127.0.0.1")
    r = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
                        "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), str(ROOT / "bench.py"),
                        "--gpus", "2", "--no-gpu", "--steady", "--steps", "2", "--warmup", "1", "--pods", "200",
                        "--nodes", "8", "--rtt-variant-steps", "0", "--inproc-variant-steps", "0",
                        "--nodes-variant", "0", "--independent-variant-steps", "0", "--independent-schedulers"],
                       capture_output=True, text=True, timeout=400, env=env, cwd="/tmp")
    assert r.returncode == 0, r.stderr[-3000:]
    d = _last_json(r.stdout)
    assert d["value"] > 0 and d["failed"] == 0 and d["scheduled"] > 0
    assert d["value_mode"].startswith("2 independent kube-scheduler stand-ins")


def test_bench_multi_rank_survives_a_hung_peer_probe(cpu_exclusive):
    """One GPU pair's peer copy never completes (a stand-in probe): every rank gives up on it
    within the pair's time box, they agree, the node model falls back to the KFD / placeholder
    link rate with the timeout named in `link_bw_source`, and the bench finishes."""
    env = dict(os.environ, MASTER_ADDR="127.0.0.1")
    r = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "4",
                        "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), str(ROOT / "bench.py"),
                        "--gpus", "4", "--no-gpu", "--steps", "1", "--warmup", "1", "--pods", "100",
                        "--nodes", "8", "--rtt-variant-ms", "0", "--steady-variant-steps", "0", "--nodes-variant", "0",
                        "--inproc-variant-steps", "0", "--independent-variant-steps", "0",
                        "--probe-standin", "hang:1-2", "--probe-pair-timeout", "1"],
                       capture_output=True, text=True, timeout=300, env=env, cwd="/tmp")
    assert r.returncode == 0, r.stderr[-3000:]
    d = _last_json(r.stdout)
    src = d["gpu"]["link_bw_source"]
    assert "ProbeTimeout" in src and "1->2" in src, src
    assert d["gpu"]["link_bw_gbs"] == 153.0 and d["scheduled"] == 100 and d["failed"] == 0


def test_steady_churn_frag_is_the_same_at_1_2_and_4_workers(tmp_path, cpu_exclusive):
    """steady-churn frag must not grow with extender workers. One kube-scheduler
    (the stand-in) drives the headline's steady pass (1,000 pods on 64 nodes, 30 % replaced a
    step), its binds over 1, 2 and 4 workers. The cause was the bind landing after the next
    filters (tests/test_lag.py); with the priorities lead (nanogpu.types.PRIORITY_LEAD) every pod
    is held where it binds from its priorities answer on, so the frag of every step is the same
    at every worker count and equals the offline replay of the extender's verbs. No skip, no
    retry: timing no longer enters."""
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "LOCAL_WORLD_SIZE")}
    got = {}
    for n in (1, 2, 4):
        full = tmp_path / f"w{n}.json"
        r = subprocess.run([sys.executable, str(ROOT / "bench.py"), "--gpus", str(n), "--no-gpu", "--steps", "1",
                            "--warmup", "1", "--rtt-variant-ms", "0", "--steady-variant-steps", "6",
                            "--nodes-variant", "0", "--inproc-variant-steps", "0", "--independent-variant-steps", "0",
                            "--decisive-variant-steps", "0", "--json-out", str(full)],
                           capture_output=True, text=True, timeout=600, env=env, cwd="/tmp")
        assert r.returncode == 0, r.stderr[-3000:]
        d = _last_json(r.stdout)
        diag = json.loads(full.read_text())["diagnostics"]
        assert d["failed_steady"] == 0
        if n > 1:
            assert diag["steady_config"].endswith("one kube-scheduler stand-in, binds over every rank's worker")
            assert d["bind_handoffs_steady"] > 0
        nom = diag["nominations_steady"]
        assert nom["moved"] == 0 and nom["adopted"] == nom["made"] > 0
        got[n] = (d["frag_pct_steady"], diag["frag_pct_steady_each_step"], diag["frag_pct_steady_native_replay_each_step"])
    for n in (2, 4):
        assert got[n][0] <= 1.2 * got[1][0], got
        assert got[n][1] == got[1][1], got
    assert got[1][1] == got[1][2], got    # the live run is the replay, step for step
    assert got[1][0] < 1.0   # the reference algorithm reads 3.80 on this stream


def test_launcher_forwards_a_term_to_its_ranks(tmp_path):
    """A timeout that TERMs `python bench.py --gpus 2` must not orphan the rank job it started."""
    import signal
    import time

    env = {k: v for k, v in os.environ.items() if k != "WORLD_SIZE"}
    p = subprocess.Popen([sys.executable, str(ROOT / "bench.py"), "--gpus", "2", "--no-gpu", "--steps", "50",
                          "--warmup", "1", "--pods", "1000"], stdout=subprocess.PIPE, stderr=subprocess.PIPE,
                         env=env, cwd="/tmp", start_new_session=True)
    try:
        time.sleep(8)                      # the ranks are up (torch imported, extenders started)
        p.send_signal(signal.SIGTERM)      # to the launcher only
        p.wait(timeout=60)
        time.sleep(2)
        # nothing of the job is left in the launcher's session
        left = subprocess.run(["pgrep", "-s", str(p.pid)], capture_output=True, text=True).stdout.split()
        assert not left, left
    finally:
        if p.poll() is None:
            os.killpg(p.pid, signal.SIGKILL)
