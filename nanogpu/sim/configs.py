"""BASELINE.json configs 1-5, each run on this framework and on a reference model.

The reference publishes no numbers and no Go toolchain is available, so the
"reference" column is this same harness driving a *reference model*:
  * placement: `compat` mode (bit-exact Go 1.16 reference algorithm, pinned against the
    oracle in tests/test_parity.py) without the HBM dimension (the reference has none);
  * concurrency: one mutex held across filter, score and the whole of bind including its
    API writes, plus the pod GET before bind (reference dealer.go:90-203, bind.go:61-82);
  * the Python (aiohttp) front door.
The reference's controller sleeps ~1 s per processed item (controller.go:185, 256-261;
SURVEY D4); that release lag is reported analytically, not simulated, which flatters the
reference under churn. Both columns use the same fake API server, RTT model and pod stream.

Usage: python -m nanogpu.sim.configs [--out profiles/bench_configs.json] [--quick]
"""
from __future__ import annotations

import argparse
import asyncio
import json
import random
import statistics
import time
from pathlib import Path

from .. import types as T
from ..app import Config, Runtime
from ..extender import server as S
from ..k8s import podutil as pu
from ..k8s.fake_apiserver import Faults, FakeKubeStore, InProcKube, serve
from ..topology.model import NodeTopology, synthetic_mi355x, synthetic_sriov_guest
from .driver import FastExtenderClient, NativeSchedulerDriver, SchedulerDriver, node_capacities

ROOT = Path(__file__).resolve().parents[2]
PARTS = {"SPX": 1, "DPX": 2, "QPX": 4, "CPX": 8}


class SerializedRouter(S.Router):
    """Reference concurrency model: one lock across every verb, held through bind's API I/O."""

    def __init__(self, ext, ready=None):
        super().__init__(ext, ready)
        self.lock = asyncio.Lock()

    async def filter(self, q, body):
        async with self.lock:
            return await super().filter(q, body)

    async def prioritize(self, q, body):
        async with self.lock:
            return await super().prioritize(q, body)

    async def bind(self, q, body):
        try:
            args = json.loads(body)
            pod = await self.ext.api.get_pod(args.get("PodNamespace") or "default", args["PodName"])
            self.ext.pods.put(pod)
        except Exception:
            pass
        async with self.lock:
            return await super().bind(q, body)


def make_nodes(n_nodes: int, gpus: int, partition: str = "SPX", topo: NodeTopology | None = None,
               prefix: str = "mi355x") -> list[dict]:
    topo = topo or synthetic_mi355x(gpus, partition)
    return [pu.make_node(f"{prefix}-{i:03d}", len(topo.devices), topo.to_json(), {"amd.com/gpu.present": "true"})
            for i in range(n_nodes)]


class Harness:
    """One extender (ours or the reference model) against one fake cluster."""

    def __init__(self, nodes: list[dict], policy: str, reference: bool = False, api_rtt_ms: float = 0.0,
                 inflight: int = 64, http_api: bool = False, track_hbm: bool = True, driver: str = "native"):
        self.track_hbm = track_hbm
        self.driver = driver     # kube-scheduler stand-in: "native" (C++, own threads) or "python"
        self.nodes = nodes
        self.policy = policy
        self.reference = reference
        self.store = FakeKubeStore(faults=Faults(latency_s=api_rtt_ms / 1e3))
        for n in nodes:
            self.store.add_node(n)
        self.inflight = inflight
        self.http_api = http_api
        self.api_runner = None

    async def __aenter__(self):
        kw = dict(port=0, host="127.0.0.1", priority=self.policy, policy_config_path="/nonexistent",
                  reservation_ttl_s=3600, max_pods=262144)
        if self.reference:
            kw.update(compat=True, track_hbm=False, frontend="aiohttp")
        elif not self.track_hbm:
            kw.update(track_hbm=False)
        if self.http_api:
            self.api_runner, port = await serve(self.store)
            self.rt = Runtime(Config(kube_api=f"http://127.0.0.1:{port}", **kw))
        else:
            self.rt = Runtime(Config(**kw), api=InProcKube(self.store))
        if self.reference:
            await self.rt.start(serve=False)
            router = SerializedRouter(self.rt.extender, self.rt.ready)
            app = S.make_app(self.rt.extender, router=router)
            self.runner, self.port = await S.start(app, "127.0.0.1", 0)
        else:
            await self.rt.start()
            self.runner, self.port = None, self.rt.bound_port
        self.client = FastExtenderClient("127.0.0.1", self.port, pool=self.inflight + 8)
        return self

    async def __aexit__(self, *exc):
        await self.client.close()
        if self.runner is not None:
            await self.runner.cleanup()
        await self.rt.stop()
        if self.api_runner is not None:
            await self.api_runner.cleanup()

    async def burst(self, pods: list[dict], seed: int = 0) -> dict:
        names = [pu.meta(n)["name"] for n in self.nodes]
        self.rt.tracer.buf.clear()
        if self.driver == "native":
            # pods created first (kubectl), then the C++ stand-in schedules them from its own
            # threads (no GIL), as kube-scheduler would from its own process
            created = [self.store.create_pod(p) for p in pods]
            drv = NativeSchedulerDriver("127.0.0.1", self.port, names, node_capacities(self.nodes),
                                        bind_threads=self.inflight, seed=seed, max_attempts=3)
            loop = asyncio.get_running_loop()
            t0 = time.perf_counter()
            stats = await loop.run_in_executor(None, drv.run, created)
        else:
            drv = SchedulerDriver(self.client, InProcKube(self.store), names, node_capacities(self.nodes),
                                  max_inflight_binds=self.inflight, seed=seed, max_attempts=3)
            t0 = time.perf_counter()
            stats = await drv.run(pods)
        wall = time.perf_counter() - t0
        binds = sorted(s["dur_ms"] for s in self.rt.tracer.dump(10 ** 9, "bind") if s["ok"])
        out = stats.summary()
        out.pop("bind_s_all", None)
        out["wall_s"] = wall
        out["ext_bind_p50_ms"] = statistics.median(binds) if binds else None
        return out

    def frag(self, min_request: int) -> dict:
        return self.rt.state.frag(min_request)

    def placements(self) -> dict[str, list]:
        return {pu.pod_key(p): [pu.node_name_of(p), (p["metadata"].get("annotations") or {})]
                for p in self.store.pods.values() if pu.node_name_of(p)}

    def hbm_overcommit(self) -> dict:
        """HBM pools (or devices with their own HBM) whose placed containers ask for more
        than they hold (the reference has no HBM dimension, so its placements can exceed
        288 GB per GPU). Returns counts of over-committed pools and GiB over."""
        from ..topology.model import from_node

        topo = {pu.meta(n)["name"]: from_node(n) for n in self.nodes}
        used: dict[tuple[str, int], int] = {}
        cap: dict[tuple[str, int], int] = {}
        for p in self.store.pods.values():
            node = pu.node_name_of(p)
            if not node or pu.is_completed(p):
                continue
            for c in pu.containers(p):
                idx = pu.container_assignment(p, c.get("name", "")) or []
                for i in idx:
                    if i < 0:
                        continue
                    d = topo[node].devices[i]
                    key = (node, 1000 + d.pool) if d.pool >= 0 else (node, i)
                    cap[key] = d.hbm_mib
                    used[key] = used.get(key, 0) + pu.container_mib(c)
        over = [v - cap[k] for k, v in used.items() if v > cap[k]]
        return {"devices_overcommitted": len(over), "devices_used": len(used),
                "overcommitted_gib": round(sum(over) / 1024, 1)}

    async def delete(self, pods: list[dict]) -> None:
        for p in pods:
            ns, name = pu.pod_ns_name(p)
            try:
                self.store.delete_pod(ns, name)
            except Exception:
                pass
        uids = [pu.pod_uid(p) for p in pods]
        for _ in range(20000):
            if not any(self.rt.state.ledger.lookup(u) for u in uids):
                break
            await asyncio.sleep(0.0005)


def _pods(n: int, sizes, hbm_gib=(0,), seed: int = 0, prefix: str = "p", containers: int = 1) -> list[dict]:
    rng = random.Random(seed)
    return [pu.make_pod(f"{prefix}{i}", [(f"c{k}", rng.choice(sizes), rng.choice(hbm_gib) * 1024)
                                         for k in range(containers)]) for i in range(n)]


def _both(fn):
    async def run(*a, **kw):
        return {"ours": await fn(*a, reference=False, **kw), "reference_model": await fn(*a, reference=True, **kw)}
    return run


# ----------------------------------------------------------------------------- configs
async def config1(reference=False, reps=20, **_):
    """kind-style plumbing: real HTTP API server, 1 fake-GPU node, 1 pod gpu-percent=20, binpack.
    The one-pod flow (create -> filter -> priorities -> bind -> delete -> release) is repeated
    `reps` times so the latency is a median, not one cold sample."""
    nodes = make_nodes(1, 1, prefix="kind-worker")
    name = pu.meta(nodes[0])["name"]
    binds, ok = [], 0
    async with Harness(nodes, "binpack", reference, http_api=True) as h:
        for k in range(reps):
            pods = _pods(1, (20,), prefix=f"p{k}-")
            r = await h.burst(pods)
            pod = h.store.get_pod("default", pu.meta(pods[0])["name"])
            ann = pod["metadata"]["annotations"]
            free = h.rt.state.status()[name]["GPUs"][0]["Percent"]
            ok += (r["scheduled"] == 1 and ann.get(T.container_annotation("c0")) == "0"
                   and ann.get(T.ANNOTATION_GPU_ASSUME) == "true" and free == 80)
            binds.append(r["bind_p50_ms"])
            await h.delete(pods)
        released = h.rt.state.status()[name]["GPUs"][0]["Percent"] == 100
    return {"scheduled": 1 if ok == reps else 0, "placement": "0" if ok == reps else "?", "status_free": 80 if ok == reps else -1,
            "reps_ok": ok, "reps": reps, "released_after_delete": released,
            "bind_p50_ms": statistics.median(binds)}


async def config2(gpus=1, reference=False, hbm_mib=None, **_):
    """1 MI355X node (G GPUs), 10 pods x (20 %, 32 GiB), binpack; plus an HBM over-commit probe."""
    topo = synthetic_mi355x(gpus, hbm_mib=hbm_mib or 288 * 1024)
    nodes = make_nodes(1, gpus, topo=topo)
    out = {}
    async with Harness(nodes, "binpack", reference) as h:
        out["burst"] = await h.burst(_pods(10, (20,), (32,)))
        out["frag"] = h.frag(20)
    # 10 pods x (10 %, 64 GiB) on one GPU: 640 GiB asked of a 288 GiB device
    async with Harness(make_nodes(1, 1, topo=synthetic_mi355x(1, hbm_mib=hbm_mib or 288 * 1024)), "binpack",
                       reference) as h:
        r = await h.burst(_pods(10, (10,), (64,), prefix="m"))
        dev_mib = topo.devices[0].hbm_mib
        out["hbm_probe"] = {"scheduled": r["scheduled"], "hbm_requested_gib": 64 * r["scheduled"],
                            "hbm_device_gib": round(dev_mib / 1024, 1),
                            "overcommitted_gib": max(0, 64 * r["scheduled"] - dev_mib // 1024)}
    return out


async def config3(gpus=8, nodes_n=8, pods_per_gpu=25, reference=False, api_rtt_ms=0.0, reps=7, **_):
    """Burst of 25 pods per GPU (200 for 8 GPUs), mixed gpu-percent {10,25,50}, spread.
    A burst lasts tens of milliseconds, so it runs `reps` times on a fresh cluster and the
    run with the median rate is reported."""
    runs = []
    for _rep in range(reps):
        nodes = make_nodes(nodes_n, gpus)
        async with Harness(nodes, "spread", reference, api_rtt_ms=api_rtt_ms) as h:
            r = await h.burst(_pods(pods_per_gpu * gpus, (10, 25, 50), seed=3))
            r["frag"] = h.frag(10)
            runs.append(r)
    runs.sort(key=lambda r: r["pods_per_s"])
    out = dict(runs[len(runs) // 2])
    out["pods_per_s_runs"] = [round(r["pods_per_s"]) for r in runs]
    return out


async def config4(reference=False, **_):
    """4-container pod on an 8-GPU node: distinct GPUs, and which ones (xGMI / NUMA)."""
    topo = synthetic_mi355x(8)
    # one degraded link and a partly used GPU make the choice non-trivial
    for a, b in ((0, 1), (1, 0)):
        topo.link_bw[a][b] = 38.0
    nodes = make_nodes(1, 8, topo=topo)
    res = {}
    async with Harness(nodes, "spread", reference) as h:
        pre = pu.make_pod("pre", [("c0", 50)])
        await h.burst([pre])
        pod = pu.make_pod("tp4", [(f"rank{k}", 25) for k in range(4)])
        r = await h.burst([pod])
        got = h.store.get_pod("default", "tp4")
        idx = [int(got["metadata"]["annotations"][T.container_annotation(f"rank{k}")]) for k in range(4)]
        gpus = [topo.devices[i].gpu for i in idx]
        pair_bw = [topo.link_bw[a][b] for i, a in enumerate(gpus) for b in gpus[i + 1:] if a != b]
        res["share_pod"] = {"devices": idx, "distinct_gpus": len(set(gpus)), "min_link_gbs": min(pair_bw or [0]),
                            "numa_nodes": sorted({topo.gpus[g].numa for g in gpus}), "scheduled": r["scheduled"]}
    # whole-GPU group (4 x 100 %): TP-4 group on free GPUs
    async with Harness(make_nodes(1, 8, topo=topo), "binpack", reference) as h:
        await h.burst([pu.make_pod("pre", [("c0", 50)])])
        pod = pu.make_pod("tp4w", [(f"rank{k}", 100) for k in range(4)])
        r = await h.burst([pod])
        got = h.store.get_pod("default", "tp4w")
        ann = got["metadata"]["annotations"]
        idx = [int(ann[T.container_annotation(f"rank{k}")]) for k in range(4)] if r["scheduled"] else []
        gpus = [topo.devices[i].gpu for i in idx]
        pair_bw = [topo.link_bw[a][b] for i, a in enumerate(gpus) for b in gpus[i + 1:] if a != b]
        res["whole_gpu_group"] = {"devices": idx, "min_link_gbs": min(pair_bw or [0]),
                                  "numa_nodes": sorted({topo.gpus[g].numa for g in gpus}),
                                  "scheduled": r["scheduled"]}
    # CPX: 8 partitions per GPU; 4 containers land on distinct physical GPUs under spread
    cpx = synthetic_mi355x(8, "CPX")
    async with Harness(make_nodes(1, 8, topo=cpx), "spread", reference) as h:
        r = await h.burst([pu.make_pod("cpx4", [(f"rank{k}", 50) for k in range(4)])])
        ann = h.store.get_pod("default", "cpx4")["metadata"]["annotations"]
        idx = [int(ann[T.container_annotation(f"rank{k}")]) for k in range(4)]
        res["cpx_share_pod"] = {"devices": idx, "distinct_gpus": len({cpx.devices[i].gpu for i in idx})}
    return res


async def config5(reference=False, rounds=5, pods_n=1000, nodes_n=8, track_hbm=True, sriov=False, seeds=1, **_):
    """8 MI355X nodes in CPX (64 partitions each), 1000-pod create/delete churn, binpack.
    `sriov`: the same 64 GPUs as 16 SR-IOV guest VMs with 4 virtual functions each.
    `seeds` > 1 repeats the churn with other pod and deletion streams and reports the mean:
    a 125-pod SR-IOV churn on 64 devices is too small for one stream to rank two policies
    (per-seed frag % spreads 1.1-2.3 for one policy, 1.2-3.8 for the other)."""
    series, total, wall = [], 0, 0.0
    for seed in range(seeds):
        if sriov:
            nodes = make_nodes(nodes_n * 2, 4, topo=synthetic_sriov_guest(4), prefix="mi355x-vm")
        else:
            nodes = make_nodes(nodes_n, 8, "CPX")
        rng = random.Random(5 + 1000 * seed)
        live: list[dict] = []
        async with Harness(nodes, "binpack", reference, track_hbm=track_hbm) as h:
            t0 = time.perf_counter()
            for r in range(rounds):
                pods = _pods(pods_n // rounds, (10, 25, 50, 100), (0, 8, 16, 32), seed=100 + r + 1000 * seed,
                             prefix=f"r{r}-")
                st = await h.burst(pods, seed=seed)
                total += st["scheduled"]
                live += [p for p in pods if pu.node_name_of(h.store.pods.get(pu.pod_ns_name(p), {}))]
                f = h.frag(10)
                oc = h.hbm_overcommit()
                series.append({"seed": seed, "round": r, "scheduled": st["scheduled"],
                               "pods_per_s": round(st["pods_per_s"], 1),
                               "hbm_overcommitted_devices": oc["devices_overcommitted"],
                               "hbm_overcommitted_gib": oc["overcommitted_gib"],
                               "frag_pct": round(f["frag_pct"], 2), "stranded_pct": round(f["stranded_pct"], 2),
                               "frag_hbm_pct": round(f["frag_mib"], 2), "used_devices": f["devices_used"]})
                rng.shuffle(live)
                half, live = live[:len(live) // 2], live[len(live) // 2:]
                await h.delete(half)
            wall += time.perf_counter() - t0
    return {"series": series, "scheduled": total, "wall_s": wall, "seeds": seeds,
            "mean_frag_pct": round(statistics.mean(s["frag_pct"] for s in series), 2),
            "mean_stranded_pct": round(statistics.mean(s["stranded_pct"] for s in series), 2),
            "max_hbm_overcommitted_devices": max(s["hbm_overcommitted_devices"] for s in series),
            "max_hbm_overcommitted_gib": max(s["hbm_overcommitted_gib"] for s in series),
            "release_lag_model_s": None if not reference else round(pods_n / 2 / 1.0, 1)}


async def run_all(quick: bool = False) -> dict:
    out: dict = {"time": time.time()}
    out["config1"] = await _both(config1)()
    out["config2"] = {f"{g}gpu": await _both(config2)(gpus=g) for g in (1, 2, 4, 8)}
    out["config3"] = {f"{g}gpu_per_node": await _both(config3)(gpus=g) for g in ((8,) if quick else (1, 2, 4, 8))}
    out["config3_rtt2ms"] = await _both(config3)(gpus=8, api_rtt_ms=2.0)
    out["config4"] = await _both(config4)()
    out["config5"] = await _both(config5)(rounds=3 if quick else 5)
    out["config5"]["ours_percent_only"] = await config5(rounds=3 if quick else 5, track_hbm=False)
    # 64 whole-GPU VFs instead of 512 CPX partitions: the same load per device is 1/8 the pods
    out["config5_sriov"] = await _both(config5)(rounds=3 if quick else 5, pods_n=125, sriov=True,
                                                seeds=4 if quick else 8)
    return out


def summary_md(r: dict) -> str:
    L = ["# BASELINE configs 1-5: this framework vs the reference model", "",
         "Generated by `python -m nanogpu.sim.configs` (see its docstring for the reference model).", ""]
    c1 = r["config1"]
    L += ["## Config 1 — plumbing (real HTTP API server, 1 node, 1 pod @ 20 %, median of 20 runs)", "",
          "| | scheduled | device | free % after | bind p50 ms (client) |", "|---|---:|---:|---:|---:|"]
    for k in ("ours", "reference_model"):
        v = c1[k]
        L.append(f"| {k} | {v['scheduled']} | {v['placement']} | {v['status_free']} | {v['bind_p50_ms']:.3f} |")
    L += ["", "## Config 2 — 1 node, 10 pods × (20 %, 32 GiB), binpack, G visible GPUs", "",
          "| G | ours scheduled | ref scheduled | HBM probe (10 × 10 %/64 GiB on 1 GPU): ours | ref | ref over-commit GiB |",
          "|---:|---:|---:|---:|---:|---:|"]
    for g, v in r["config2"].items():
        L.append(f"| {g} | {v['ours']['burst']['scheduled']} | {v['reference_model']['burst']['scheduled']} | "
                 f"{v['ours']['hbm_probe']['scheduled']} | {v['reference_model']['hbm_probe']['scheduled']} | "
                 f"{v['reference_model']['hbm_probe']['overcommitted_gib']} |")
    L += ["", "## Config 3 — 8 nodes, 25 pods per GPU, mixed {10,25,50} %, spread", "",
          "Median of 7 bursts. Bind p50 is given twice: as kube-scheduler sees it (request to "
          "response, including the wait in the extender's queue while the burst floods in) and "
          "inside the extender (the verb itself).", "",
          "| GPUs/node | pods | ours pods/s | ref pods/s | ours bind p50 ms (sched / ext) | "
          "ref bind p50 ms (sched / ext) | ours frag % | ref frag % |",
          "|---:|---:|---:|---:|---:|---:|---:|---:|"]

    def _ms(v):
        return "-" if v is None else f"{v:.3f}"

    for g, v in list(r["config3"].items()) + [("8 (API RTT 2 ms)", r["config3_rtt2ms"])]:
        o, f = v["ours"], v["reference_model"]
        L.append(f"| {g} | {o['scheduled']} | {o['pods_per_s']:.0f} | {f['pods_per_s']:.0f} | "
                 f"{_ms(o['bind_p50_ms'])} / {_ms(o.get('ext_bind_p50_ms'))} | "
                 f"{_ms(f['bind_p50_ms'])} / {_ms(f.get('ext_bind_p50_ms'))} | "
                 f"{o['frag']['frag_pct']:.2f} | {f['frag']['frag_pct']:.2f} |")
    c4 = r["config4"]
    L += ["", "## Config 4 — 4-container pod on one 8-GPU node (GPU0–1 link degraded to 38 GB/s, GPU0 half used)", "",
          "| case | ours devices | ours min link GB/s | ours NUMA | ref devices | ref min link GB/s | ref NUMA |",
          "|---|---|---:|---|---|---:|---|"]
    for case in ("share_pod", "whole_gpu_group"):
        o, f = c4["ours"][case], c4["reference_model"][case]
        L.append(f"| {case} | {o['devices']} | {o['min_link_gbs']} | {o['numa_nodes']} | {f['devices']} | "
                 f"{f['min_link_gbs']} | {f['numa_nodes']} |")
    o, f = c4["ours"]["cpx_share_pod"], c4["reference_model"]["cpx_share_pod"]
    L.append(f"| cpx_share_pod (distinct physical GPUs) | {o['devices']} | {o['distinct_gpus']} GPUs | | {f['devices']} | "
             f"{f['distinct_gpus']} GPUs | |")
    c5 = r["config5"]
    L += ["", "## Config 5 — 8 CPX nodes (512 partitions), create/delete churn, binpack", "",
          "| | scheduled | mean frag % | mean stranded % | max HBM-over-committed pools | max over-commit GiB | wall s |",
          "|---|---:|---:|---:|---:|---:|---:|"]
    for k in ("ours", "ours_percent_only", "reference_model"):
        v = c5[k]
        L.append(f"| {k} | {v['scheduled']} | {v['mean_frag_pct']} | {v['mean_stranded_pct']} | "
                 f"{v['max_hbm_overcommitted_devices']} | {v['max_hbm_overcommitted_gib']} | {v['wall_s']:.2f} |")
    L += ["", "HBM is accounted per memory partition: under NPS1 the 8 CPX partitions of a GPU share its "
          "288 GB pool. `ours_percent_only` ignores HBM like the reference does; the over-commit columns "
          "count HBM pools whose placed containers ask for more than the pool holds.", "",
          "Reference release lag under churn (not simulated): ~1 released pod per second per controller "
          "worker (reference controller.go:185, 256-261), i.e. "
          f"{c5['reference_model']['release_lag_model_s']} s to release one churn round's deletions with THREADNESS=1.", ""]
    c5s = r.get("config5_sriov")
    if c5s:
        L += ["## Config 5 (SR-IOV) — the same 64 GPUs as 16 guest VMs × 4 virtual functions, churn, binpack", "",
              "Guests see their VFs' own VRAM but no xGMI links and no NUMA layout "
              "(`topology.model.synthetic_sriov_guest`, virtualization GUEST). Mean over several pod/deletion streams (seeds). 125 pods: 64 whole-GPU VFs "
              "hold 1/8 of the 512 CPX partitions' device count, so this is the same load per device.", "",
              "| | scheduled | mean frag % | mean stranded % | max HBM-over-committed devices | max over-commit GiB | wall s |",
              "|---|---:|---:|---:|---:|---:|---:|"]
        for k in ("ours", "reference_model"):
            v = c5s[k]
            L.append(f"| {k} | {v['scheduled']} | {v['mean_frag_pct']} | {v['mean_stranded_pct']} | "
                     f"{v['max_hbm_overcommitted_devices']} | {v['max_hbm_overcommitted_gib']} | {v['wall_s']:.2f} |")
        L.append("")
    return "\n".join(L)


def main(argv=None) -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default=str(ROOT / "profiles" / "bench_configs.json"))
    ap.add_argument("--quick", action="store_true")
    a = ap.parse_args(argv)
    r = asyncio.run(run_all(a.quick))
    Path(a.out).parent.mkdir(parents=True, exist_ok=True)
    Path(a.out).write_text(json.dumps(r, indent=1, default=str))
    md = summary_md(r)
    Path(a.out).with_suffix(".md").write_text(md)
    print(md)
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
