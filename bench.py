"""Headline benchmark: pods/s + p50 bind latency + GPU frag%, 1k-pod burst on 8xMI355X nodes.

Metric and config come from BASELINE.json ("pods/sec + p50 bind latency + GPU frag%, 1k-pod
burst on 8xMI355X"). The reference publishes no number, so vs_baseline is null.

What one step is (all of it inside the timed region):
  * a burst of `--pods` (default 1000) pods is created in the API server, mixed
    gpu-percent {10, 25, 50} with HBM requests {8, 16, 32, 64} GiB;
  * every pod goes through the full extender protocol over loopback HTTP. A kube-scheduler
    stand-in runs in its own process (as kube-scheduler does in a cluster): a serial
    scheduling cycle filter -> priorities -> select host on one keep-alive connection
    (kube-scheduler's score combining, nanogpu/sim/kubescore.py), and binds sent the moment a
    host is chosen. The extender answers filter/priorities in its native C++ front door,
    reserves on the native ledger, and its C++ writer threads PATCH the placement
    annotations and POST the binding to the API server, then commit;
  * after the burst the whole burst is deleted; the pod controller sees the DELETED events
    on its watch and releases every share from the ledger (BASELINE config 5's churn).
The API server (default) is ONE native HTTP API server (native/src/apiserver.cpp) in a
process of its own, shared by every rank: binds are real REST writes, the pod controller
(rank 0 only, worker 0 of a replica) follows a real chunked watch. `--inproc-api` gives each
rank an in-process store instead (round 1's extender-isolated setup; `value_inproc_api`).
`value` = pods bound per second over the K timed steps (whole job, all ranks).
`value_rtt2ms` repeats the run with a 2 ms round trip on every API answer.
The stand-in is C++ by default (kube-scheduler is compiled Go; the Python stand-in's
interpreter time per pod exceeded the extender's and capped the rate): `--driver python`
selects the Python one, `--inproc-driver` runs a Python stand-in inside the extender's
event loop.

Scaling (`--gpus N`, one torchrun rank per GPU; plain `python bench.py --gpus N` starts the N
ranks itself through torch.distributed.run, `launch_ranks`): every rank is one extender worker; all
workers share ONE native ledger in /dev/shm (the SO_REUSEPORT replica design of
nanogpu.app) and ONE API server, each drives 1/N of the burst through its own HTTP
endpoint, so the burst and the cluster are fixed while workers are added ("strong" scaling). The GPUs are used for the
node model: each rank reads its MI355X through the native KFD/amdsmi reader + HIP probe
(HBM copy rate); the xGMI link weights the topology scorer uses come from the peer-pull probe
over every pair of visible GPUs (all ranks together), else from the rate KFD publishes for the
links (`measured_links`). With N > 1 the RCCL all-reduce busBW is reported as a labelled
collective aggregate. All of that is untimed.
Data: synthetic pods; cluster of `--nodes` simulated nodes cloned from the discovered MI355X.
"""
from __future__ import annotations

import argparse
import asyncio
import json
import os
import statistics
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parent
sys.path.insert(0, str(ROOT))

# the harness (nanogpu/sim/benchlib.py); hop_summary and measured_links are also read by the tests
from nanogpu.sim.benchlib import (BIND_HOPS, ApiServerProc, _first_vs_median, _frag_mean, _pct,  # noqa: E402,F401
                                  cycle_share, driver_main, hop_summary, hops_by_decile, measured_links,
                                  node_template, nodes_variant_keys, reference_model_frag, run_rank, steady_keys)

METRIC = "pods/sec + p50 bind latency + GPU frag%, 1k-pod burst on 8×MI355X"


def parse_args():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--pods", type=int, default=1000, help="pods per burst (whole job)")
    ap.add_argument("--nodes", type=int, default=64, help="simulated 8xMI355X nodes")
    ap.add_argument("--gpus-per-node", type=int, default=8)
    ap.add_argument("--partition", default="SPX", choices=["SPX", "DPX", "QPX", "CPX"])
    ap.add_argument("--policy", default="binpack")
    ap.add_argument("--compat", action="store_true", help="reference (Go 1.16) placement semantics")
    ap.add_argument("--api-rtt-ms", type=float, default=0.0, help="modelled API-server round trip")
    ap.add_argument("--rtt-variant-ms", type=float, default=2.0,
                    help="after the timed steps, a second pass with this API round trip (0: none)")
    ap.add_argument("--rtt-variant-steps", type=int, default=3)
    ap.add_argument("--decisive-filter", action="store_true",
                    help="the extender's filter answers only the node priorities would rank first (one "
                         "round trip a pod; nanogpu --decisive-filter)")
    ap.add_argument("--decisive-variant-steps", type=int, default=5,
                    help="after the timed steps, a pass with --decisive-filter (0: none)")
    ap.add_argument("--inproc-api", action="store_true",
                    help="each rank gets an in-process API store of its own (round 1's extender-isolated "
                         "setup) instead of the default: ONE API server for the whole job over HTTP (the "
                         "native API server, native/src/apiserver.cpp, in its own process) that every "
                         "rank's extender talks REST to, with only rank 0 running the pod controller")
    ap.add_argument("--inproc-variant-steps", type=int, default=3,
                    help="after the timed steps, a pass with --inproc-api (0: none)")
    ap.add_argument("--steady", action="store_true",
                    help="steady-state churn instead of bursts: --pods fill the cluster once, then every step "
                         "deletes 30 %% of the live pods and creates as many (nanogpu.sim.workload.steady)")
    ap.add_argument("--steady-variant-steps", type=int, default=6,
                    help="after the timed steps, a --steady pass with this many timed steps (0: none); "
                         "frag_pct_steady is the mean of its second half")
    ap.add_argument("--nodes-variant", type=int, default=1000,
                    help="after the timed steps, a pass on this many nodes with kube-scheduler's node "
                         "sampling (numFeasibleNodesToFind); 0: none")
    ap.add_argument("--nodes-variant-pods", type=int, default=0,
                    help="pods per burst of the --nodes-variant pass (0: --pods scaled to the same occupancy)")
    ap.add_argument("--nodes-variant-steps", type=int, default=2)
    ap.add_argument("--independent-schedulers", action="store_true",
                    help="with N ranks: N independent kube-scheduler stand-ins, one per extender worker, each "
                         "scheduling 1/N of the burst. Default: ONE stand-in (rank 0's) drives every pod, its "
                         "cycle on rank 0's extender worker, its binds spread over all N workers (a cluster "
                         "runs one active kube-scheduler)")
    ap.add_argument("--independent-variant-steps", type=int, default=3,
                    help="with N > 1 ranks, after the timed steps, an --independent-schedulers pass "
                         "(value_independent_schedulers; 0: none)")
    ap.add_argument("--apiserver-spin-us", type=float, default=5000.0,
                    help="the shared API server's IO threads poll this long after their last event before "
                         "sleeping (default 5 ms: a kube-apiserver serving a cluster is never idle between one "
                         "scheduler's bursts; its CPU is reported, apiserver_cpu_us_per_pod; 0: sleep at once)")
    ap.add_argument("--apiserver-threads", type=int, default=0,
                    help="shared API server IO threads (0: 4; more spinning threads starve its bulk create at 8 ranks)")
    ap.add_argument("--bind-writer-mode", choices=["inline", "evented", "frontdoor", "threads"], default="evented",
                    help="the extender's native bind writer: one epoll thread (evented), the front door sending "
                         "and one epoll thread reading the answers (frontdoor), the front door alone (inline), "
                         "or blocking threads")
    ap.add_argument("--no-assume-label", action="store_true",
                    help="the extender binds with the binding alone (no label PATCH): one API write per bind")
    ap.add_argument("--no-native-pod-watch", action="store_true",
                    help="the extender reads its pod watch with aiohttp on the event loop (A/B of the "
                         "native watch thread)")
    ap.add_argument("--no-gpu", action="store_true", help="skip GPU discovery (CPU-only rehearsal)")
    ap.add_argument("--json-out", default="")
    ap.add_argument("--cpu-profile-out", default="",
                    help="native CPU sampling profile of the headline pass's timed steps (rank 0's "
                         "extender process, every thread, symbolized) as JSON into this file")
    ap.add_argument("--io-tally", action="store_true",
                    help="count and time the extender's system calls and hot phases by call site "
                         "(native/include/nanogpu/iotally.h) over the headline pass's timed steps: "
                         "io_per_pod_rank0 in the diagnostics (calls a pod, us a pod, ns a call)")
    # the deployment's front-door settings (deploy/nano-gpu-scheduler-amd.yaml): 1 epoll
    # thread that polls 8 us after each event; `--busy-poll-us 0 --frontend-threads 4` is the
    # server's plain default (about 10 % lower here, README "Results")
    ap.add_argument("--frontend-threads", type=int, default=1, help="native front door epoll workers")
    ap.add_argument("--busy-poll-us", type=int, default=int(os.environ.get("NANOGPU_BUSY_POLL_US", "8")),
                    help="native front door busy-poll window (the deployment's: 8 us catches kube-scheduler's "
                         "next request at 64 nodes and stops polling through the long gaps of big clusters)")
    ap.add_argument("--busy-poll-prio-us", type=int, default=int(os.environ.get("NANOGPU_BUSY_POLL_PRIO_US", "-1")),
                    help="the busy-poll window after a priorities answer (-1: --busy-poll-us, 0: sleep)")
    ap.add_argument("--cpu-affinity", default="auto", choices=["auto", "none"],
                    help="auto: pin each rank (extender + its scheduler stand-in) to one L3 domain on its "
                         "GPU's NUMA node (nanogpu.affinity)")
    ap.add_argument("--probe-pair-timeout", type=float, default=30.0,
                    help="time box of each GPU pair's peer-copy probe (s); the RCCL ring gets 4x")
    ap.add_argument("--probe-standin", default="",
                    help="tests: a stand-in peer probe (hang:SRC-DST never finishes that pair)")
    ap.add_argument("--spin-recv", action=argparse.BooleanOptionalAction, default=True,
                    help="front door busy poll tries a non-blocking recv on the last cycle answer's connection "
                         "first (the deployment's default; --no-spin-recv: epoll_wait(0) alone)")
    ap.add_argument("--spin-recv-binds", action="store_true",
                    help="... and, when that finds nothing, the connection the last bind answer went out on")
    ap.add_argument("--sysfs-root", default="",
                    help="tests: the KFD sysfs tree the launcher counts visible GPUs in (default: /sys)")
    return ap.parse_args()


# --------------------------------------------------------------------------- launcher
def launch_ranks(args) -> int:
    """`--gpus N` (N > 1) without a torchrun environment: this process starts the N ranks
    itself, `python -m torch.distributed.run --nproc-per-node N bench.py <same args>` as a
    child, and exits with its return code. The ranks write the JSON line to the stdout they
    inherit. Nothing here touches the GPU (no HIP call, no exec): the visible GPUs are
    counted from KFD sysfs and the visibility variables (nanogpu.topology.visible), and
    fewer than N is an error, never a silent 1-rank run."""
    import socket
    import subprocess

    if not args.no_gpu:
        from nanogpu.topology.visible import visible_gpu_count

        seen = visible_gpu_count(args.sysfs_root)
        if seen < args.gpus:
            print(f"bench: --gpus {args.gpus} needs {args.gpus} visible GPUs; {seen} visible "
                  f"(KFD sysfs{' under ' + args.sysfs_root if args.sysfs_root else ''}, "
                  f"ROCR/HIP_VISIBLE_DEVICES)", file=sys.stderr)
            return 2
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    env = dict(os.environ, MASTER_ADDR="127.0.0.1")
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")   # RCCL's dmabuf IPC on this host driver
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes", "1", "--nproc-per-node", str(args.gpus),
           "--master-addr", "127.0.0.1", "--master-port", str(port), str(Path(__file__).resolve()), *sys.argv[1:]]
    print(f"bench: starting {args.gpus} ranks: {' '.join(cmd[1:8])} ...", file=sys.stderr, flush=True)
    import signal

    child = subprocess.Popen(cmd, env=env)

    def forward(signum, _frame):   # a timeout's TERM (or ^C) reaches the ranks: no orphaned job
        try:
            child.send_signal(signum)
        except OSError:
            pass

    for sig in (signal.SIGTERM, signal.SIGINT, signal.SIGHUP):
        signal.signal(sig, forward)
    return child.wait()


# --------------------------------------------------------------------------- distributed
class Dist:
    def __init__(self, want: int):
        self.world = int(os.environ.get("WORLD_SIZE", "1"))
        self.rank = int(os.environ.get("RANK", "0"))
        self.local_rank = int(os.environ.get("LOCAL_RANK", "0"))
        self.dist = None
        self.device = None
        self.cuda = False
        if want > 1 and self.world != want:
            # main() launches the ranks itself when WORLD_SIZE is unset; a torchrun job whose
            # size disagrees with --gpus would report a curve point it did not measure
            raise SystemExit(f"bench: --gpus {want} but WORLD_SIZE={self.world}")

    def init(self, use_gpu: bool):
        import torch

        self.cuda = use_gpu and torch.cuda.is_available()
        if self.cuda:
            torch.cuda.set_device(self.local_rank)
            self.device = torch.device("cuda", self.local_rank)
        if self.world > 1:
            import torch.distributed as dist

            os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
            dist.init_process_group("nccl" if self.cuda else "gloo")
            self.dist = dist

    def barrier(self):
        if self.dist is not None:
            if self.cuda:
                import torch

                torch.cuda.set_device(self.local_rank)   # also when called from a helper thread
                self.dist.barrier(device_ids=[self.local_rank])
            else:
                self.dist.barrier()

    def sync(self):
        if self.cuda:
            import torch

            torch.cuda.synchronize()

    def max(self, v: float) -> float:
        if self.dist is None:
            return v
        import torch

        t = torch.tensor([v], dtype=torch.float64, device=self.device if self.cuda else "cpu")
        self.dist.all_reduce(t, op=self.dist.ReduceOp.MAX)
        return float(t.item())

    def gather_obj(self, obj):
        if self.dist is None:
            return [obj]
        if self.cuda:
            import torch

            torch.cuda.set_device(self.local_rank)   # also when called from a helper thread
        out = [None] * self.world
        self.dist.all_gather_object(out, obj)
        return out

    def bcast_obj(self, obj):
        if self.dist is None:
            return obj
        lst = [obj]
        self.dist.broadcast_object_list(lst, src=0)
        return lst[0]

    def close(self):
        if self.dist is not None:
            self.dist.destroy_process_group()
















































def _cpulist(cpus: list[int]) -> str:
    return ",".join(map(str, cpus)) if cpus else "unpinned"


# printed last on the line, in this order: what BASELINE's metric is made of
HEADLINE_LAST = ("value_independent_schedulers", "frag_pct_steady_reference_model", "frag_pct_steady",
                 "extender_cpu_us_per_pod_rank0", "frag_pct_reference_model", "frag_hbm_pct", "frag_pct",
                 "p99_bind_extender_ms", "p99_bind_ms", "p50_bind_ms", "pods_per_s_first_filter_to_last_bind",
                 "value")
# bulky per-step / per-thread records: --json-out only
DIAG_KEYS = ("step_diag_rank0", "bind_hops_us_by_decile_rank0", "io_per_pod_rank0", "controller_keys_per_pod_rank0", "python_requests_per_pod_rank0", "schedule_ms_each_step_rank0", "phase_ms_per_step_rank0",
             "extender_cpu_us_per_pod_by_thread_rank0", "extender_kernel_pct_by_thread_rank0",
             "extender_cpu_us_per_pod_user_kernel_rank0", "frag_pct_steady_each_step", "nominations",
             "nominations_steady", "frag_pct_steady_native_replay_each_step", "native_verb_mean_us", "frag_reference_model_source", "host_selection",
             "one_scheduler_config", "steady_config", "cpu_layout")


def order_line(full: dict) -> tuple[dict, dict]:
    """(the printed line, the diagnostics): diagnostics and every `nominations_*` /
    `native_verb_mean_us_*` map move out; the headline keys go last."""
    diag = {k: full[k] for k in full
            if k in DIAG_KEYS or k.startswith(("nominations_", "native_verb_mean_us_"))}
    line = {k: v for k, v in full.items() if k not in diag and k not in HEADLINE_LAST}
    gpu = full.get("gpu")
    if isinstance(gpu, dict) and "link_bw_matrix_gbs" in gpu:   # 8 x 8 rates: diagnostics
        diag["link_bw_matrix_gbs"] = gpu["link_bw_matrix_gbs"]
        line["gpu"] = {k: v for k, v in gpu.items() if k != "link_bw_matrix_gbs"}
    # whatever else the line carries, it stays under ~3.8 KB: the largest side keys move out
    keep = {"metric", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better", "scaling",
            "vs_baseline", "dtype", "data", "config", "value_mode", "scheduled", "failed", "bind_hops_us",
            "bind_tail_hop", "gpu"}
    budget = 3800 - sum(len(json.dumps({k: full[k]})) for k in HEADLINE_LAST if k in full)
    while len(json.dumps(line)) > budget:
        side = [k for k in line if k not in keep]
        if not side:
            break
        big = max(side, key=lambda k: len(json.dumps(line[k])))
        diag[big] = line.pop(big)
    for k in HEADLINE_LAST:
        if k in full:
            line[k] = full[k]
    return line, diag


def headline_line(d: Dist, args, res: dict, out: dict, cpus: list[int], api_proc, gpu_info: dict, topo,
                  variant, one_v, steady_v, nodes_v, inproc_v, dec_v=None) -> tuple[dict, dict]:
    from nanogpu import affinity
    from nanogpu import types as T

    fr = res["frag"]
    full = {
        "metric": METRIC, "value": out["value"], "unit": "pods/s", "n_gpus": d.world,
        "steps": args.steps, "warmup": args.warmup, "ms_per_step": out["ms_per_step"],
        "higher_is_better": True, "scaling": "strong", "vs_baseline": None, "dtype": "n/a",
        # who drives the extender: a cluster runs ONE active kube-scheduler, so with N ranks the
        # headline is one stand-in whose binds spread over every worker
        # (--independent-schedulers: one per rank, value_independent_schedulers)
        "value_mode": ("one kube-scheduler stand-in" if d.world == 1 else
                       f"one kube-scheduler stand-in, binds over all {d.world} extender workers"
                       if args.one_scheduler else
                       f"{d.world} independent kube-scheduler stand-ins, one per extender worker"),
        "data": "synthetic (pod bursts; simulated nodes cloned from the discovered MI355X)",
        "config": {"model": f"nano-gpu-scheduler extender ({args.policy}{', compat' if args.compat else ''})",
                   "global_batch": args.pods, "seq_len": None,
                   "parallelism": f"{d.world} extender worker(s), shared native ledger",
                   "cluster": f"{args.nodes} nodes x {args.gpus_per_node} MI355X ({args.partition})",
                   "api_rtt_ms": args.api_rtt_ms,
                   # one native HTTP API server in its own process shared by all ranks (default),
                   # or --inproc-api's per-rank in-process store (value_inproc_api)
                   "api_server": ("in-process store per rank" if args.inproc_api else
                                  f"one native HTTP API server, own process "
                                  f"({args.apiserver_threads or 4} IO threads, "
                                  f"max {T.API_MAX_MUTATING_INFLIGHT} mutating requests in flight: 429 over it; "
                                  + (f"IO threads poll {1e6 * api_proc.spin_s:g} us after their last event)"
                                     if api_proc is not None and api_proc.spin_s > 0 else "IO threads sleep when idle)")),
                   "apiserver_cpu_us_per_pod": out.get("apiserver_cpu_us_per_pod"),
                   "cpus_rank0": _cpulist(cpus),
                   "cpus_apiserver": _cpulist(api_proc.cpus) if api_proc is not None else None,
                   "frontend": f"{args.frontend_threads} threads, busy-poll {args.busy_poll_us} us"
                               + (f" ({args.busy_poll_prio_us} us after priorities)" if args.busy_poll_prio_us >= 0 else "")},
        # physical cores vs SMT siblings of the pinned CPUs, and how busy the siblings were
        "cpu_layout": {"rank0": affinity.cpu_layout(cpus),
                       "apiserver": affinity.cpu_layout(api_proc.cpus) if api_proc is not None else None},
        "cpu_busy_pct_rank0": res.get("cpu_busy_pct"),
        "relocated_rank0": res.get("relocated"),
        # other tenants' CPUs on the rank's domain, every 4 timed steps (ContentionWatch)
        "foreign_cpus_rank0": res.get("foreign_cpus"),
        # ... and on the shared API server's domain (its own threads' CPU time taken out)
        "foreign_cpus_apiserver": res.get("foreign_cpus_api"),
        "pods_per_s_first_filter_to_last_bind": out["value_burst_window"],
        # POST /scheduler/bind wall time as kube-scheduler's stand-in sees it (request written ->
        # reply read), every bind of the timed steps on all ranks
        "p50_bind_ms": out["p50_bind_ms"], "p99_bind_ms": out["p99_bind_ms"],
        # the same binds without the API server's answer time (bind_hops' `api` hop): the part of
        # a bind's latency the extender owns (`bind_tail_hop` names who owns the rest of the tail)
        "p50_bind_extender_ms": out["p50_bind_extender_ms"], "p99_bind_extender_ms": out["p99_bind_extender_ms"],
        # extender side of the same binds: request bytes read -> reply handed to the kernel
        "p50_bind_frontdoor_ms": out["p50_bind_frontdoor_ms"],
        "p99_bind_frontdoor_ms": out["p99_bind_frontdoor_ms"],
        # the same binds split by hop (p50, p99, mean of the slowest 1 %; us) and the hop whose
        # slowest-1 % mean exceeds its median most: where the p99 bind's time goes
        "extender_share_of_cycle": cycle_share(res)[0],
        "extender_held_share_of_cycle": cycle_share(res)[1],
        "bind_hops_us": (out.get("bind_hops") or {}).get("us"),
        "bind_tail_hop": (out.get("bind_hops") or {}).get("tail_hop"),
        "bind_hops_us_by_decile_rank0": hops_by_decile(res.get("bind_hops_steps") or []),
        # the API hop's mean over the first tenth of each burst vs the median tenth: a tail at
        # the burst start (the API server's cores waking) or spread over it
        "bind_api_us_first_tenth_vs_median_tenth": _first_vs_median(hops_by_decile(res.get("bind_hops_steps") or []),
                                                                     "api"),
        "frag_pct": round(statistics.mean(f["frag_pct"] for f in fr), 3) if fr else None,
        "frag_hbm_pct": round(statistics.mean(f["frag_mib"] for f in fr), 3) if fr else None,
        "stranded_pct": round(statistics.mean(f["stranded_pct"] for f in fr), 3) if fr else None,
        "scheduled": out["scheduled"], "failed": out["failed"], "bind_retries": out["bind_errors"],
        "api_429s": out.get("api_429s"),
        "bindings_first_rank0": out.get("bindings_first"),
        "host_selection": "kube-scheduler combining (LeastAllocated + BalancedAllocation + PodTopologySpread + "
                          "10 x extender)",
        "nominations": res["nominations"],
        "controller_keys_per_pod_rank0": (round(res["controller_keys"] / max(1, res["scheduled"]), 3)
                                          if res.get("controller_keys") is not None else None),
        "python_requests_per_pod_rank0": round(res.get("python_requests", 0) / max(1, res["scheduled"]), 3),
        "nomination_adopt_pct": (round(100.0 * res["nominations"]["adopted"] / res["nominations"]["made"], 2)
                                 if res["nominations"]["made"] else None),
        "p50_queue_to_bound_ms_rank0": (round(statistics.mean(st.get("e2e_p50_ms", 0.0) for st in res["steps"]), 3)
                                        if res["steps"] else None),
        "unschedulable_attempts": out["unschedulable"],
        "gpu": gpu_info,
        "native_verb_mean_us": res.get("native"),
        "phase_ms_per_step_rank0": res.get("phase_ms"),
        "schedule_ms_each_step_rank0": res.get("schedule_ms_steps"),
        "schedule_ms_by_rank": out["schedule_ms_by_rank"],
        "bind_handoffs": out["bind_handoffs"],
        "step_diag_rank0": res.get("step_diag"),
        # CPU time of the rank-0 extender process (all its threads) per pod it handled, without
        # the bench harness's own work on its main thread (HarnessCpu, reported next to it)
        "extender_cpu_us_per_pod_rank0": round(res.get("cpu_us_per_pod", 0.0), 1),
        "bench_harness_cpu_us_per_pod_rank0": round(res.get("harness_cpu_us_per_pod", 0.0), 2),
        "extender_rss_mib_before_after_rank0": res.get("rss_mib"),
        "extender_loop_cpu_us_per_pod_rank0": round(res.get("loop_cpu_us_per_pod", 0.0), 1),
        "extender_cpu_us_per_pod_by_thread_rank0": res.get("cpu_us_per_pod_by_thread"),
        "extender_cpu_us_per_pod_user_kernel_rank0": res.get("cpu_us_per_pod_user_kernel"),
        "extender_kernel_pct_by_thread_rank0": res.get("kernel_pct_by_thread"),
    }
    if res.get("io_per_pod") is not None:
        full["io_per_pod_rank0"] = res["io_per_pod"]
    full.update(reference_model_frag(args, topo))
    if variant is not None:
        tag = f"rtt{args.rtt_variant_ms:g}ms"
        if "error" in variant:
            full[f"value_{tag}"] = None
            full[f"error_{tag}"] = variant["error"]
        else:
            full[f"value_{tag}"] = variant["value"]
            full[f"p50_bind_ms_{tag}"] = variant["p50_bind_ms"]
            full[f"p99_bind_ms_{tag}"] = variant["p99_bind_ms"]
            full[f"api_429s_{tag}"] = variant.get("api_429s")
            full[f"bindings_first_rank0_{tag}"] = variant.get("bindings_first")
    if one_v is not None:
        if "error" in one_v:
            full["value_independent_schedulers"] = None
            full["error_independent_schedulers"] = one_v["error"]
        else:
            full["value_independent_schedulers"] = one_v["value"]
            full["p50_bind_ms_independent_schedulers"] = one_v["p50_bind_ms"]
            full["steps_independent_schedulers"] = args.independent_variant_steps
    full.update(steady_keys(args, topo, steady_v))
    full.update(nodes_variant_keys(args, topo, nodes_v))
    if dec_v is not None:
        # the same bursts with the decisive filter (kube-scheduler left one feasible node: no
        # scoring, no priorities call); its own score plugins have no say in this mode
        if "error" in dec_v:
            full["value_decisive_filter"] = None
            full["error_decisive_filter"] = dec_v["error"]
        else:
            dres, dout = dec_v["res"], dec_v["out"]
            full["value_decisive_filter"] = dout["value"]
            full["p50_bind_ms_decisive_filter"] = dout["p50_bind_ms"]
            full["frag_pct_decisive_filter"] = _frag_mean(dres["frag"])
            full["priorities_calls_per_pod_decisive_filter"] = dres.get("prio_per_pod")
            full["extender_cpu_us_per_pod_decisive_filter"] = round(dres.get("cpu_us_per_pod", 0.0), 1)
    if inproc_v is not None:
        if "error" in inproc_v:
            full["value_inproc_api"] = None
            full["error_inproc_api"] = inproc_v["error"]
        else:
            full["value_inproc_api"] = inproc_v["value"]
            full["p50_bind_ms_inproc_api"] = inproc_v["p50_bind_ms"]
    return order_line(full)


def main() -> int:
    args = parse_args()
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        return launch_ranks(args)
    # stdout carries the one JSON line and nothing else: everything else this process and its
    # children write there (gloo's connection reports on every group created, library chatter)
    # goes to stderr; the line is written to the original stdout at the end
    sys.stdout.flush()
    line_fd = os.dup(1)
    os.dup2(2, 1)
    cpus: list[int] = []
    rank_cpus: list[int] = []
    rank0_numa = -1
    if args.cpu_affinity == "auto":
        # before any process is spawned or the GPU is touched: children inherit the mask
        from nanogpu import affinity

        lr, lws = int(os.environ.get("LOCAL_RANK", "0")), int(os.environ.get("LOCAL_WORLD_SIZE", "1"))
        numas = [] if args.no_gpu else affinity.gpu_numa_nodes()
        mine = numas[lr] if lr < len(numas) else -1
        ranks = [numas[r] if r < len(numas) else -1 for r in range(lws)] if lws > 1 else None
        cpus = affinity.pick_cpus(mine, lr, ranks)
        # every local rank's domain (deterministic with several ranks): the shared API server
        # keeps off all of them, though they are idle when it starts
        rank_cpus = [c for r in range(lws) for c in affinity.pick_cpus(ranks[r], r, ranks)] if ranks else list(cpus)
        rank0_numa = ranks[0] if ranks else mine
        sharing = sum(1 for r in range(lws) if affinity.pick_cpus(ranks[r], r, ranks) == cpus) if ranks else 1
        if not affinity.apply(cpus):
            cpus = []
        cores = len(cpus) / max(1, sharing) if cpus else (os.cpu_count() or 1) / max(1, lws)
    else:
        cores = (os.cpu_count() or 1) / max(1, int(os.environ.get("LOCAL_WORLD_SIZE", "1")))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if world > 1 and not args.independent_schedulers:
        # one kube-scheduler for the job: rank 0's worker serves its cycle, the others only its
        # binds (whose latency is the API server's), so rank 0 is the one front door that polls
        # for the next request, on the cores the ranks share
        if int(os.environ.get("RANK", "0")) != 0:
            args.busy_poll_us = 0
            args.busy_poll_prio_us = 0
        else:
            cores = len(cpus) if cpus else (os.cpu_count() or 1)
    if cores < 6 and args.busy_poll_us:
        # a rank keeps ~6 threads busy (2 front-door workers, its Python loop and executor, the
        # stand-in's cycle and binder): with fewer cores, spinning workers would steal them
        args.busy_poll_us = 0
        args.busy_poll_prio_us = 0
    # the kube-scheduler stand-in's process: started before anything touches the GPU (a fresh
    # interpreter, no HIP state)
    import multiprocessing as mp

    ctx = mp.get_context("spawn")
    conn, child = ctx.Pipe()
    drv_proc = ctx.Process(target=driver_main, args=(child,), daemon=True)
    drv_proc.start()
    api_proc = None
    if int(os.environ.get("RANK", "0")) == 0:
        # the shared API server's process, like the stand-in's: before anything touches the GPU
        api_proc = ApiServerProc(avoid=rank_cpus, near=rank0_numa)
    args._placement = None
    if cpus and int(os.environ.get("LOCAL_WORLD_SIZE", "1")) == 1:
        args._placement = {"cpus": list(cpus), "numa": rank0_numa,
                           "pids": [os.getpid()] + ([drv_proc.pid] if drv_proc is not None else []),
                           "apiserver": None, "api_pid": api_proc.proc.pid if api_proc is not None else None}
    d = Dist(args.gpus)
    d.init(use_gpu=not args.no_gpu)
    # the deployment that exists: one active kube-scheduler in front of every extender worker
    args.one_scheduler = d.world > 1 and not args.independent_schedulers
    topo, gpu_info = node_template(d, args)
    variant = inproc_v = steady_v = nodes_v = one_v = dec_v = None
    try:
        args._headline = True    # the native CPU profile covers this pass only
        res = run_pass(d, args, topo, conn, "main", api_proc)
        args._headline = False
        shared_api = not args.inproc_api
        if args.steady_variant_steps > 0 and not args.steady and shared_api:
            # steady-state churn (BASELINE config 5 at scale): the cluster is never emptied
            # placement quality is a property of the deployment that exists: ONE kube-scheduler
            # (with N > 1 ranks, its binds spread over every rank's worker)
            s_args = argparse.Namespace(**{**vars(args), "steady": True, "steps": args.steady_variant_steps,
                                           "warmup": 2, "api_rtt_ms": 0.0,
                                           "one_scheduler": d.world > 1})
            try:
                steady_v = (s_args, run_pass(d, s_args, topo, conn, "steady", api_proc))
                steady_v = (s_args, steady_v[1], summarize(d, s_args, steady_v[1]))
            except Exception as e:
                steady_v = {"error": f"{type(e).__name__}: {e}"}
        if d.world > 1 and args.independent_variant_steps > 0 and args.one_scheduler and not args.steady:
            # N kube-schedulers, one per worker: what the workers sustain when the one
            # scheduler's serial cycle is not the limit (a deployment nobody runs; labelled)
            o_args = argparse.Namespace(**{**vars(args), "one_scheduler": False,
                                           "steps": args.independent_variant_steps, "warmup": 1,
                                           "api_rtt_ms": 0.0})
            try:
                one_v = summarize(d, o_args, run_pass(d, o_args, topo, conn, "one", api_proc))
            except Exception as e:
                one_v = {"error": f"{type(e).__name__}: {e}"}
        if (args.nodes_variant > 0 and args.nodes_variant_steps > 0 and args.nodes_variant != args.nodes
                and not args.steady and shared_api):
            # a large cluster behind kube-scheduler's node sampling: the extender sees only the
            # share of feasible nodes numFeasibleNodesToFind lets through, from a rotating start
            nv_pods = args.nodes_variant_pods or round(args.pods * args.nodes_variant / max(1, args.nodes))
            n_args = argparse.Namespace(**{**vars(args), "nodes": args.nodes_variant, "pods": nv_pods,
                                           "steps": args.nodes_variant_steps, "warmup": 1, "api_rtt_ms": 0.0, "one_scheduler": d.world > 1})
            try:
                r = run_pass(d, n_args, topo, conn, "nodes", api_proc)
                nodes_v = (n_args, r, summarize(d, n_args, r))
            except Exception as e:
                nodes_v = {"error": f"{type(e).__name__}: {e}"}
        if args.rtt_variant_ms > 0:
            # the same burst with a modelled API-server round trip on every API call (untimed
            # for `value`; its own clock): what the pods/s above excludes
            v_args = argparse.Namespace(**{**vars(args), "api_rtt_ms": args.rtt_variant_ms,
                                           "steps": args.rtt_variant_steps, "warmup": 1, })
            try:
                variant = summarize(d, v_args, run_pass(d, v_args, topo, conn, "rtt", api_proc))
            except Exception as e:   # the headline result stands; say what failed
                variant = {"error": f"{type(e).__name__}: {e}"}
        if args.decisive_variant_steps > 0 and not args.decisive_filter and not args.steady and not args.compat:
            x_args = argparse.Namespace(**{**vars(args), "decisive_filter": True,
                                           "steps": args.decisive_variant_steps, "warmup": 1,
                                           "api_rtt_ms": 0.0})
            try:
                r = run_pass(d, x_args, topo, conn, "decisive", api_proc)
                dec_v = {"res": r, "out": summarize(d, x_args, r)}
            except Exception as e:
                dec_v = {"error": f"{type(e).__name__}: {e}"}
        if args.inproc_variant_steps > 0 and not args.inproc_api:
            # round 1's extender-isolated setup: an in-process store per rank, no HTTP
            # (each rank its own store: a stand-in per rank, each binding on its own worker)
            i_args = argparse.Namespace(**{**vars(args), "inproc_api": True, "api_rtt_ms": 0.0, "one_scheduler": False,
                                           "steps": args.inproc_variant_steps, "warmup": 1,
                                           })
            try:
                inproc_v = summarize(d, i_args, run_pass(d, i_args, topo, conn, "inproc"))
            except Exception as e:
                inproc_v = {"error": f"{type(e).__name__}: {e}"}
    finally:
        if drv_proc is not None:
            try:
                conn.send(("stop",))
            except OSError:
                pass
            drv_proc.join(10)
            if drv_proc.is_alive():
                drv_proc.terminate()
        if api_proc is not None:
            api_proc.close()
    out = summarize(d, args, res)
    if d.rank == 0:
        final_cpus = args._placement["cpus"] if getattr(args, "_placement", None) else cpus
        line, diag = headline_line(d, args, res, out, final_cpus, api_proc, gpu_info, topo,
                                   variant, one_v, steady_v, nodes_v, inproc_v, dec_v)
        # the driver keeps the last 8 KB of stdout: ONE compact line (< 4 KB) with the
        # headline keys last; the per-step diagnostics go to --json-out only
        os.write(line_fd, (json.dumps(line) + "\n").encode())
        if args.json_out:
            Path(args.json_out).write_text(json.dumps({**line, "diagnostics": diag}, indent=1))
    d.close()
    return 0


def run_pass(d: Dist, args, topo, conn, tag: str, api_proc=None) -> dict:
    """One bench pass on a fresh shared ledger (all ranks)."""
    if d.rank == 0:   # progress on stderr (a long run is seen to be alive)
        print(f"bench: pass {tag}: {args.steps} steps of {args.pods} pods on {args.nodes} nodes",
              file=sys.stderr, flush=True)
    ledger_path = d.bcast_obj(f"/dev/shm/nanogpu-bench-{os.environ.get('MASTER_PORT', os.getpid())}-{tag}-"
                              f"{int(time.time())}" if d.rank == 0 else None)
    from nanogpu.native import core

    if d.rank == 0:
        # the shared region is laid out before any rank attaches; the harness keeps no handle
        # on it (Ledger::attached counts the extender processes: one worker defers its
        # nominations past the answer, several do not)
        led = core().Ledger(ledger_path, max(1024, args.nodes), max(65536, 4 * args.pods), True)
        del led
    d.barrier()
    try:
        return asyncio.run(run_rank(d, args, topo, ledger_path, conn, api_proc))
    finally:
        d.barrier()
        if d.rank == 0:
            try:
                os.unlink(ledger_path)
            except OSError:
                pass












def summarize(d: Dist, args, res: dict) -> dict:
    """Whole-job numbers of one pass (collective: every rank calls it)."""
    elapsed = d.max(res["elapsed_s"])
    rows = [h for r in d.gather_obj(res.get("bind_hops_ns", [])) for h in r]
    hops = hop_summary(rows)
    # the extender's own part of each bind: its wall time (request read -> reply handed to the
    # kernel) without the API server's answer time (the `api` hop) and the wait for room in the
    # admission window (`window`: every slot held by API requests not answered yet, i.e. the
    # API server's backpressure; both hops are on the line in bind_hops_us)
    ext = sorted(sum(h) - h[BIND_HOPS.index("api")] - h[BIND_HOPS.index("window")] for h in rows)
    scheduled_all = sum(d.gather_obj(res["scheduled"]))
    api_cpu = res.get("apiserver_cpu_s")
    client = sorted(b for r in d.gather_obj(res["client_bind_ms"]) for b in r)
    front = sorted(b for r in d.gather_obj(res["frontdoor_bind_ms"]) for b in r)
    py = sorted(b for r in d.gather_obj(res["bind_ms"]) for b in r)
    scheduled = sum(d.gather_obj(res["scheduled"]))
    # BASELINE's own definition: pods bound / (last successful bind - first filter),
    # per burst over all ranks, summed over the timed bursts
    windows = d.gather_obj([(st.get("t_first_filter", 0.0), st.get("t_last_bind", 0.0)) for st in res["steps"]])
    win = 0.0
    for k in range(min(len(w) for w in windows) if windows else 0):
        firsts = [w[k][0] for w in windows if w[k][0] > 0]
        lasts = [w[k][1] for w in windows if w[k][1] > 0]
        if firsts and lasts:
            win += max(lasts) - min(firsts)
    return {"value": round(scheduled / elapsed, 2) if elapsed > 0 else 0.0,
            "p50_bind_extender_ms": round(ext[len(ext) // 2] / 1e6, 4) if ext else None,
            "p99_bind_extender_ms": round(ext[min(len(ext) - 1, int(0.99 * len(ext)))] / 1e6, 4) if ext else None,
            "apiserver_cpu_us_per_pod": round(1e6 * api_cpu / scheduled_all, 1) if api_cpu is not None and scheduled_all else None,
            "value_burst_window": round(scheduled / win, 2) if win > 0 else None,
            "ms_per_step": round(1e3 * elapsed / max(1, args.steps), 3),
            "p50_bind_ms": round(statistics.median(client), 4) if client else None,
            "p99_bind_ms": _pct(client, 0.99),
            "p50_bind_frontdoor_ms": round(statistics.median(front), 4) if front else None,
            "p99_bind_frontdoor_ms": _pct(front, 0.99),
            "p50_bind_python_ms": round(statistics.median(py), 4) if py else None,
            "scheduled": scheduled, "failed": sum(d.gather_obj(res["failed"])),
            "unschedulable": sum(d.gather_obj(res["unschedulable_attempts"])),
            "bind_errors": sum(d.gather_obj(res["bind_errors"])),
            "bind_handoffs": res.get("bind_handoffs"),
            "bind_hops": hops,
            # the API server's max-in-flight admission: 429s answered in this pass (rank 0 holds it)
            "api_429s": ((res.get("apiserver") or {}).get("admission") or {}).get("too_many_requests"),
            # rank 0's bindings sent ahead of their labels (a saturated admission window)
            "bindings_first": res.get("bindings_first"),
            # each rank's mean stand-in span per step: the slowest sets the peak barrier
            "schedule_ms_by_rank": [round(v, 2) for v in d.gather_obj((res.get("phase_ms") or {}).get("schedule_ms", 0.0))]}












if __name__ == "__main__":
    sys.exit(main())
