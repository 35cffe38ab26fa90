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
import random
import statistics
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parent
sys.path.insert(0, str(ROOT))

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
    ap.add_argument("--apiserver-keep-heap", action="store_true",
                    help="the shared API server's process keeps freed heap memory (no trim / unmap)")
    ap.add_argument("--apiserver-spin-us", type=float, default=5000.0,
                    help="the shared API server's IO threads poll this long after their last event before "
                         "sleeping (default 5 ms: a kube-apiserver serving a cluster is never idle between one "
                         "scheduler's bursts; its CPU is reported, apiserver_cpu_us_per_pod; 0: sleep at once)")
    ap.add_argument("--apiserver-history", type=int, default=0,
                    help="the shared API server's watch cache, events per kind (0: 65536)")
    ap.add_argument("--apiserver-threads", type=int, default=0,
                    help="shared API server IO threads (0: one per rank, 4 to 16)")
    ap.add_argument("--bind-writer-threads", type=int, default=0,
                    help="extender's native bind writer threads per rank, 8 binds in flight each "
                         "(0: 16 split over the ranks, at least 2)")
    ap.add_argument("--inflight-binds", type=int, default=64)
    ap.add_argument("--bind-writer-mode", choices=["inline", "evented", "frontdoor", "threads"], default="evented",
                    help="the extender's native bind writer: one epoll thread (evented), the front door sending "
                         "and one epoll thread reading the answers (frontdoor), the front door alone (inline), "
                         "or blocking threads")
    ap.add_argument("--no-assume-label", action="store_true",
                    help="the extender binds with the binding alone (no label PATCH): one API write per bind")
    ap.add_argument("--no-native-pod-watch", action="store_true",
                    help="the extender reads its pod watch with aiohttp on the event loop (A/B of the "
                         "native watch thread)")
    ap.add_argument("--no-overlap-create", action="store_true",
                    help="create the next burst only after this one is released (by default the "
                         "workload's clients create it while the pod controller releases)")
    ap.add_argument("--no-gpu", action="store_true", help="skip GPU discovery (CPU-only rehearsal)")
    ap.add_argument("--json-out", default="")
    ap.add_argument("--profile-out", default="", help="cProfile the timed steps (rank 0) into this file")
    ap.add_argument("--cpu-profile-out", default="",
                    help="native CPU sampling profile of the headline pass's timed steps (rank 0's "
                         "extender process, every thread, symbolized) as JSON into this file")
    ap.add_argument("--io-tally", action="store_true",
                    help="count and time the extender's system calls and hot phases by call site "
                         "(native/include/nanogpu/iotally.h) over the headline pass's timed steps: "
                         "io_per_pod_rank0 in the diagnostics (calls a pod, us a pod, ns a call)")
    ap.add_argument("--no-nominate", action="store_true", help="priorities do not nominate (Ledger::nominate)")
    ap.add_argument("--no-kube-combine", action="store_true",
                    help="the stand-in takes the extender's arg-max instead of kube-scheduler's plugin + "
                         "weighted-extender sum (nanogpu/sim/kubescore.py)")
    # the deployment's front-door settings (deploy/nano-gpu-scheduler-amd.yaml): 1 epoll
    # thread that polls 8 us after each event; `--busy-poll-us 0 --frontend-threads 4` is the
    # server's plain default (about 10 % lower here, README "Results")
    ap.add_argument("--frontend-threads", type=int, default=1, help="native front door epoll workers")
    ap.add_argument("--busy-poll-us", type=int, default=int(os.environ.get("NANOGPU_BUSY_POLL_US", "8")),
                    help="native front door busy-poll window (the deployment's: 8 us catches kube-scheduler's "
                         "next request at 64 nodes and stops polling through the long gaps of big clusters)")
    ap.add_argument("--lazy-label-answers", action="store_true",
                    help="native writer: label PATCH answers read lazily (nanogpu --lazy-label-answers)")
    ap.add_argument("--busy-poll-prio-us", type=int, default=int(os.environ.get("NANOGPU_BUSY_POLL_PRIO_US", "-1")),
                    help="the busy-poll window after a priorities answer (-1: --busy-poll-us, 0: sleep)")
    ap.add_argument("--driver", default="native", choices=["native", "python"],
                    help="kube-scheduler stand-in: C++ (native/src/schedsim.cpp) or the Python threaded one")
    ap.add_argument("--cpu-affinity", default="auto", choices=["auto", "none"],
                    help="auto: pin each rank (extender + its scheduler stand-in) to one L3 domain on its "
                         "GPU's NUMA node (nanogpu.affinity)")
    ap.add_argument("--stall-trace", default="",
                    help="sample the extender's Python threads every ms in the timed steps; write gaps/stalls here")
    ap.add_argument("--probe-pair-timeout", type=float, default=30.0,
                    help="time box of each GPU pair's peer-copy probe (s); the RCCL ring gets 4x")
    ap.add_argument("--probe-standin", default="",
                    help="tests: a stand-in peer probe (hang:SRC-DST never finishes that pair)")
    ap.add_argument("--batch-labels", action="store_true",
                    help="the extender's writer batches the label PATCHes of bound pods (default: each pipelined "
                         "behind its binding)")
    ap.add_argument("--spin-recv", action=argparse.BooleanOptionalAction, default=True,
                    help="front door busy poll tries a non-blocking recv on the last cycle answer's connection "
                         "first (the deployment's default; --no-spin-recv: epoll_wait(0) alone)")
    ap.add_argument("--spin-recv-binds", action="store_true",
                    help="... and, when that finds nothing, the connection the last bind answer went out on")
    ap.add_argument("--spin-nap", action="store_true",
                    help="the extender's front door sleeps its busy-poll window instead of polling it")
    ap.add_argument("--bind-first", action="store_true",
                    help="the extender's front door reserves a batch's binds before its filters")
    ap.add_argument("--one-loop", action="store_true",
                    help="run the harness's step driving on the extender's asyncio loop (its CPU then "
                         "bracketed and subtracted) instead of giving the extender a loop thread of its own")
    ap.add_argument("--no-relocate", action="store_true",
                    help="keep the rank on the L3 domain picked at start even when other tenants load it "
                         "(by default a busy domain is left for a quieter one after the warm-up, and during "
                         "the timed steps when other tenants keep half a CPU of it busy)")
    ap.add_argument("--inproc-driver", action="store_true",
                    help="run the kube-scheduler stand-in inside the extender process (default: own process)")
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


class StallSampler:
    """Diagnostics (--stall-trace): a thread samples every Python thread's stack each ms.
    A gap between samples means the sampler could not get the GIL (a native call holding
    it, or the process descheduled); a long run of identical main-thread stacks is a slow
    Python call. Both are written out with the stacks around them."""

    def __init__(self, period_s: float = 0.001):
        import threading

        self.period = period_s
        self.samples: list = []
        self.on = threading.Event()
        self.stop_ev = threading.Event()
        self.main_id = threading.main_thread().ident
        self.th = threading.Thread(target=self._run, daemon=True)
        self.th.start()

    @staticmethod
    def _stack(frame, depth: int = 10) -> list[str]:
        out = []
        while frame is not None and len(out) < depth:
            c = frame.f_code
            out.append(f"{Path(c.co_filename).name}:{frame.f_lineno}:{c.co_name}")
            frame = frame.f_back
        return out

    def _run(self) -> None:
        while not self.stop_ev.is_set():
            if self.on.wait(0.05):
                fr = sys._current_frames()
                self.samples.append((time.perf_counter(), {tid: self._stack(f) for tid, f in fr.items()
                                                           if tid != self.th.ident}))
                time.sleep(self.period)

    def report(self, path: str, gap_s: float = 0.01) -> None:
        self.stop_ev.set()
        out = {"gaps": [], "n_samples": len(self.samples)}
        for (t0, s0), (t1, s1) in zip(self.samples, self.samples[1:]):
            if t1 - t0 > gap_s:
                out["gaps"].append({"t": round(t0, 4), "gap_ms": round(1e3 * (t1 - t0), 2),
                                    "main_before": s0.get(self.main_id), "main_after": s1.get(self.main_id),
                                    "others_before": {str(k): v[:4] for k, v in s0.items() if k != self.main_id}})
        Path(path).write_text(json.dumps(out, indent=1))


def _thread_group(is_main: bool, comm: str) -> str:
    if is_main:
        return "main"
    if comm.startswith("ngpu-"):
        return comm.rstrip("0123456789")
    return "bench-harness" if comm.startswith("bench-") else "other"


def thread_ticks() -> dict[str, list[int]]:
    """[user, kernel] clock ticks of this process's threads by group (thread_cpu's groups),
    from /proc/self/task/*/stat utime and stime: what share of each group's CPU is kernel
    time (syscalls, and on loopback the receiving side's TCP path a send runs)."""
    pid = os.getpid()
    out: dict[str, list[int]] = {}
    try:
        tids = os.listdir(f"/proc/{pid}/task")
    except OSError:
        return out
    for tid in tids:
        try:
            with open(f"/proc/{pid}/task/{tid}/stat") as f:
                st = f.read()
        except OSError:
            continue
        comm = st[st.index("(") + 1:st.rindex(")")]
        fields = st[st.rindex(")") + 2:].split()
        acc = out.setdefault(_thread_group(tid == str(pid), comm), [0, 0])
        acc[0] += int(fields[11])
        acc[1] += int(fields[12])
    return out


def thread_cpu() -> dict[str, float]:
    """CPU seconds of this process's threads by group: the Python main thread (event loop:
    informer, controller, Python routes), the native front door's epoll workers (ngpu-fe*,
    busy polling included), the bind writers (ngpu-wr*), and the rest (executor threads, the
    interpreter's helpers). From /proc/self/task/*/schedstat (ns on CPU), else stat ticks."""
    pid = os.getpid()
    hz = os.sysconf("SC_CLK_TCK")
    out: dict[str, float] = {}
    try:
        tids = os.listdir(f"/proc/{pid}/task")
    except OSError:
        return out
    for tid in tids:
        base = f"/proc/{pid}/task/{tid}"
        try:
            with open(base + "/comm") as f:
                comm = f.read().strip()
            try:
                with open(base + "/schedstat") as f:
                    cpu = int(f.read().split()[0]) / 1e9
            except (OSError, ValueError, IndexError):
                with open(base + "/stat") as f:
                    st = f.read()
                fields = st[st.rindex(")") + 2:].split()
                cpu = (int(fields[11]) + int(fields[12])) / hz
        except (OSError, ValueError):
            continue
        group = _thread_group(tid == str(pid), comm)
        out[group] = out.get(group, 0.0) + cpu
    return out


# --------------------------------------------------------------------------- node template
class StandinProbe:
    """`--probe-standin hang:SRC-DST` (tests): a peer probe over `world` stand-in GPUs whose
    SRC -> DST copy never completes (and ignores its own deadline); every other pair 100 GB/s."""

    def __init__(self, spec: str, n: int):
        kind, _, pair = spec.partition(":")
        if kind != "hang":
            raise ValueError(f"--probe-standin: unknown stand-in {spec!r}")
        a, b = pair.split("-")
        self.hang = (int(a), int(b))
        self.n = n

    def peer_bandwidth(self, src, dst, nbytes, iters, deadline_s=30.0):
        if (src, dst) == self.hang:
            time.sleep(3600)
        return {"gbs": 100.0, "pull_gbs": 100.0, "dma_gbs": 0.0, "peer_access": True}


def measured_links(d: Dist, host: dict, gpus_per_node: int, group=None, standin: str = "",
                   pair_timeout_s: float = 30.0) -> tuple[float, list | None, str]:
    """Per-link xGMI weights for the node model (per direction, GB/s): the peer-pull probe
    over every visible pair when this job sees the node's GPUs (all ranks take part), else
    the rate KFD publishes for this GPU's links (a 1-GPU container still sees them), else
    the placeholder. Every pair is time-boxed and the ranks agree on the outcome
    (calibrate.link_matrix over the CPU `group`): a failed or timed-out probe is recorded in
    the source and never aborts or hangs the bench."""
    from nanogpu.probe.calibrate import link_matrix, reader_link_gbs

    link, src = 153.0, "placeholder (no xGMI link visible)"
    rd = reader_link_gbs(host)
    if rd > 0:
        link, src = rd, "kfd io_link max_bandwidth (native topology reader)"
    P = None
    if standin:
        ndev = d.world if d.dist is not None else 2
        P = StandinProbe(standin, ndev)
    elif not d.cuda:
        return link, None, src
    else:
        import torch

        ndev = torch.cuda.device_count()
    try:
        m = None
        if d.dist is not None and d.world == ndev and d.world > 1:
            m = link_matrix(ndev, dist=d.dist, rank=d.local_rank, P=P, group=group, pair_timeout_s=pair_timeout_s)
        elif d.dist is None and ndev > 1:
            m = link_matrix(ndev, P=P, pair_timeout_s=pair_timeout_s)
        if m is not None:
            off = [v for a, r in enumerate(m) for b, v in enumerate(r) if a != b]
            src = f"peer-pull probe, {ndev} GPUs, every pair (copy kernel over xGMI)"
            return min(off), (m if ndev == gpus_per_node else None), src
    except Exception as e:
        src += f"; peer probe failed: {type(e).__name__}: {e}"
    return link, None, src


def node_template(d: Dist, args) -> tuple[object, dict]:
    from nanogpu.topology.model import synthetic_mi355x

    info = {"gpu": None, "link_bw_source": "placeholder"}
    hbm_mib = 288 * 1024
    if not args.no_gpu:
        from nanogpu.probe.calibrate import local_gpu_facts

        facts = local_gpu_facts(0 if not d.cuda else d.local_rank)
        gpus = facts["host"].get("gpus") or []
        props = facts.get("props") or {}
        if gpus:
            hbm_mib = int(gpus[0]["vram_bytes"]) // (1 << 20)
        elif props.get("total_mem_bytes"):
            hbm_mib = int(props["total_mem_bytes"]) // (1 << 20)
        info["gpu"] = {"gcn_arch": props.get("gcn_arch"), "cus": props.get("cus"),
                       "hbm_mib": hbm_mib, "partition": gpus[0].get("compute_partition") if gpus else None,
                       "numa": gpus[0].get("numa") if gpus else None}
        if d.cuda:
            # node-agent calibration on the real device (untimed): streaming HBM3E rate
            from nanogpu.probe.calibrate import hbm_bandwidth

            info["gpu"]["hbm_copy_gbs"] = round(hbm_bandwidth(d.local_rank, 1 << 30, 10), 1)
    link, matrix = 153.0, None
    # the calibration's own CPU group: its barriers, row exchange and agreements carry a
    # timeout and cannot queue behind a wedged GPU stream
    cal = None
    if d.dist is not None and (not args.no_gpu or args.probe_standin):
        from datetime import timedelta

        cal = d.dist.new_group(backend="gloo", timeout=timedelta(seconds=max(60.0, 4 * args.probe_pair_timeout)))
    if not args.no_gpu or args.probe_standin:
        link, matrix, src = measured_links(d, facts["host"] if not args.no_gpu else {}, args.gpus_per_node,
                                           group=cal, standin=args.probe_standin,
                                           pair_timeout_s=args.probe_pair_timeout)
        info["link_bw_source"] = src
        if matrix is not None:
            info["link_bw_matrix_gbs"] = [[round(v, 1) for v in r] for r in matrix]
            # the matrix goes to the diagnostics; its spread stays on the line
            off = sorted(v for a, r in enumerate(matrix) for b, v in enumerate(r) if a != b)
            info["link_bw_gbs_min_median_max"] = [round(off[0], 1), round(off[len(off) // 2], 1), round(off[-1], 1)]
        if d.dist is not None and d.cuda and "failed" not in src:
            # RCCL all-reduce busBW over all ranks: a collective aggregate, labelled as such;
            # time-boxed on a communicator of its own, the outcome agreed by every rank
            from nanogpu.probe.calibrate import ring_busbw_bounded

            try:
                v, why = ring_busbw_bounded(d.dist, d.device, cal, timeout_s=4 * args.probe_pair_timeout)
                info["rccl_allreduce_busbw_gbs"] = round(v, 1) if v is not None else why
            except Exception as e:
                info["rccl_allreduce_busbw_gbs"] = f"error: {type(e).__name__}: {e}"
    info["link_bw_gbs"] = round(link, 1)
    topo = synthetic_mi355x(args.gpus_per_node, args.partition, hbm_mib=hbm_mib, link_gbs=link,
                            link_matrix=matrix)
    if info["gpu"]:
        topo.calibration = {k: v for k, v in info["gpu"].items() if k in ("hbm_copy_gbs", "cus")}
    return topo, info


# --------------------------------------------------------------------------- workload
SIZES = (10, 25, 50)
HBM_GIB = (8, 16, 32, 64)


def burst(rank: int, world: int, total: int, step: int, seed: int) -> list[dict]:
    """Deterministic (sizes, owners and UIDs), so the driver process rebuilds the same objects
    (nanogpu.sim.workload: three pods in five belong to one of 16 ReplicaSets)."""
    import uuid

    from nanogpu.sim import workload as W

    pods = []
    for spec in W.burst_specs(step, total, seed):
        i = spec.key
        if i % world != rank:
            continue
        uid = str(uuid.UUID(int=((step & 0xFFFFFFFF) << 64) | (rank << 32) | i))
        pods.append(W.make_pod(spec, f"s{step}-p{i}", f"bench-r{rank}", uid))
    return pods


STEADY_CHURN = 0.3
STEADY_SEED = 11


def steady_pod(spec, rank: int = 0) -> dict:
    """A pod of the steady-state stream (nanogpu.sim.workload.steady): it lives across steps
    until the stream deletes it. Its name, namespace and UID do not depend on the rank count
    (workload.steady_pod): N workers replay the 1-worker stream."""
    from nanogpu.sim import workload as W

    return W.steady_pod(spec)


def steady_stream(args):
    """Step 0 fills the cluster with --pods pods; each later step deletes 30 % of the live pods
    and creates as many (warm-up steps first, then the timed ones)."""
    from nanogpu.sim import workload as W

    return W.steady(1 + args.warmup + args.steps, args.pods, STEADY_CHURN, STEADY_SEED)


def apiserver_main(conn, avoid: list[int] | None = None, near: int = -1) -> None:
    """The shared API server's process: native API servers (native/src/apiserver.cpp), one
    per bench pass, on an L3 domain of their own, plus a command pipe through which rank 0
    plays the workload's clients (bulk create / delete of a step's pods; the pod JSON is
    shipped before the clock starts). Started before the bench touches the GPU."""
    import json as _json

    from nanogpu import affinity
    from nanogpu.native import core

    try:   # off the ranks' CCDs: widen the inherited mask, then take the least busy domain
        os.sched_setaffinity(0, range(os.cpu_count() or 1))
    except OSError:
        pass
    affinity.apply(affinity.pick_cpus_avoiding(avoid or [], near))
    srv = None
    pool = None
    steps: dict = {}
    keys: dict = {}   # the clients know their pods' names: keyed at load, not per delete
    while True:
        msg = conn.recv()
        op = msg[0]
        if op == "start":            # a fresh server: (threads, modelled RTT in seconds[, keep heap])
            if len(msg) > 3 and msg[3]:
                # glibc keeps freed memory instead of trimming / unmapping it: a burst's writes
                # after the previous burst's bulk delete then reuse pages instead of faulting
                # them back in (M_TRIM_THRESHOLD -1, M_MMAP_THRESHOLD -3)
                import ctypes

                libc = ctypes.CDLL("libc.so.6")
                libc.mallopt(-1, 1 << 30)
                libc.mallopt(-3, 32 << 20)
            if srv is not None:
                srv.stop()
            steps.clear()
            keys.clear()
            # watch cache: 64k events per kind (--apiserver-history). A burst makes about 4k
            # (create, bind, label, delete): from the ~16th step on every event evicts an old
            # version, freed under the store's lock (profiles/soak_r05.md)
            srv = core().ApiServer("127.0.0.1", 0, msg[1], msg[5] if len(msg) > 5 and msg[5] else 1 << 16)
            srv.set_latency(msg[2])
            # polling only on CPUs of its own: on the ranks' cores it would take them from the extender
            own = not (set(os.sched_getaffinity(0)) & set(avoid or []))
            spin = msg[4] if len(msg) > 4 and msg[4] > 0 and own else 0.0
            if spin > 0:
                srv.set_spin(spin)
            # kube-apiserver's default --max-mutating-requests-inflight: over it, 429 + Retry-After
            srv.set_max_mutating_inflight(msg[6] if len(msg) > 6 else 0)
            conn.send((srv.port, sorted(os.sched_getaffinity(0)), spin))
        elif op == "nodes":
            for n in msg[1]:
                srv.call("POST", "/api/v1/nodes", n)
            conn.send(len(msg[1]))
        elif op == "load":
            steps[msg[1]] = msg[2]
            keys[msg[1]] = [(m.get("namespace", "default"), m["name"])
                            for m in (_json.loads(t)["metadata"] for t in msg[2])]
            conn.send(True)
        elif op == "create":
            t = time.perf_counter()
            codes = srv.create_pods(steps[msg[1]])
            conn.send((sum(1 for c in codes if c == 201), time.perf_counter() - t))
            if os.environ.get("NANOGPU_BENCH_DEBUG"):
                print(f"create {msg[1]} {t:.4f} -> {time.perf_counter():.4f}", file=sys.stderr)
        elif op == "delete":
            steps.pop(msg[1], None)
            t = time.perf_counter()
            n = srv.delete_pods(keys.pop(msg[1]))
            conn.send((n, time.perf_counter() - t))
            if os.environ.get("NANOGPU_BENCH_DEBUG"):
                print(f"delete {msg[1]} {t:.4f} -> {time.perf_counter():.4f}", file=sys.stderr)
        elif op == "churn":
            # the workload's clients at one moment: this burst's deletes and the next burst's
            # creates arrive together. The create runs on a second thread (both calls drop the
            # GIL): its parsing overlaps the delete; its inserts follow the delete's lock hold.
            # One parse thread: more would slow the delete, which the release waits on.
            # Replies: the delete's first, then the create's.
            if pool is None:   # one long-lived worker: no thread start per step
                from concurrent.futures import ThreadPoolExecutor

                pool = ThreadPoolExecutor(1)

            def create_next(step=msg[2]):
                t0 = time.perf_counter()
                codes = srv.create_pods(steps[step], 1)
                return sum(1 for c in codes if c == 201), time.perf_counter() - t0

            fut = pool.submit(create_next)
            steps.pop(msg[1], None)
            t = time.perf_counter()
            n = srv.delete_pods(keys.pop(msg[1]))
            conn.send((n, time.perf_counter() - t))
            conn.send(fut.result())
        elif op == "churn_keys":
            # steady-state churn: the given pods (created in earlier steps) are deleted, then
            # this step's pods are created; one reply each
            steps_keys = msg[1]
            t = time.perf_counter()
            n = srv.delete_pods(steps_keys) if steps_keys else 0
            conn.send((n, time.perf_counter() - t))
            t = time.perf_counter()
            codes = srv.create_pods(steps.pop(msg[2])) if msg[2] in steps else []
            conn.send((sum(1 for c in codes if c == 201), time.perf_counter() - t))
        elif op == "stats":
            conn.send(_json.loads(srv.stats()))
        elif op == "cpu":            # this process's CPU seconds (IO threads, polling included)
            conn.send(time.process_time())
        elif op == "end":            # the pass is over
            if srv is not None:
                srv.stop()
                srv = None
            conn.send(True)
        else:
            if srv is not None:
                srv.stop()
            conn.send(True)
            return


async def wait_released(ledger, uids: list[str], timeout_s: float = 10.0) -> bool:
    """Until the ledger holds none of `uids` (the pod controller's releases). Polled every
    20 µs from an executor thread: the event loop stays free for the watch (the in-process
    and aiohttp watches deliver the DELETED events on it), and the harness's waiting does not
    spin the extender process's event loop, whose CPU time the bench reports. Deletions arrive
    in order: the last pod first, then all of them once (one native call for the lot)."""
    def poll() -> bool:
        end = time.perf_counter() + timeout_s
        while time.perf_counter() < end:
            if not ledger.holds_any(uids[-1:]) and not ledger.holds_any(uids):
                return True
            time.sleep(20e-6)
        return False

    return await asyncio.get_running_loop().run_in_executor(None, poll)


class HarnessCpu:
    """CPU the bench harness itself spends on the extender process's main thread (the stand-in's
    step summary off the pipe, the frag measurement, the per-step records, the contention
    watch): `with hc:` around synchronous harness code only. The extender's CPU per pod is
    reported without it (a deployed extender runs none of it) and it is reported on its own."""

    def __init__(self):
        self.s = 0.0
        self.t = 0.0

    def __enter__(self):
        self.t = time.thread_time()
        return self

    def __exit__(self, *exc):
        self.s += time.thread_time() - self.t
        return False


def rss_mib() -> float:
    """This process's resident memory, MiB (/proc/self/status VmRSS)."""
    try:
        for line in open("/proc/self/status"):
            if line.startswith("VmRSS:"):
                return round(int(line.split()[1]) / 1024, 1)
    except OSError:
        pass
    return 0.0


def set_thread_comm(name: str) -> None:
    """Names the calling OS thread (/proc/self/task/<tid>/comm, 15 bytes): thread_cpu() groups
    the process's CPU by these names."""
    import ctypes

    try:
        ctypes.CDLL(None, use_errno=True).prctl(15, name.encode()[:15], 0, 0, 0)   # PR_SET_NAME
    except (OSError, AttributeError):
        pass


class ContentionMonitor:
    """The contention watches (affinity.ContentionWatch) on a harness thread of their own,
    every `period_s` while the timed steps run: their /proc and sysfs reads (3-4 ms a round on
    a 256-CPU host) stay off the steps' path, where they used to sit between every 4th step.
    A relocation it decides is made from this thread (sched_setaffinity of every thread)."""

    def __init__(self, watch, api_watch, pl: dict, results: dict, period_s: float = 0.1):
        import threading

        self.watch, self.api_watch, self.pl, self.results = watch, api_watch, pl, results
        self.period_s = period_s
        self.steps_done = 0            # the step loop's progress, for the relocation record
        self.stop_ev = threading.Event()
        self.th = threading.Thread(target=self._run, name="bench-harness", daemon=True)
        self.th.start()

    def _run(self) -> None:
        from nanogpu import affinity

        set_thread_comm("bench-harness")
        while not self.stop_ev.wait(self.period_s):
            foreign, to = self.watch.check()
            if self.api_watch is not None:
                self.results["foreign_cpus_api"].append(round(self.api_watch.check()[0], 2))
            self.results["foreign_cpus"].append(round(foreign, 2))
            if to is not None:
                affinity.relocate(self.pl["pids"], to)
                self.results["relocated"] = dict(self.results.get("relocated") or {}, mid_run_from=self.pl["cpus"],
                                                 mid_run_to=to, at_step=self.steps_done)
                self.pl["cpus"] = self.watch.cpus = to

    def close(self) -> None:
        self.stop_ev.set()
        self.th.join(5.0)


class ExtenderLoop:
    """The extender's asyncio loop on a thread of its own ("ngpu-loop"), as in a deployment,
    where `python -m nanogpu` runs nothing else on it: the harness drives the steps from the
    main thread, so the extender's CPU a pod is its own threads' CPU, measured, instead of the
    main thread's minus the harness parts that can be bracketed."""

    def __init__(self):
        import threading

        self.loop = asyncio.new_event_loop()
        started = threading.Event()

        def run():
            set_thread_comm("ngpu-loop")
            asyncio.set_event_loop(self.loop)
            started.set()
            self.loop.run_forever()

        self.th = threading.Thread(target=run, name="ngpu-loop", daemon=True)
        self.th.start()
        started.wait()

    async def run(self, coro):
        """Awaits `coro` run on the extender's loop."""
        return await asyncio.wrap_future(asyncio.run_coroutine_threadsafe(coro, self.loop))

    def close(self) -> None:
        self.loop.call_soon_threadsafe(self.loop.stop)
        self.th.join(10.0)
        if not self.th.is_alive():
            self.loop.close()


async def arecv(conn, hc: HarnessCpu | None = None):
    """conn.recv() awaited on the event loop (the pipe's fd in the selector): no executor
    thread, whose start can wait milliseconds for the GIL while the loop is busy."""
    if not conn.poll():
        loop = asyncio.get_running_loop()
        fut = loop.create_future()
        fd = conn.fileno()

        def ready():
            if not fut.done():
                fut.set_result(None)

        loop.add_reader(fd, ready)
        try:
            await fut
        finally:
            loop.remove_reader(fd)
    if hc is None:
        return conn.recv()
    with hc:
        return conn.recv()


class ApiServerProc:
    """Rank 0's handle on the shared API server process (spawned once, before any GPU use;
    `start()` gives each bench pass a fresh server)."""

    def __init__(self, avoid: list[int] | None = None, near: int = -1):
        import multiprocessing as mp

        ctx = mp.get_context("spawn")
        self.conn, child = ctx.Pipe()
        self.proc = ctx.Process(target=apiserver_main, args=(child, avoid, near), daemon=True)
        self.proc.start()
        self.url = ""
        self.cpus: list[int] = []
        self.spin_s = 0.0   # the IO threads' polling window in effect (0 when it shares the ranks' CPUs)

    def _rpc(self, *msg):
        self.conn.send(msg)
        return self.conn.recv()

    def start(self, threads: int, latency_s: float = 0.0, keep_heap: bool = False, spin_s: float = 0.0,
              history: int = 0, max_inflight: int = 0) -> str:
        port, self.cpus, self.spin_s = self._rpc("start", threads, latency_s, keep_heap, spin_s, history, max_inflight)
        self.url = f"http://127.0.0.1:{port}"
        return self.url

    def add_nodes(self, nodes: list[dict]) -> None:
        self._rpc("nodes", [json.dumps(n, separators=(",", ":")) for n in nodes])

    def load(self, step: int, pods: list[dict]) -> None:
        self._rpc("load", step, [json.dumps(p, separators=(",", ":")) for p in pods])

    async def create(self, step: int) -> tuple[int, float]:
        """(pods created, seconds the server spent on them)"""
        self.conn.send(("create", step))
        return await arecv(self.conn)

    async def delete(self, step: int) -> tuple[int, float]:
        self.conn.send(("delete", step))
        return await arecv(self.conn)

    async def churn(self, step: int, nxt: int) -> tuple[tuple[int, float], asyncio.Future]:
        """Delete `step`'s pods while `nxt`'s are created: the delete's answer, and a future of
        the create's."""
        self.conn.send(("churn", step, nxt))
        deleted = await arecv(self.conn)
        return deleted, asyncio.ensure_future(arecv(self.conn))

    async def churn_keys(self, dels: list[tuple[str, str]], create_step: int):
        """Steady state: delete `dels` (namespace, name), then create `create_step`'s pods:
        ((deleted, s), (created, s))."""
        self.conn.send(("churn_keys", dels, create_step))
        return await arecv(self.conn), await arecv(self.conn)

    def stats(self) -> dict:
        return self._rpc("stats")

    def cpu_s(self) -> float:
        return self._rpc("cpu")

    def end(self) -> None:
        self._rpc("end")

    def close(self) -> None:
        try:
            self._rpc("stop")
        except (OSError, EOFError):
            pass
        self.proc.join(10)
        if self.proc.is_alive():
            self.proc.terminate()


def driver_main(conn) -> None:
    """kube-scheduler stand-in in its own process (as in a real cluster): for each pass of
    the bench it receives the extender's address and the pass's steps, builds their pods,
    then for every step schedules that step's pods (already created in the API server by the
    main process) and returns the driver stats. The scheduling cycle is serial on a blocking
    connection; binds run on a thread pool."""
    from nanogpu.sim.driver import NativeSchedulerDriver, ThreadedSchedulerDriver
    from nanogpu.sim.kubescore import KubeScoring

    st = {"cfg": None, "work": {}, "session": None, "cls": NativeSchedulerDriver, "live": {}, "specs": {}}

    def configure(cfg: dict) -> None:
        # steady-state churn needs the stand-in's pod cache: the native stand-in only
        cls = ThreadedSchedulerDriver if cfg.get("driver") == "python" and not cfg.get("steady") \
            else NativeSchedulerDriver
        native = cls is NativeSchedulerDriver
        cfg["name_index"] = {n: i for i, n in enumerate(cfg["names"])}
        # the pods of every step, built before the clock starts (the main process does the same)
        work = {}
        st["live"], st["specs"], st["stream"] = {}, {}, None
        if cfg.get("steady"):
            # steady-state churn: pods live across steps; the stand-in keeps kube-scheduler's
            # cache of them (node, requests, owner) and hands it to every run
            stream = st["stream"] = steady_stream(argparse.Namespace(**cfg["steady"]))
            for step in cfg["steps"]:
                # the one scheduler of the job schedules every rank's pods
                specs = [s for s in stream[step].creates
                         if cfg.get("bind_ports") or s.key % cfg["world"] == cfg["rank"]]
                st["specs"][step] = specs
                work[step] = NativeSchedulerDriver.prepare_native([steady_pod(s, s.key % cfg["world"])
                                                                   for s in specs])
        for step in ([] if cfg.get("steady") else cfg["steps"]):
            if cfg.get("bind_ports"):   # the one scheduler of the job: every rank's pods
                pods = [p for r in range(cfg["world"]) for p in burst(r, cfg["world"], cfg["pods"], step, 7)]
            else:
                pods = burst(cfg["rank"], cfg["world"], cfg["pods"], step, 7)
            work[step] = NativeSchedulerDriver.prepare_native(pods) if native else pods
        cfg["kube_obj"] = KubeScoring() if cfg.get("kube") else None
        session = None
        if native:
            from nanogpu.native import core

            session = core().SchedulerSession()   # keep-alive connections across the pass's steps
        st.update(cfg=cfg, work=work, session=session, cls=cls)
        conn.send("ready")

    def serve() -> None:
        while True:
            msg = conn.recv()
            if isinstance(msg, dict):
                st.pop("spent", None)
                configure(msg)
                continue
            if msg[0] == "live":
                # the pods the other ranks' stand-ins placed last step: a kube-scheduler's cache
                # holds every bound pod (its informer), not only the ones it scheduled itself
                st["live"].update(msg[1])
                continue
            if msg[0] != "step":
                break
            cfg, work, session, cls = st["cfg"], st["work"], st["session"], st["cls"]
            native = cls is NativeSchedulerDriver
            step = msg[1]
            # native: connections of the epoll binder (a bind leaves as soon as its host is
            # chosen, as kube-scheduler's per-pod bind goroutines); Python: pool threads
            kw = ({"session": session, "bind_threads": 256, "kube": cfg["kube_obj"],
                   "bind_ports": cfg.get("bind_ports")} if native
                  else {"bind_threads": min(32, cfg["inflight"])})
            t0 = time.perf_counter()
            drv = cls("127.0.0.1", cfg["port"], cfg["names"], cfg["caps"], seed=step * 1009 + cfg["rank"], **kw)
            if st["stream"] is not None:
                live = st["live"]
                for key in st["stream"][step].deletes:
                    live.pop(key, None)
                stats = drv.run(prepared=work.pop(step), live=list(live.values()))
                args_k, node_of = drv._placed[-1]
                idx = cfg["name_index"]
                placed = []
                for spec, a, node in zip(st["specs"].pop(step), args_k, node_of):
                    if node:
                        live[spec.key] = (idx[node], a[4], a[5], a[6], a[7])
                        placed.append((spec.key, live[spec.key]))
            else:
                stats = drv.run(prepared=work.pop(step)) if native else drv.run(work.pop(step))
            t1 = time.perf_counter()
            sm = stats.summary()
            if st["stream"] is not None:
                sm["live_placed"] = placed   # for the other ranks' stand-ins (their informers)
            t2 = time.perf_counter()
            conn.send(sm)
            # the step's driver and pod records are freed at the next configure, not inside the
            # next step's clock (thousands of objects)
            drv.close()
            st.setdefault("spent", []).append(drv)
            if os.environ.get("NANOGPU_BENCH_DEBUG"):
                print(f"drv step {step}: pre {1e3*(stats.t_first_filter-t0):.3f} run {1e3*(t1-t0):.3f} "
                      f"post {1e3*(t1-stats.t_last_bind):.3f} summary {1e3*(t2-t1):.3f} send {1e3*(time.perf_counter()-t2):.3f}",
                      file=sys.stderr)

    prof_path = os.environ.get("NANOGPU_DRIVER_PROFILE")
    if prof_path:
        import cProfile

        cProfile.runctx("serve()", globals(), {"serve": serve}, prof_path)
    else:
        serve()


async def run_rank(d: Dist, args, topo, ledger_path: str, conn=None, api_proc: ApiServerProc | None = None) -> dict:
    from nanogpu import types as T
    from nanogpu.app import Config, Runtime
    from nanogpu.k8s import podutil as pu
    from nanogpu.k8s.fake_apiserver import Faults, FakeKubeStore, InProcKube
    from nanogpu.sim.driver import FastExtenderClient, SchedulerDriver, node_capacities
    from nanogpu.sim import workload as W

    # --shared-api: ONE API server for the job, as in a cluster: the native API server in its
    # own process (ApiServerProc), reached over HTTP by every rank's extender. Only rank 0 runs
    # the pod controller (worker 0 of a replica), so every release goes through its watch.
    # Rank 0 is also the workload's client: it has the API server create and delete every
    # rank's pods. Without it each rank has an in-process store of its own (extender-isolated).
    shared = not getattr(args, "inproc_api", False) and conn is not None and (api_proc is not None or d.rank != 0)
    loop = asyncio.get_running_loop()
    # with the API server in its own process nothing the harness touches lives on the
    # extender's loop: the extender gets a loop thread of its own (the in-process store's
    # watches do, so that pass keeps one loop and brackets the harness's CPU instead)
    ext = ExtenderLoop() if shared and not getattr(args, "one_loop", False) else None
    if ext is not None:
        from concurrent.futures import ThreadPoolExecutor

        # the harness's executor threads (barriers, release polls) named as the harness's
        loop.set_default_executor(ThreadPoolExecutor(4, initializer=set_thread_comm,
                                                     initargs=("bench-harness",)))

    async def on_ext(coro):
        return await (ext.run(coro) if ext is not None else coro)

    async def barrier() -> None:
        if d.world == 1:
            return
        if shared:   # keep the loop turning (watch, controller) while other ranks catch up
            await loop.run_in_executor(None, d.barrier)
        else:
            d.barrier()

    topo_json = topo.to_json()
    n_dev = len(topo.devices)
    nodes = [pu.make_node(f"mi355x-{i:03d}", n_dev, topo_json, {"amd.com/gpu.present": "true"})
             for i in range(args.nodes)]
    store, apisrv = None, None
    if shared:
        url = None
        if d.rank == 0:
            apisrv = api_proc
            url = apisrv.start(args.apiserver_threads or min(16, max(4, d.world)), args.api_rtt_ms / 1e3,
                               args.apiserver_keep_heap, args.apiserver_spin_us / 1e6, args.apiserver_history,
                               T.API_MAX_MUTATING_INFLIGHT)
            if getattr(args, "_placement", None):
                args._placement["apiserver"] = list(apisrv.cpus)
            apisrv.add_nodes(nodes)
        url = d.bcast_obj(url)
        from nanogpu.k8s.client import KubeClient, KubeConfig

        def rt_api_make():
            return KubeClient(KubeConfig(server=url), pool=args.inflight_binds + 8,
                              native_watch=not args.no_native_pod_watch)
    else:
        # the watch history a real API server keeps is a bounded cache, and not in our process
        store = FakeKubeStore(history=8192, faults=Faults(latency_s=args.api_rtt_ms / 1e3))
        for n in nodes:
            store.add_node(n)
        rt_api = InProcKube(store)

        def rt_api_make():
            return rt_api
    cfg = Config(port=0, host="127.0.0.1", priority=args.policy, compat=args.compat, ledger_path=ledger_path,
                 max_nodes=max(1024, args.nodes), max_pods=max(65536, 4 * args.pods),
                 policy_config_path="/nonexistent/policy.yaml", reservation_ttl_s=3600,
                 busy_poll_us=args.busy_poll_us, busy_poll_prio_us=args.busy_poll_prio_us, lazy_label_answers=args.lazy_label_answers,
                 frontend_threads=args.frontend_threads,
                 nominate=not args.no_nominate,
                 bind_writer_threads=args.bind_writer_threads or max(2, 16 // d.world),
                 bind_writer_mode=args.bind_writer_mode, assume_label=not args.no_assume_label,
                 # every rank's extender writes to the one API server: they share its in-flight limit
                 api_inflight_share=d.world if shared else 1,
                 bind_first=args.bind_first, spin_nap=args.spin_nap, spin_recv=args.spin_recv, spin_recv_binds=args.spin_recv_binds, batch_labels=args.batch_labels,
                 decisive_filter=getattr(args, "decisive_filter", False))
    all_steps_pre = [10_000 + w for w in range(args.warmup)] + list(range(args.steps))

    async def start_runtime():   # built and started on the extender's loop
        r = Runtime(cfg, worker=d.rank if shared else 0, api=rt_api_make())
        await r.start()
        return r

    rt = await on_ext(start_runtime())
    client = FastExtenderClient("127.0.0.1", rt.bound_port, pool=args.inflight_binds + 8)
    names = [pu.meta(n)["name"] for n in nodes]
    caps = node_capacities(nodes)
    api = InProcKube(store) if store is not None else None   # the workload's client (creates, deletes)
    steady = bool(getattr(args, "steady", False))
    stream = steady_stream(args) if steady else None
    if apisrv is not None and steady:
        for k, stp in enumerate(stream):
            apisrv.load(k, [steady_pod(s, s.key % d.world) for s in stp.creates])
    elif apisrv is not None:
        for st in all_steps_pre:
            apisrv.load(st, [p for r in range(d.world) for p in burst(r, d.world, args.pods, st, 7)])
    pod_ctrl = rt.controllers[-1] if rt.leader else None
    results = {"steps": [], "frag": [], "client_bind_s": [], "frontdoor_bind_ms": [], "bind_hops_ns": []}
    if rt.native is not None:
        # each native bind's hop split (front door -> writer -> API server -> front door)
        rt.native.fe.set_bind_hops(True)

    # synthetic pod objects are generated up front (client-side data, not scheduler work);
    # their creation in the API server, scheduling, deletion and release are all timed
    all_steps = [10_000 + w for w in range(args.warmup)] + list(range(args.steps))
    bursts = {} if steady else {s: burst(d.rank, d.world, args.pods, s, 7) for s in all_steps}
    # their UIDs too (deterministic, set by burst()): the release check's keys, not scheduler work
    burst_uids = {s: [pu.pod_uid(p) for p in ps] for s, ps in bursts.items()}

    # one scheduler (the default with N ranks): ONE kube-scheduler stand-in for the job (rank 0's) drives every pod; its
    # scheduling cycle stays on rank 0's worker, its binds spread over every rank's worker (the
    # connections a Service spreads over an extender's workers)
    one = bool(getattr(args, "one_scheduler", False)) and d.world > 1
    ports = d.gather_obj(rt.bound_port) if one else None
    drives = conn is not None and (not one or d.rank == 0)
    if conn is not None and drives:
        conn.send({"port": rt.bound_port, "names": names, "caps": caps, "rank": d.rank, "world": d.world,
                   "bind_ports": ports,
                   "pods": args.pods, "inflight": args.inflight_binds, "driver": args.driver,
                   "kube": not args.no_kube_combine,
                   "steady": {"warmup": args.warmup, "steps": args.steps, "pods": args.pods} if steady else None,
                   "steps": list(range(len(stream))) if steady else
                   [10_000 + w for w in range(args.warmup)] + list(range(args.steps))})
        await loop.run_in_executor(None, conn.recv)   # the stand-in has built its pods

    # The workload's clients create the next burst while the pod controller releases this one
    # (delete, then create, in the API server; the scheduling of the next burst still starts
    # only after every release). Each timed step's create and release stay inside the clock:
    # the first timed burst is created in the timed region, never during a warm-up release.
    overlap = apisrv is not None and not getattr(args, "no_overlap_create", False)
    created: dict = {}       # step -> its create, started during the previous step's release
    srv_ms: dict = {}        # step -> the API server's own create/delete time
    hc = HarnessCpu()        # the harness's own CPU on the main thread (not the extender's)

    # the front door's per-bind records (wall time, hop split) are taken once, after the timed
    # steps (no per-step copy inside the clock): each step only marks how many there are
    bind_marks: list = []
    spent: list = []   # finished steps' pod objects, freed after the timed steps

    def mark_binds() -> None:
        if rt.native is not None:
            bind_marks.append(rt.native.fe.bind_samples_waiting())

    def take_binds() -> None:
        if rt.native is None:
            return
        walls, hops = rt.native.fe.take_bind_wall(), rt.native.fe.take_bind_hops()
        results["frontdoor_bind_ms"] = [1e3 * x for x in walls]
        results["bind_hops_ns"] = hops
        steps_h, prev = [], 0
        for _, nh in bind_marks:
            steps_h.append(hops[prev:nh])
            prev = nh
        results["bind_hops_steps"] = steps_h

    async def one_step_steady(step: int, timed: bool) -> dict:
        """Steady-state churn: this step's deletions (pods of earlier steps) and creations, the
        controller's releases, then the stand-in schedules the new pods next to the live ones."""
        t_step0 = time.perf_counter()
        dels = stream[step].deletes
        phases: dict = {}
        if apisrv is not None:
            (n_d, dt_d), (n_c, dt_c) = await apisrv.churn_keys(
                [(W.STEADY_NAMESPACE, f"k{k}") for k in dels], step)
            phases.update(delete_srv_ms=1e3 * dt_d, create_srv_ms=1e3 * dt_c)
        with hc:
            uids = [W.steady_uid(k) for k in dels]
        if uids:
            await wait_released(rt.state.ledger, uids)
        phases["release_ms"] = 1e3 * (time.perf_counter() - t_step0)
        if shared:
            await barrier()
        t_send = time.perf_counter()
        if drives:
            with hc:
                conn.send(("step", step))
            summary = await arecv(conn, hc)
        else:            # one scheduler: rank 0's stand-in schedules this rank's pods too
            from nanogpu.sim.driver import DriverStats

            summary = DriverStats().summary()
        phases["schedule_wall_ms"] = 1e3 * (time.perf_counter() - t_send)
        placed = summary.pop("live_placed", [])
        if shared and not one:
            # the barrier, carrying each rank's placements to the other ranks' stand-ins
            every = await loop.run_in_executor(None, d.gather_obj, placed)
            others = [kv for r, lst in enumerate(every) if r != d.rank for kv in lst]
            if others:
                conn.send(("live", others))
        else:
            await barrier()
        with hc:
            frag = rt.state.frag(min(SIZES))
            phases.update(create_ms=0.0, schedule_ms=1e3 * summary["span_s"])
            client_s = summary.pop("bind_s_all", [])
            if timed:
                results["client_bind_s"].extend(client_s)
                mark_binds()
        return {"stats": summary, "frag": frag, "phases": phases}

    async def one_step(step: int, timed: bool, nxt: int | None = None) -> dict:
        if steady:
            return await one_step_steady(step, timed)
        pods = bursts.pop(step)
        # the step's pod objects (client-side data) are kept until the timed steps are over:
        # dropped here, their ~30k Python objects would be freed inside the clock (~1 ms a step)
        spent.append(pods)
        t_step0 = tc = time.perf_counter()
        if conn is not None:
            # the pods are created in the API server (this process), then the scheduler
            # process schedules them through the extender's HTTP front door. A burst comes
            # from many clients at once: with a modelled API RTT the creates overlap.
            if api is not None:
                if args.api_rtt_ms > 0:
                    await asyncio.gather(*(api.create_pod(p) for p in pods))
                else:
                    for p in pods:
                        await api.create_pod(p)
            elif apisrv is not None:
                fut = created.pop(step, None)   # every rank's pods
                n_c, dt_c = await (fut if fut is not None else apisrv.create(step))
                srv_ms.setdefault(step, {})["create_srv_ms"] = 1e3 * dt_c
            tc = time.perf_counter() - tc
            if shared:
                tb = time.perf_counter()
                await barrier()                     # every rank's pods exist
                srv_ms.setdefault(step, {})["barrier_create_ms"] = 1e3 * (time.perf_counter() - tb)
            t_send = time.perf_counter()
            if drives:
                with hc:
                    conn.send(("step", step))
                summary = await arecv(conn, hc)
            else:            # one scheduler: rank 0's stand-in schedules this rank's pods too
                from nanogpu.sim.driver import DriverStats

                summary = DriverStats().summary()
            # the stand-in's span is first filter -> last bind; this adds its per-step set-up,
            # summary and the pipe
            srv_ms.setdefault(step, {})["schedule_wall_ms"] = 1e3 * (time.perf_counter() - t_send)
        else:
            # one kube-scheduler stand-in per rank; distinct tie-break streams per rank
            from nanogpu.sim.kubescore import KubeScoring

            drv = SchedulerDriver(client, api, names, caps, max_inflight_binds=args.inflight_binds,
                                  seed=step * 1009 + d.rank, kube=None if args.no_kube_combine else KubeScoring())
            tc = 0.0
            summary = (await drv.run(pods)).summary()
        ts = time.perf_counter()
        # all ranks finished their share of the burst: peak occupancy
        await barrier()
        tb = time.perf_counter()
        srv_ms.setdefault(step, {})["barrier_peak_ms"] = 1e3 * (tb - ts)
        with hc:
            frag = rt.state.frag(min(SIZES))
        uids = burst_uids.pop(step)
        t_frag = time.perf_counter()
        srv_ms[step]["frag_ms"] = 1e3 * (t_frag - tb)
        if store is not None:
            for p in pods:
                m = pu.meta(p)
                try:
                    store.delete_pod(m["namespace"], m["name"])
                except Exception:
                    pass
        elif apisrv is not None:
            if overlap and nxt is not None:
                (n_d, dt_d), created[nxt] = await apisrv.churn(step, nxt)
            else:
                n_d, dt_d = await apisrv.delete(step)
            srv_ms.setdefault(step, {}).update(delete_srv_ms=1e3 * dt_d, peak_ms=1e3 * (t_frag - ts),
                                               delete_rpc_ms=1e3 * (time.perf_counter() - t_frag))
        # the pod controller releases on DELETED; wait until our shares are gone
        await wait_released(rt.state.ledger, uids)
        t_rel = time.perf_counter()
        if pod_ctrl is not None and (pod_ctrl.queue.depth() or pod_ctrl.queue.processing):
            # (read across threads: an empty queue now is what drain() would return at once on)
            await on_ext(pod_ctrl.queue.drain(5.0))
        srv_ms.setdefault(step, {})["drain_ms"] = 1e3 * (time.perf_counter() - t_rel)
        if os.environ.get("NANOGPU_BENCH_DEBUG"):
            print(f"step {step} start {t_step0:.4f} release {ts:.4f} end {time.perf_counter():.4f}", file=sys.stderr)
        hc.__enter__()
        phases = {"create_ms": 1e3 * tc, "schedule_ms": 1e3 * summary["span_s"],
                  "release_ms": 1e3 * (time.perf_counter() - ts)}
        phases.update(srv_ms.pop(step, {}))
        client_s = summary.pop("bind_s_all", [])
        if timed:
            results["client_bind_s"].extend(client_s)
            mark_binds()
            diag = {"t0": round(t_step0, 4), "t1": round(time.perf_counter(), 4)}
            diag.update({k: round(summary.get(k, 0.0), 2) for k in ("cycle_max_ms", "cycle_sum_ms", "cycle_wire_ms", "bind_max_ms")})
            diag["unschedulable"] = summary.get("unschedulable_attempts", 0)
            diag.update({k: round(v, 2) for k, v in phases.items() if k != "schedule_ms"})
            if rt.native is not None:
                fs = rt.native.fe.stats()
                diag["fe_loop_max_ms"] = round(1e3 * fs["loop_max_s"], 2)
                diag["fe_phase_max_ms"] = [round(1e3 * x, 2) for x in fs["phase_max_s"]]
                diag["fe_filter_max_ms"] = round(1e3 * fs["filter"]["max_s"], 2)
                diag["fe_prio_max_ms"] = round(1e3 * fs["priorities"]["max_s"], 2)
                diag["fe_reserve_max_ms"] = round(1e3 * fs["bind_reserve"]["max_s"], 2)
                diag["py_take_wait_max_ms"] = round(1e3 * rt.native.take_wait_max_s, 2)
                rt.native.fe.reset_max()
                rt.native.take_wait_max_s = 0.0
            diag["gc_ms"] = round(1e3 * gc_pause["sum"], 2)
            diag["gc_max_ms"] = round(1e3 * gc_pause["max"], 2)
            gc_pause.update(sum=0.0, max=0.0, n=0)
            diag["t2"] = round(time.perf_counter(), 4)
            results.setdefault("diag", []).append(diag)
        hc.__exit__(None, None, None)
        return {"stats": summary, "frag": frag, "phases": phases}

    from nanogpu.app import tune_gc

    tune_gc()   # what `python -m nanogpu` does after start-up
    import gc

    gc_pause = {"t0": 0.0, "sum": 0.0, "max": 0.0, "n": 0}

    def on_gc(phase, info):   # cyclic-GC pauses of this (extender) process
        if phase == "start":
            gc_pause["t0"] = time.perf_counter()
        else:
            dt = time.perf_counter() - gc_pause["t0"]
            gc_pause["sum"] += dt
            gc_pause["max"] = max(gc_pause["max"], dt)
            gc_pause["n"] += 1

    gc.callbacks.append(on_gc)
    if steady:   # step 0 fills the cluster; then the warm-up churn steps; then the timed ones
        warm_ids, timed_ids = list(range(1 + args.warmup)), list(range(1 + args.warmup, len(stream)))
    else:
        warm_ids, timed_ids = [10_000 + w for w in range(args.warmup)], list(range(args.steps))
    for k, w in enumerate(warm_ids):
        await one_step(w, False, warm_ids[k + 1] if k + 1 < len(warm_ids) else None)
    moved = None
    if d.world == 1 and getattr(args, "_placement", None) and not getattr(args, "no_relocate", False):
        # the job is idle here: if other tenants have moved onto this domain (cores or SMT
        # siblings) since it was picked, move the extender and its stand-in to a quieter one
        from nanogpu import affinity

        pl = args._placement
        to = affinity.quieter_domain(pl["cpus"], pl["numa"], exclude=pl.get("apiserver") or [])
        if to is not None:
            affinity.relocate(pl["pids"], to)
            moved = {"from": pl["cpus"], "to": to}
            pl["cpus"] = to
        if pl.get("apiserver") and pl.get("api_pid"):   # the shared API server's domain likewise
            to = affinity.quieter_domain(pl["apiserver"], pl["numa"], exclude=pl["cpus"])
            if to is not None:
                affinity.relocate([pl["api_pid"]], to)
                moved = dict(moved or {}, apiserver_from=pl["apiserver"], apiserver_to=to)
                pl["apiserver"] = to
                if apisrv is not None:
                    apisrv.cpus = to
    results["relocated"] = moved
    results["rss_mib"] = [rss_mib()]   # the extender process's resident memory, before / after the timed steps
    rt.tracer.buf.clear()
    if rt.native is not None:   # the warm-up steps' bind records
        rt.native.fe.take_bind_wall()
        rt.native.fe.take_bind_hops()
    await barrier()
    d.sync()
    prof = None
    if args.profile_out and d.rank == 0:
        import cProfile

        prof = cProfile.Profile()
        prof.enable()
    sampler = StallSampler() if args.stall_trace and d.rank == 0 else None
    native_prof = bool(args.cpu_profile_out and d.rank == 0 and getattr(args, "_headline", False))
    if native_prof:
        from nanogpu import _native

        native_prof = _native.sampler_start(1000)
    io_tally = bool(args.io_tally and getattr(args, "_headline", False))
    if io_tally:
        from nanogpu import _native

        _native.io_tally_reset()
        _native.io_tally_enable(True)
    nom0 = rt.state.ledger.nomination_counts()
    ctrl0 = pod_ctrl.queue.processed if pod_ctrl is not None else 0
    fe_stats = rt.native.fe.stats if rt.native is not None else (lambda: {})
    handoffs0 = fe_stats().get("bind_handoffs", 0)
    py0 = fe_stats().get("python", {}).get("count", 0)
    prio0 = fe_stats().get("priorities", {}).get("count", 0)
    from nanogpu import affinity

    # other tenants moving onto the rank's domain mid-run: checked every 0.1 s by a harness
    # thread, the job moves to a quieter domain when they keep half a CPU or more of it busy
    # (set up before the clock and the CPU snapshots)
    monitor = None
    if d.world == 1 and getattr(args, "_placement", None) and not getattr(args, "no_relocate", False):
        pl = args._placement
        watch = affinity.ContentionWatch(pl["cpus"], pl["pids"], pl["numa"], exclude=pl.get("apiserver") or [])
        watch.check()
        results["foreign_cpus"] = []
        api_watch = None
        if pl.get("apiserver") and pl.get("api_pid"):
            # the shared API server's domain too: read only (it is never moved mid-run)
            api_watch = affinity.ContentionWatch(pl["apiserver"], [pl["api_pid"]], pl["numa"])
            api_watch.check()
            results["foreign_cpus_api"] = []
        monitor = ContentionMonitor(watch, api_watch, pl, results)
    hc.s = 0.0
    api_cpu0 = apisrv.cpu_s() if apisrv is not None else None   # the shared API server's process
    cpu0, loop_cpu0 = time.process_time(), time.thread_time()
    threads0, ticks0, times0 = thread_cpu(), thread_ticks(), os.times()
    snap0 = affinity.cpu_snapshot()
    t0 = time.perf_counter()
    if sampler is not None:
        sampler.on.set()
    for k, s in enumerate(timed_ids):
        r = await one_step(s, True, timed_ids[k + 1] if k + 1 < len(timed_ids) else None)
        results["steps"].append(r["stats"])
        results["frag"].append(r["frag"])
        results.setdefault("phases", []).append(r["phases"])
        if monitor is not None:
            monitor.steps_done = k + 1
        if k % 100 == 99 and d.rank == 0:   # a long run's heartbeat (one line per 100 steps)
            print(f"bench: {k + 1} timed steps", file=sys.stderr, flush=True)
    if io_tally:
        from nanogpu import _native

        _native.io_tally_enable(False)
        results["io_tally"] = _native.io_tally()
    await barrier()
    d.sync()
    elapsed = time.perf_counter() - t0
    # the clock has stopped: the harness's own records from here (off the timed steps)
    if api_cpu0 is not None:
        results["apiserver_cpu_s"] = apisrv.cpu_s() - api_cpu0
    with hc:
        if monitor is not None:
            monitor.close()
        take_binds()
        spent.clear()
        results["rss_mib"].append(rss_mib())
    if sampler is not None:
        sampler.report(args.stall_trace)
    if native_prof:
        from nanogpu import _native
        from nanogpu.obs import cpu_profile

        Path(args.cpu_profile_out).write_text(json.dumps(cpu_profile(_native.sampler_stop()), indent=1))
    if prof is not None:
        import io
        import pstats

        prof.disable()
        buf = io.StringIO()
        pstats.Stats(prof, stream=buf).sort_stats(os.environ.get("NANOGPU_PROF_SORT", "tottime")).print_stats(45)
        Path(args.profile_out).write_text(buf.getvalue())
    # how busy this rank's cores, their SMT siblings, the API server's and the whole host were
    # while the clock ran (other tenants on the siblings slow every hand-off)
    mine = sorted(os.sched_getaffinity(0))
    groups = {"rank": mine, "rank_smt_siblings": affinity.smt_siblings(mine)} \
        if len(mine) < (os.cpu_count() or 1) else {}
    if apisrv is not None and apisrv.cpus:
        groups.update(apiserver=apisrv.cpus, apiserver_smt_siblings=affinity.smt_siblings(apisrv.cpus))
    results["cpu_busy_pct"] = affinity.busy_report(snap0, affinity.cpu_snapshot(), groups)
    nom1 = rt.state.ledger.nomination_counts()
    results["nominations"] = {k: nom1[k] - nom0[k] for k in nom1}
    # binds a worker answered natively with the pod another worker's filter parsed (the
    # shared ledger's bind handoff): the one-scheduler passes' binds on ranks other than 0
    results["bind_handoffs"] = sum(d.gather_obj(fe_stats().get("bind_handoffs", 0) - handoffs0))
    results["nomination_margin"] = rt.state.ledger.nomination_margin
    # pods the Python pod controller processed (the native watch keeps the rest from it)
    results["controller_keys"] = (pod_ctrl.queue.processed - ctrl0) if pod_ctrl is not None else None
    results["python_requests"] = fe_stats().get("python", {}).get("count", 0) - py0   # routed to Python
    results["unschedulable_attempts"] = sum(st.get("unschedulable_attempts", 0) for st in results["steps"])
    cycles = sum(st.get("cycles", 0) for st in results["steps"])
    results["nodes_sent_per_filter"] = (round(sum(st.get("nodes_sent_filter", 0) for st in results["steps"]) / cycles, 1)
                                        if cycles else None)
    n_sched = max(1, sum(st["scheduled"] for st in results["steps"]))
    cpu1, loop_cpu1 = time.process_time(), time.thread_time()
    threads1, ticks1, times1 = thread_cpu(), thread_ticks(), os.times()
    dthr = {g: threads1[g] - threads0.get(g, 0.0) for g in threads1}
    if ext is not None:
        # the main thread and its executor threads are the harness's alone; the extender's
        # Python loop is the "ngpu-loop" thread
        harness_s = dthr.pop("main", 0.0) + dthr.pop("bench-harness", 0.0)
        dthr["main"] = dthr.pop("ngpu-loop", 0.0)
        loop_s = dthr["main"]
    else:
        dthr["main"] = dthr.get("main", 0.0) - hc.s
        loop_s = loop_cpu1 - loop_cpu0 - hc.s
        harness_s = hc.s + dthr.pop("bench-harness", 0.0)   # the contention monitor's thread
    results["cpu_us_per_pod"] = 1e6 * (cpu1 - cpu0 - harness_s) / n_sched
    if "io_tally" in results:   # (calls, s) by call site -> calls a pod, us a pod, ns a call
        results["io_per_pod"] = {k: [round(n / n_sched, 3), round(1e6 * sec / n_sched, 2), round(1e9 * sec / max(1, n))]
                                 for k, (n, sec) in sorted(results.pop("io_tally").items())}
    results["harness_cpu_us_per_pod"] = 1e6 * harness_s / n_sched
    results["extender_loop_thread"] = ext is not None
    results["cpu_us_per_pod_by_thread"] = {g: round(1e6 * dthr[g] / n_sched, 1) for g in sorted(dthr)}
    # user / kernel split (10 ms ticks: about 1 % resolution over a 20-step run)
    results["cpu_us_per_pod_user_kernel"] = [round(1e6 * (times1.user - times0.user) / n_sched, 1),
                                             round(1e6 * (times1.system - times0.system) / n_sched, 1)]
    kshare = {}
    for g, (u1, k1) in ticks1.items():
        u0, k0 = ticks0.get(g, [0, 0])
        if (u1 - u0) + (k1 - k0) >= 5:
            kshare[g] = round(100.0 * (k1 - k0) / ((u1 - u0) + (k1 - k0)), 1)
    if ext is not None:   # the extender's Python loop reported as "main", as without the split
        kshare.pop("main", None)
        kshare.pop("bench-harness", None)
        if "ngpu-loop" in kshare:
            kshare["main"] = kshare.pop("ngpu-loop")
    results["kernel_pct_by_thread"] = kshare
    results["loop_cpu_us_per_pod"] = 1e6 * loop_s / n_sched
    # the Python part of each bind (API writes + commit): a sub-phase of the wall time
    binds = sorted(s["dur_ms"] for s in rt.tracer.dump(10 ** 9, "bind") if s["ok"])
    results["elapsed_s"] = elapsed
    results["bind_ms"] = binds
    results["scheduled"] = sum(s["scheduled"] for s in results["steps"])
    if rt.native is not None:
        ns = rt.native.fe.stats()
        results["native"] = {v: round(1e6 * ns[v]["seconds_total"] / max(1, ns[v]["count"]), 2)
                             for v in ("filter", "priorities", "filter_wall", "priorities_wall")}
        # priorities runs only when more than one node passed the filter
        results["prio_per_pod"] = round((ns["priorities"]["count"] - prio0) / max(1, results["scheduled"]), 3)
        results["native"]["prio_per_filter"] = round(ns["priorities"]["count"] / max(1, ns["filter"]["count"]), 4)
    results["phase_ms"] = {k: round(statistics.mean(p[k] for p in results["phases"]), 2)
                           for k in ("create_ms", "schedule_ms", "release_ms", "create_srv_ms", "delete_srv_ms")
                           if all(k in p for p in results["phases"])} if results.get("phases") else None
    results["schedule_ms_steps"] = [round(p["schedule_ms"], 1) for p in results.get("phases", [])]
    results["step_diag"] = results.get("diag", [])
    results["client_bind_ms"] = [round(1e3 * x, 4) for x in results.pop("client_bind_s")]
    results["failed"] = sum(s["failed"] for s in results["steps"])
    results["bind_errors"] = sum(s["bind_errors"] for s in results["steps"])
    await client.close()
    if apisrv is not None:
        results["apiserver"] = apisrv.stats()
    await barrier()          # no rank still talks to the shared API server
    await on_ext(rt.stop())
    if ext is not None:
        ext.close()
    if apisrv is not None:
        apisrv.end()
    return results


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
                                  f"({args.apiserver_threads or min(16, max(4, d.world))} IO threads, "
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
        "host_selection": "extender arg-max" if args.no_kube_combine else
                          "kube-scheduler combining (LeastAllocated + BalancedAllocation + 10 x extender)",
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
    drv_proc, conn = None, None
    if not args.inproc_driver:
        # started before anything touches the GPU: a fresh interpreter, no HIP state
        import multiprocessing as mp

        ctx = mp.get_context("spawn")
        conn, child = ctx.Pipe()
        drv_proc = ctx.Process(target=driver_main, args=(child,), daemon=True)
        drv_proc.start()
    api_proc = None
    if int(os.environ.get("RANK", "0")) == 0 and not args.inproc_driver:
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
        shared_api = not args.inproc_api and not args.inproc_driver
        if args.steady_variant_steps > 0 and not args.steady and shared_api:
            # steady-state churn (BASELINE config 5 at scale): the cluster is never emptied
            # placement quality is a property of the deployment that exists: ONE kube-scheduler
            # (with N > 1 ranks, its binds spread over every rank's worker)
            s_args = argparse.Namespace(**{**vars(args), "steady": True, "steps": args.steady_variant_steps,
                                           "warmup": 2, "profile_out": "", "stall_trace": "", "api_rtt_ms": 0.0,
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
                                           "profile_out": "", "stall_trace": "", "api_rtt_ms": 0.0})
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
                                           "steps": args.nodes_variant_steps, "warmup": 1, "profile_out": "",
                                           "stall_trace": "", "api_rtt_ms": 0.0, "one_scheduler": d.world > 1})
            try:
                r = run_pass(d, n_args, topo, conn, "nodes", api_proc)
                nodes_v = (n_args, r, summarize(d, n_args, r))
            except Exception as e:
                nodes_v = {"error": f"{type(e).__name__}: {e}"}
        if args.rtt_variant_ms > 0:
            # the same burst with a modelled API-server round trip on every API call (untimed
            # for `value`; its own clock): what the pods/s above excludes
            v_args = argparse.Namespace(**{**vars(args), "api_rtt_ms": args.rtt_variant_ms,
                                           "steps": args.rtt_variant_steps, "warmup": 1, "profile_out": "",
                                           "stall_trace": ""})
            try:
                variant = summarize(d, v_args, run_pass(d, v_args, topo, conn, "rtt", api_proc))
            except Exception as e:   # the headline result stands; say what failed
                variant = {"error": f"{type(e).__name__}: {e}"}
        if args.decisive_variant_steps > 0 and not args.decisive_filter and not args.steady and not args.compat:
            x_args = argparse.Namespace(**{**vars(args), "decisive_filter": True,
                                           "steps": args.decisive_variant_steps, "warmup": 1,
                                           "profile_out": "", "stall_trace": "", "api_rtt_ms": 0.0})
            try:
                r = run_pass(d, x_args, topo, conn, "decisive", api_proc)
                dec_v = {"res": r, "out": summarize(d, x_args, r)}
            except Exception as e:
                dec_v = {"error": f"{type(e).__name__}: {e}"}
        if args.inproc_variant_steps > 0 and not args.inproc_api and not args.inproc_driver:
            # round 1's extender-isolated setup: an in-process store per rank, no HTTP
            # (each rank its own store: a stand-in per rank, each binding on its own worker)
            i_args = argparse.Namespace(**{**vars(args), "inproc_api": True, "api_rtt_ms": 0.0, "one_scheduler": False,
                                           "steps": args.inproc_variant_steps, "warmup": 1,
                                           "profile_out": "", "stall_trace": ""})
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


def _pct(a: list, q: float):
    return round(a[min(len(a) - 1, int(q * len(a)))], 4) if a else None


# the hops of a native bind (nanogpu/bindhops.h), in order: parse + ledger reserve, hand-off to
# the writer's loop, request built and sent, the API server's answer, commit + reply posted to
# the front door, reply written to kube-scheduler's connection
BIND_HOPS = ("reserve", "handoff", "send", "api", "commit", "reply")


def hop_summary(rows: list) -> dict | None:
    """{hop: [p50, p99, mean over the slowest 1 % of binds]} in us, and the hop that owns the
    tail (largest excess of its tail mean over its p50)."""
    n = len(rows)
    if not n:
        return None
    cols = [sorted(c) for c in zip(*rows)]
    by_total = sorted(range(n), key=lambda i: sum(rows[i]))
    tail = by_total[min(n - 1, int(0.99 * n)):]
    out = {}
    for h, name in enumerate(BIND_HOPS):
        t = sum(rows[i][h] for i in tail) / len(tail)
        out[name] = [round(cols[h][n // 2] / 1e3, 1), round(cols[h][min(n - 1, int(0.99 * n))] / 1e3, 1),
                     round(t / 1e3, 1)]
    owner = max(BIND_HOPS, key=lambda k: out[k][2] - out[k][0])
    return {"us": out, "tail_hop": owner, "n": n}


def hops_by_decile(steps: list) -> dict | None:
    """Each hop's mean (us) over the binds of each tenth of a step, in the order they were
    answered, averaged over the steps: whether a hop's tail sits at the start of a burst (cores
    that slept through the gap between steps) or spreads over it."""
    rows = [[] for _ in range(10)]
    for hops in steps:
        n = len(hops)
        if n < 10:
            continue
        for k, h in enumerate(hops):
            rows[min(9, 10 * k // n)].append(h)
    if not rows[0]:
        return None
    return {name: [round(sum(r[h] for r in rows[dc]) / len(rows[dc]) / 1e3, 1) for dc in range(10)]
            for h, name in enumerate(BIND_HOPS)}


def _first_vs_median(dec: dict | None, hop: str):
    if not dec or hop not in dec:
        return None
    v = dec[hop]
    return [v[0], sorted(v)[len(v) // 2]]


def summarize(d: Dist, args, res: dict) -> dict:
    """Whole-job numbers of one pass (collective: every rank calls it)."""
    elapsed = d.max(res["elapsed_s"])
    rows = [h for r in d.gather_obj(res.get("bind_hops_ns", [])) for h in r]
    hops = hop_summary(rows)
    # the extender's own part of each bind: its wall time (request read -> reply handed to the
    # kernel) without the API server's answer time (the `api` hop)
    ext = sorted(sum(h) - h[BIND_HOPS.index("api")] for h in rows)
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
            # each rank's mean stand-in span per step: the slowest sets the peak barrier
            "schedule_ms_by_rank": [round(v, 2) for v in d.gather_obj((res.get("phase_ms") or {}).get("schedule_ms", 0.0))]}


def _frag_mean(frags: list[dict], key: str = "frag_pct"):
    return round(statistics.mean(f[key] for f in frags), 3) if frags else None


def steady_keys(args, topo, v) -> dict:
    """frag% under steady-state churn, live (second half of the pass's timed steps), with the
    reference algorithm and the native one replayed offline on the same stream."""
    if v is None:
        return {}
    if isinstance(v, dict):
        return {"value_steady": None, "error_steady": v["error"]}
    s_args, res, out = v
    half = res["frag"][len(res["frag"]) // 2:]
    keys = {"value_steady": out["value"], "p50_bind_ms_steady": out["p50_bind_ms"],
            "frag_pct_steady": _frag_mean(half), "frag_hbm_pct_steady": _frag_mean(half, "frag_mib"),
            "frag_pct_steady_each_step": [round(f["frag_pct"], 3) for f in res["frag"]],
            "nominations_steady": res.get("nominations"),
            "bind_handoffs_steady": res.get("bind_handoffs"),
            "steps_steady": s_args.steps, "failed_steady": out["failed"],
            "steady_config": f"{s_args.pods} pods fill {s_args.nodes} nodes, then each step deletes "
                             f"{int(100 * STEADY_CHURN)} % of the live pods and creates as many; frag = mean of "
                             f"the last {len(half)} of {s_args.steps} timed steps"
                             + ("; one kube-scheduler stand-in, binds over every rank's worker"
                                if getattr(s_args, "one_scheduler", False) else "")}
    if args.partition == "SPX" and args.policy == "binpack" and not args.compat:
        from nanogpu import types as T
        from nanogpu.sim import fragsim

        hbm = topo.devices[0].hbm_mib if topo.devices else 288 * 1024
        n_steps = 1 + s_args.warmup + s_args.steps
        kw = dict(steps=n_steps, nodes=s_args.nodes, hbm_mib=hbm, initial=s_args.pods, churn=STEADY_CHURN,
                  seed=STEADY_SEED, first=1 + s_args.warmup + s_args.steps // 2)
        ref = fragsim.steady_state(True, kube=True, **kw)
        # the extender's own verbs replayed offline on the same stream (fragsim.steady_protocol):
        # with the priorities lead the live run matches it step for step at any worker count
        nat = fragsim.steady_protocol(0, lead=T.PRIORITY_LEAD, **kw)
        keys.update(frag_pct_steady_reference_model=ref["frag_pct"],
                    frag_hbm_pct_steady_reference_model=ref["frag_hbm_pct"],
                    frag_pct_steady_native_replay=nat["frag_pct"],
                    frag_pct_steady_native_replay_each_step=nat["frag_pct_each_step"][1 + s_args.warmup:])
    return keys


def cycle_share(res: dict) -> tuple[float | None, float | None, float | None]:
    """Who owns kube-scheduler's serial cycle (filter -> priorities -> host chosen), over the
    pass's timed steps: (share of the cycle the stand-in waited on the extender, request sent ->
    answer read; share the extender held the requests, first byte read -> answer handed to the
    kernel; share its native verbs computed, body parse -> answer built). wire - held is the
    loopback transit plus the stand-in's own send / wake-up / recv; 1 - wire is the stand-in's
    own work (node sampling, request building, plugin scores, host selection)."""
    steps = res.get("steps") or []
    cyc = sum(st.get("cycle_sum_ms", 0.0) for st in steps)
    wire = sum(st.get("cycle_wire_ms", 0.0) for st in steps)
    n = sum(st.get("cycles", 0) for st in steps)
    nat = res.get("native") or {}
    if cyc <= 0:
        return None, None, None
    pp = nat.get("prio_per_filter", 1.0)
    verbs_ms = n * (nat.get("filter", 0.0) + pp * nat.get("priorities", 0.0)) / 1e3
    held_ms = n * (nat.get("filter_wall", 0.0) + pp * nat.get("priorities_wall", 0.0)) / 1e3
    return round(wire / cyc, 3), round(held_ms / cyc, 3), round(verbs_ms / cyc, 3)


def nodes_variant_keys(args, topo, v) -> dict:
    """The --nodes-variant pass: pods/s, frag%, the reference model's frag% on the same bursts
    and node sampling, and how often kube-scheduler's choice agreed with the nomination."""
    if v is None:
        return {}
    tag = f"nodes{args.nodes_variant}"
    if isinstance(v, dict):
        return {f"value_{tag}": None, f"error_{tag}": v["error"]}
    n_args, res, out = v
    nom = res.get("nominations") or {}
    keys = {f"value_{tag}": out["value"], f"p50_bind_ms_{tag}": out["p50_bind_ms"],
            f"frag_pct_{tag}": _frag_mean(res["frag"]), f"failed_{tag}": out["failed"],
            f"unschedulable_{tag}": out["unschedulable"], f"steps_{tag}": n_args.steps,
            f"pods_per_burst_{tag}": n_args.pods,
            f"nomination_adopt_pct_{tag}": round(100.0 * nom["adopted"] / nom["made"], 2) if nom.get("made") else None,
            f"nominations_{tag}": nom,
            f"nodes_sent_per_filter_{tag}": res.get("nodes_sent_per_filter"),
            f"schedulers_{tag}": "one kube-scheduler stand-in, binds over every rank's worker"
            if getattr(n_args, "one_scheduler", False) else "one kube-scheduler stand-in per rank",
            f"native_verb_mean_us_{tag}": res.get("native")}
    (keys[f"extender_share_of_cycle_{tag}"], keys[f"extender_held_share_of_cycle_{tag}"],
     keys[f"extender_verb_share_of_cycle_{tag}"]) = cycle_share(res)
    st = res.get("steps") or []
    if st and sum(x.get("cycles", 0) for x in st):
        keys[f"cycle_us_{tag}"] = round(1e3 * sum(x.get("cycle_sum_ms", 0.0) for x in st)
                                        / sum(x.get("cycles", 0) for x in st), 1)
    if args.partition == "SPX" and args.policy == "binpack" and not args.compat:
        from nanogpu.sim import fragsim

        hbm = topo.devices[0].hbm_mib if topo.devices else 288 * 1024
        kw = dict(steps=n_args.steps, nodes=n_args.nodes, hbm_mib=hbm, pods=n_args.pods, kube=True)
        keys[f"frag_pct_{tag}_reference_model"] = fragsim.headline(True, **kw)["frag_pct"]
        keys[f"frag_pct_{tag}_native_replay"] = fragsim.headline(False, **kw)["frag_pct"]
    return keys


def reference_model_frag(args, topo) -> dict:
    """frag% of the reference algorithm (compat mode: the Go raters bit for bit) on the same
    bursts, replayed offline through the same ledger (nanogpu.sim.fragsim) — the reference
    publishes no number; this is its placement on this workload. Also the native replay, so
    the live run's frag_pct can be checked against a serial replay."""
    if args.partition != "SPX" or args.policy != "binpack" or args.compat:
        return {"frag_pct_reference_model": None}
    from nanogpu.sim import fragsim

    hbm = topo.devices[0].hbm_mib if topo.devices else 288 * 1024
    kw = dict(steps=args.steps, nodes=args.nodes, hbm_mib=hbm, pods=args.pods, kube=not args.no_kube_combine)
    ref, nat = fragsim.headline(True, **kw), fragsim.headline(False, **kw)
    return {"frag_pct_reference_model": ref["frag_pct"], "frag_hbm_pct_reference_model": ref["frag_hbm_pct"],
            "stranded_pct_reference_model": ref["stranded_pct"], "frag_pct_native_replay": nat["frag_pct"],
            "frag_reference_model_source": "offline serial replay of the timed bursts behind the same "
                                           "kube-scheduler model (node sampling, NodeResourcesFit, plugin "
                                           "scores, PodTopologySpread, 10 x extender), reference binpack "
                                           "(compat mode, bit-exact with rater.go) vs native binpack"}


if __name__ == "__main__":
    sys.exit(main())
