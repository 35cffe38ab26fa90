"""The bench harness behind bench.py: what one rank runs for one pass, and the helpers the
headline line is built from (bench.py keeps the driver contract: arguments, the launcher, the
ranks' collectives, the pass sequence and the JSON line).

  * the node model of the discovered MI355X (node_template, measured_links: HIP probe, KFD
    io_link rates, the peer-pull matrix over every visible pair);
  * the workload (bench bursts and the steady-churn stream, nanogpu.sim.workload);
  * the shared API server process (apiserver_main / ApiServerProc: native/src/apiserver.cpp) and
    the kube-scheduler stand-in process (driver_main: native/src/schedsim.cpp);
  * run_rank: one extender worker (nanogpu.app.Runtime on a loop thread of its own) driven
    through the timed steps, with the per-step and per-thread records;
  * the summaries the line reports (bind hop split, cycle share, frag replays of the reference
    algorithm and of the extender's own verbs on the same streams: nanogpu.sim.fragsim).
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
    # without a GPU (--no-gpu rehearsals) the node is the MI355X the box reports: amdgpu's VRAM
    # size there is 294,896 MiB (tests/fixtures/sysfs/mi355x_real), 16 MiB under 288 GiB, which
    # moves HBM fits at the margin: the rehearsal and the GPU run then schedule the same node
    hbm_mib = MI355X_VRAM_MIB
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
MI355X_VRAM_MIB = 294_896   # amdgpu's VRAM of one MI355X as the box reports it (mem_info_vram_total)
INFLIGHT_BINDS = 64   # the stand-in's binds in flight in Python mode, and the harness's API client pool
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
        if op == "start":   # a fresh server: (IO threads, modelled RTT s, spin window s, mutating limit)
            _, threads, latency_s, spin_s, max_inflight = msg
            if srv is not None:
                srv.stop()
            steps.clear()
            keys.clear()
            # watch cache: 64k events per kind. A burst makes about 4k (create, bind, label,
            # delete): from the ~16th step on every event evicts an old version, freed under the
            # store's lock (profiles/soak_r05.md)
            srv = core().ApiServer("127.0.0.1", 0, threads, 1 << 16)
            srv.set_latency(latency_s)
            # polling only on CPUs of its own: on the ranks' cores it would take them from the extender
            own = not (set(os.sched_getaffinity(0)) & set(avoid or []))
            spin = spin_s if spin_s > 0 and own else 0.0
            if spin > 0:
                srv.set_spin(spin)
            # kube-apiserver's default --max-mutating-requests-inflight: over it, 429 + Retry-After
            srv.set_max_mutating_inflight(max_inflight)
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

    def start(self, threads: int, latency_s: float = 0.0, spin_s: float = 0.0, max_inflight: int = 0) -> str:
        port, self.cpus, self.spin_s = self._rpc("start", threads, latency_s, spin_s, max_inflight)
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
    """kube-scheduler stand-in in its own process (as in a real cluster; native/src/schedsim.cpp):
    for each pass of the bench it receives the extender's address and the pass's steps, builds
    their pods, then for every step schedules that step's pods (already created in the API
    server) and returns the driver stats. The scheduling cycle is serial on one keep-alive
    connection; each bind leaves as soon as its host is chosen (kube-scheduler's per-pod bind
    goroutines), on the connections of an epoll binder."""
    from nanogpu.native import core
    from nanogpu.sim.driver import NativeSchedulerDriver
    from nanogpu.sim.kubescore import KubeScoring

    st = {"cfg": None, "work": {}, "session": None, "live": {}, "specs": {}, "stream": None}

    def configure(cfg: dict) -> None:
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
                work[step] = NativeSchedulerDriver.prepare_native([steady_pod(s) for s in specs])
        for step in ([] if cfg.get("steady") else cfg["steps"]):
            if cfg.get("bind_ports"):   # the one scheduler of the job: every rank's pods
                pods = [p for r in range(cfg["world"]) for p in burst(r, cfg["world"], cfg["pods"], step, 7)]
            else:
                pods = burst(cfg["rank"], cfg["world"], cfg["pods"], step, 7)
            work[step] = NativeSchedulerDriver.prepare_native(pods)
        cfg["kube_obj"] = KubeScoring() if cfg.get("kube") else None
        # keep-alive connections across the pass's steps
        st.update(cfg=cfg, work=work, session=core().SchedulerSession())
        conn.send("ready")

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
        cfg, work, step = st["cfg"], st["work"], msg[1]
        drv = NativeSchedulerDriver("127.0.0.1", cfg["port"], cfg["names"], cfg["caps"], seed=step * 1009 + cfg["rank"],
                                    session=st["session"], bind_threads=256, kube=cfg["kube_obj"],
                                    bind_ports=cfg.get("bind_ports"))
        placed = []
        if st["stream"] is not None:
            live = st["live"]
            for key in st["stream"][step].deletes:
                live.pop(key, None)
            stats = drv.run(prepared=work.pop(step), live=list(live.values()))
            args_k, node_of = drv._placed[-1]
            idx = cfg["name_index"]
            for spec, a, node in zip(st["specs"].pop(step), args_k, node_of):
                if node:
                    live[spec.key] = (idx[node], a[4], a[5], a[6], a[7])
                    placed.append((spec.key, live[spec.key]))
        else:
            stats = drv.run(prepared=work.pop(step))
        sm = stats.summary()
        if st["stream"] is not None:
            sm["live_placed"] = placed   # for the other ranks' stand-ins (their informers)
        conn.send(sm)
        # the step's driver and pod records are freed at the next configure, not inside the
        # next step's clock (thousands of objects)
        drv.close()
        st.setdefault("spent", []).append(drv)


async def run_rank(d: Dist, args, topo, ledger_path: str, conn=None, api_proc: ApiServerProc | None = None) -> dict:
    from nanogpu import types as T
    from nanogpu.app import Config, Runtime
    from nanogpu.k8s import podutil as pu
    from nanogpu.k8s.fake_apiserver import Faults, FakeKubeStore, InProcKube
    from nanogpu.sim.driver import node_capacities
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
    ext = ExtenderLoop() if shared else None
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
            url = apisrv.start(args.apiserver_threads or 4, args.api_rtt_ms / 1e3,
                               args.apiserver_spin_us / 1e6,
                               T.API_MAX_MUTATING_INFLIGHT)
            if getattr(args, "_placement", None):
                args._placement["apiserver"] = list(apisrv.cpus)
            apisrv.add_nodes(nodes)
        url = d.bcast_obj(url)
        from nanogpu.k8s.client import KubeClient, KubeConfig

        def rt_api_make():
            return KubeClient(KubeConfig(server=url), pool=INFLIGHT_BINDS + 8,
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
                 busy_poll_us=args.busy_poll_us, busy_poll_prio_us=args.busy_poll_prio_us,
                 frontend_threads=args.frontend_threads,
                 bind_writer_threads=max(2, 16 // d.world),
                 bind_writer_mode=args.bind_writer_mode, assume_label=not args.no_assume_label,
                 # every rank's extender writes to the one API server: they share its in-flight limit
                 api_inflight_share=d.world if shared else 1,
                 spin_recv=args.spin_recv, spin_recv_binds=args.spin_recv_binds,
                 decisive_filter=getattr(args, "decisive_filter", False))
    all_steps_pre = [10_000 + w for w in range(args.warmup)] + list(range(args.steps))

    async def start_runtime():   # built and started on the extender's loop
        r = Runtime(cfg, worker=d.rank if shared else 0, api=rt_api_make())
        await r.start()
        return r

    rt = await on_ext(start_runtime())
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
                   "pods": args.pods, "inflight": INFLIGHT_BINDS, "kube": True,
                   "steady": {"warmup": args.warmup, "steps": args.steps, "pods": args.pods} if steady else None,
                   "steps": list(range(len(stream))) if steady else
                   [10_000 + w for w in range(args.warmup)] + list(range(args.steps))})
        await loop.run_in_executor(None, conn.recv)   # the stand-in has built its pods

    # The workload's clients create the next burst while the pod controller releases this one
    # (delete, then create, in the API server; the scheduling of the next burst still starts
    # only after every release). Each timed step's create and release stay inside the clock:
    # the first timed burst is created in the timed region, never during a warm-up release.
    overlap = apisrv is not None
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
    if d.world == 1 and getattr(args, "_placement", None):
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
    if d.world == 1 and getattr(args, "_placement", None):
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
    if native_prof:
        from nanogpu import _native
        from nanogpu.obs import cpu_profile

        Path(args.cpu_profile_out).write_text(json.dumps(cpu_profile(_native.sampler_stop()), indent=1))
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
        kws = rt.native.fe.kube_writer_stats()
        results["bindings_first"] = kws.get("bindings_first") if kws else None
    results["phase_ms"] = {k: round(statistics.mean(p[k] for p in results["phases"]), 2)
                           for k in ("create_ms", "schedule_ms", "release_ms", "create_srv_ms", "delete_srv_ms")
                           if all(k in p for p in results["phases"])} if results.get("phases") else None
    results["schedule_ms_steps"] = [round(p["schedule_ms"], 1) for p in results.get("phases", [])]
    results["step_diag"] = results.get("diag", [])
    results["client_bind_ms"] = [round(1e3 * x, 4) for x in results.pop("client_bind_s")]
    results["failed"] = sum(s["failed"] for s in results["steps"])
    results["bind_errors"] = sum(s["bind_errors"] for s in results["steps"])
    if apisrv is not None:
        results["apiserver"] = apisrv.stats()
    await barrier()          # no rank still talks to the shared API server
    await on_ext(rt.stop())
    if ext is not None:
        ext.close()
    if apisrv is not None:
        apisrv.end()
    return results


def _pct(a: list, q: float):
    return round(a[min(len(a) - 1, int(q * len(a)))], 4) if a else None


# the hops of a native bind (nanogpu/bindhops.h), in order: parse + ledger reserve, hand-off to
# the writer's loop, request built and sent, the API server's answer, commit + reply posted to
# the front door, reply written to kube-scheduler's connection
# the writer's wait for room in the admission window ("window": every slot held by unanswered
# API requests) is the API server's backpressure, apart from the writer's own send
BIND_HOPS = ("reserve", "handoff", "window", "send", "api", "commit", "reply")


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

        hbm = topo.devices[0].hbm_mib if topo.devices else MI355X_VRAM_MIB
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

        hbm = topo.devices[0].hbm_mib if topo.devices else MI355X_VRAM_MIB
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

    hbm = topo.devices[0].hbm_mib if topo.devices else MI355X_VRAM_MIB
    kw = dict(steps=args.steps, nodes=args.nodes, hbm_mib=hbm, pods=args.pods, kube=True)
    ref, nat = fragsim.headline(True, **kw), fragsim.headline(False, **kw)
    return {"frag_pct_reference_model": ref["frag_pct"], "frag_hbm_pct_reference_model": ref["frag_hbm_pct"],
            "stranded_pct_reference_model": ref["stranded_pct"], "frag_pct_native_replay": nat["frag_pct"],
            "frag_reference_model_source": "offline serial replay of the timed bursts behind the same "
                                           "kube-scheduler model (node sampling, NodeResourcesFit, plugin "
                                           "scores, PodTopologySpread, 10 x extender), reference binpack "
                                           "(compat mode, bit-exact with rater.go) vs native binpack"}
