"""Process wiring: informers, controllers, policy reload, telemetry, HTTP server, workers.

Reference: cmd/main.go:75-137 (flags -> rater -> clientset -> signals -> informer factory
-> controller -> DSContext -> verbs -> router -> ListenAndServe). Differences:
  * the ledger is rebuilt after the informers sync (reference builds the dealer before
    WaitForCacheSync, SURVEY §3.1 ordering hazard);
  * `workers > 1` forks SO_REUSEPORT replicas that share one native ledger in /dev/shm;
    worker 0 is the leader (pod controller, telemetry, reservation sweeper), every worker
    runs a node informer and serves all verbs;
  * first SIGINT/SIGTERM drains, a second exits(1) (reference signals.go:16-30).
"""
from __future__ import annotations

import asyncio
import logging
import os
import signal
import time
import sys
from dataclasses import dataclass, field

from . import types as T

log = logging.getLogger("nanogpu")


@dataclass
class Config:
    priority: str = T.PRIORITY_BINPACK
    policy_config_path: str = T.DEFAULT_POLICY_PATH
    prometheus_url: str = T.DEFAULT_PROMETHEUS_URL
    instance_port: str = "9100"                 # accepted for flag compatibility (unused, as in the reference)
    sync_period_s: float = 5.0
    is_load_schedule: bool = False
    port: int = T.DEFAULT_PORT
    host: str = "0.0.0.0"
    threadness: int = 1
    kubeconfig: str | None = None
    kube_api: str | None = None                 # explicit API server URL (tests / fake cluster)
    compat: bool = False
    score_normalize: bool = False
    topology_weight: float = 1.0
    track_hbm: bool = True
    workers: int = 1
    ledger_path: str = ""
    max_nodes: int = 4096
    max_pods: int = 131072
    verify_pod_on_bind: bool = False
    native_bind_writes: bool = True             # C++ writer threads do the bind's API writes
    bind_writer_threads: int = 16               # x KubeWriter::kBatch (8) binds in flight (threads mode,
    #                                             and evented / inline when api_max_inflight is 0)
    api_max_inflight: int = T.API_MAX_MUTATING_INFLIGHT   # kube-apiserver's mutating in-flight limit
    api_inflight_share: int = 0                 # extender processes sharing it (0: `workers`)
    bind_writer_mode: str = "evented"           # inline (front-door workers) | evented (one epoll thread) |
    #                                             frontdoor (front-door workers send, one epoll thread reads) | threads
    native_pod_watch: bool = True               # a C++ thread reads and filters the pod watch (podwatch.cpp)
    # the reference's `nano-gpu/assume` label, PATCHed beside the binding; off: one write a bind
    # (the binding carries the annotations; this project's agent selects pods by node)
    assume_label: bool = True
    bind_first: bool = False                    # front door: a batch's binds before its filters
    spin_nap: bool = False                      # front door: sleep the busy-poll window, not poll it
    spin_recv: bool = True                      # front door: poll the last cycle answer's connection with recv first
    spin_recv_binds: bool = False               # ... then the last bind answer's
    batch_labels: bool = False                  # native writer: batch label PATCHes after bindings (off: pipelined)
    lazy_label_answers: bool = False            # native writer: read label PATCH answers lazily (no wake-up each)
    watch_assigned_only: bool = True            # pod informer: bound pods only (spec.nodeName!=)
    api_write_timeout_s: float = 30.0           # native bind writer: an API answer due within this
    reservation_ttl_s: float = 60.0
    nominate: bool = True              # priorities nominate the top node (Ledger::nominate)
    decisive_filter: bool = False      # filter answers only the top node (one round trip a pod)
    priority_lead: int = T.PRIORITY_LEAD   # priorities: the nominated node's lead (0: off)
    nomination_ttl_s: float = 5.0
    policy_reload_s: float = 3.0
    fake_cluster: int = 0                       # >0: serve against an in-process fake cluster of N nodes
    fake_gpus_per_node: int = 8
    fake_partition: str = "SPX"
    seed: int = 0
    frontend: str = "native"                    # native (C++ epoll front door) | aiohttp
    leader_elect: bool = False                  # Lease-based active/standby replicas
    lease_name: str = "nano-gpu-scheduler"
    lease_namespace: str = "kube-system"
    lease_duration_s: float = 15.0
    lease_renew_deadline_s: float = 10.0
    lease_retry_s: float = 2.0
    identity: str = ""
    frontend_threads: int = 4
    busy_poll_us: int = 0                       # native workers spin this long after an event
    busy_poll_prio_us: int = -1                 # ... after a priorities answer (-1: busy_poll_us)
    cpu_affinity: str = "none"                  # none | auto (one L3 domain per worker) | cpu list
    request_sizes: list = field(default_factory=list)   # share sizes binpack's waste model fixes
    learn_sizes: bool = True                    # ...plus the sizes the ledger sees requested
    gpu_node_selectors: list = field(default_factory=lambda: [T.AMD_GPU_NODE_LABEL, T.LEGACY_GPU_NODE_LABEL])

    def writer_max_binds(self) -> int:
        """Binds one worker's native writer keeps in flight at most (its admission window's start
        and ceiling): 3/4 of kube-apiserver's mutating in-flight limit, shared by the extender's
        processes, a bind being two mutating requests with the label PATCH (one without). The
        rest of the limit is left to the cluster's other clients. 0: bind_writer_threads x 8."""
        if self.api_max_inflight <= 0:
            return 0
        share = self.api_inflight_share or max(1, self.workers)
        per_bind = 2 if self.assume_label else 1
        return max(2, (3 * self.api_max_inflight // 4) // (share * per_bind))


class Runtime:
    """Everything one worker process runs; also used in-process by tests and the bench."""

    def __init__(self, cfg: Config, worker: int = 0, api=None):
        from .extender.verbs import Extender
        from .obs import Metrics, Tracer
        from .state.cluster import ClusterState

        self.cfg = cfg
        self.worker = worker
        self.leader = worker == 0
        self.api = api
        self.node_informer = None
        self.pod_informer = None
        self.state = ClusterState(
            policy=cfg.priority, compat=cfg.compat, load_aware=cfg.is_load_schedule,
            topo_weight=cfg.topology_weight, seed=cfg.seed, ledger_path=cfg.ledger_path,
            max_nodes=cfg.max_nodes, max_pods=cfg.max_pods, track_hbm=cfg.track_hbm,
            node_source=self._node_from_cache, score_normalize=cfg.score_normalize, nominate=cfg.nominate,
            request_sizes=cfg.request_sizes, learn_sizes=cfg.learn_sizes, decisive_filter=cfg.decisive_filter,
            priority_lead=cfg.priority_lead)
        self.metrics = Metrics()
        self.tracer = Tracer()
        self.extender: Extender | None = None
        self.ready = asyncio.Event()
        self.tasks: list[asyncio.Task] = []
        self.controllers = []
        self.poller = None
        self.watcher = None
        self.runner = None
        self.native = None
        self.elector = None
        self.router = None
        self.bound_port = 0
        self._fake = None

    def _node_from_cache(self, name: str):
        return self.node_informer.get(name) if self.node_informer else None

    async def _make_api(self):
        if self.api is not None:
            return self.api
        if self.cfg.fake_cluster > 0:
            from .k8s import podutil as pu
            from .k8s.fake_apiserver import FakeKubeStore, InProcKube
            from .topology.model import synthetic_mi355x

            store = FakeKubeStore()
            topo = synthetic_mi355x(self.cfg.fake_gpus_per_node, self.cfg.fake_partition).to_json()
            devices = self.cfg.fake_gpus_per_node * {"SPX": 1, "DPX": 2, "QPX": 4, "CPX": 8}[self.cfg.fake_partition]
            for i in range(self.cfg.fake_cluster):
                store.add_node(pu.make_node(f"mi355x-{i}", devices, topo, {"amd.com/gpu.present": "true"}))
            self._fake = store
            return InProcKube(store)
        from .k8s.client import KubeClient, KubeConfig

        return KubeClient(KubeConfig.auto(self.cfg.kubeconfig, self.cfg.kube_api),
                          native_watch=self.cfg.native_pod_watch)

    async def start(self, serve: bool = True) -> None:
        from .config.policy import PolicyWatcher
        from .controller.pods import NodeController, PodController
        from .extender import server
        from .extender.verbs import Extender
        from .k8s.informer import Informer

        self.api = await self._make_api()
        self.node_informer = Informer(self.api, "nodes", resync_s=self.cfg.sync_period_s)
        self.controllers.append(NodeController(self.state, self.node_informer))
        self.tasks.append(self.node_informer.start())
        if self.leader:
            # the controllers read a pod's identity, nano-gpu/* annotations and limits, node
            # and phase: the REST watch decodes just those (native), not the whole object
            # assigned pods only (`spec.nodeName!=`, the selector kube-scheduler's own informer
            # uses for them): a pending pod is the extender's business through its verbs, not
            # the controller's, and an unschedulable pod's condition updates never reach us
            self.pod_informer = Informer(self.api, "pods", slim=True, prefilter=self.state.ledger,
                                         field_selector=T.ASSIGNED_PODS if self.cfg.watch_assigned_only else None)
            pc = PodController(self.state, self.pod_informer, workers=self.cfg.threadness, metrics=self.metrics,
                               relabel=self._relabel if self.cfg.assume_label else None)
            self.controllers.append(pc)
            pc.start()
            self.tasks.append(self.pod_informer.start())
        await self.node_informer.synced.wait()
        if self.pod_informer is not None:
            await self.pod_informer.synced.wait()
            await self.controllers[-1].queue.drain(30.0)   # initial ADDs rebuild the ledger
        self.extender = Extender(self.state, self.api, self.metrics, self.tracer,
                                 verify_pod_on_bind=self.cfg.verify_pod_on_bind, assume_label=self.cfg.assume_label)
        # policy file: real hot reload
        self.watcher = PolicyWatcher(self.cfg.policy_config_path, self.cfg.policy_reload_s)
        self.watcher.subscribe(self._apply_policy)
        if self.cfg.is_load_schedule and self.leader:
            from .telemetry.poller import LoadPoller
            from .telemetry.prom import PromClient

            self.poller = LoadPoller(self.state, PromClient(self.cfg.prometheus_url), self.node_informer.list,
                                     selectors=self.cfg.gpu_node_selectors, metrics=self.metrics,
                                     get_node=self.node_informer.get)
            self.watcher.subscribe(self.poller.on_policy)
        self.watcher.load_now()
        if os.path.exists(self.cfg.policy_config_path):
            self.tasks.append(self.watcher.start())
        elif self.cfg.is_load_schedule:
            log.warning("load-aware scheduling enabled but %s is missing; no metrics will be polled",
                        self.cfg.policy_config_path)
        if self.leader:
            self.tasks.append(asyncio.ensure_future(self._sweeper()))
        if self.cfg.leader_elect and self.leader:
            # not before the Lease says so; the other workers read the same shared flag
            self.state.ledger.serving = False
        self.ready.set()
        if self.cfg.leader_elect and self.leader:
            import socket

            from .k8s.lease import LeaderElector

            ident = self.cfg.identity or f"{socket.gethostname()}-{os.getpid()}"
            self.elector = LeaderElector(self.api, ident, self.cfg.lease_namespace, self.cfg.lease_name,
                                         self.cfg.lease_duration_s, self.cfg.lease_renew_deadline_s,
                                         self.cfg.lease_retry_s, on_change=self._on_leadership)
            self.tasks.append(self.elector.start())
        if serve:
            router = server.Router(self.extender, self.ready)
            self.router = router
            router.extra_metrics = self._informer_metrics
            if self.cfg.leader_elect:
                # every worker of the replica follows the elector's flag in the shared ledger
                # (only worker 0 runs the elector)
                ledger = self.state.ledger
                router.serving = lambda: ledger.serving
            if self.cfg.frontend == "native":
                self.native = server.NativeServer(router, self.cfg.host, self.cfg.port, self.cfg.frontend_threads)
                self.native.fe.set_serving(True)   # the ledger's shared flag gates it as well
                self.native.fe.set_busy_poll_us(self.cfg.busy_poll_us)
                self.native.fe.set_busy_poll_prio_us(self.cfg.busy_poll_prio_us)
                self.native.fe.set_bind_first(self.cfg.bind_first)
                self.native.fe.set_spin_nap(self.cfg.spin_nap)
                self.native.fe.set_spin_recv(self.cfg.spin_recv)
                self.native.fe.set_spin_recv_binds(self.cfg.spin_recv_binds)
                api_cfg = getattr(self.api, "config", None)
                if self.cfg.native_bind_writes and not self.cfg.verify_pod_on_bind and api_cfg is not None:
                    ext = self.extender
                    if self.native.enable_native_writes(api_cfg, self.cfg.bind_writer_threads, ext.api_retries,
                                                        ext.record_events, self.cfg.bind_writer_mode != "threads",
                                                        self.cfg.assume_label, self.cfg.api_write_timeout_s,
                                                        self.cfg.bind_writer_mode == "inline",
                                                        self.cfg.batch_labels, self.cfg.writer_max_binds()):
                        log.info("worker %d: bind API writes in native writer threads (%d)", self.worker,
                                 self.cfg.bind_writer_threads)
                        self.native.fe.set_fe_send(self.cfg.bind_writer_mode == "frontdoor")
                        self.native.fe.set_lazy_labels(self.cfg.lazy_label_answers)
                self.native.start()
                self.bound_port = self.native.port
            else:
                app = server.make_app(self.extender, self.ready, router=router)
                self.runner, self.bound_port = await server.start(app, self.cfg.host, self.cfg.port,
                                                                  reuse_port=self.cfg.workers > 1)
            log.info("worker %d serving on :%d (%s front door, policy=%s compat=%s)", self.worker, self.bound_port,
                     self.cfg.frontend, self.state.policy, self.state.options.compat)

    async def _relabel(self, ns: str, name: str, node: str) -> None:
        """The assume label of a placed pod, guarded by its node (podutil.label_patch)."""
        from .k8s import podutil as pu

        await self.api.patch_pod(ns, name, pu.label_patch(node))

    def _informer_metrics(self) -> bytes:
        f = self.pod_informer.watch_filter if self.pod_informer is not None else None
        if f is None:
            return b""
        return ("# HELP nanogpu_pod_watch_native_released_total deleted pods released by the native watch filter\n"
                "# TYPE nanogpu_pod_watch_native_released_total counter\n"
                f"nanogpu_pod_watch_native_released_total {f.released}\n"
                "# HELP nanogpu_pod_watch_dropped_total pod events the native filter kept from the controller\n"
                "# TYPE nanogpu_pod_watch_dropped_total counter\n"
                f"nanogpu_pod_watch_dropped_total {f.dropped}\n").encode()

    def _on_leadership(self, leader: bool) -> None:
        self.state.ledger.serving = leader

    def _apply_policy(self, spec) -> None:
        pol = spec.policy or self.state.policy
        self.state.set_policy(pol, compat=spec.compat, topo_weight=spec.topology_weight)
        if spec.score_normalize is not None:
            self.state.score_normalize = bool(spec.score_normalize)

    async def _sweeper(self) -> None:
        period = min(max(1.0, self.cfg.reservation_ttl_s / 4), max(0.05, self.cfg.nomination_ttl_s / 4))
        next_res = 0.0
        loop = asyncio.get_running_loop()
        # the scans walk the whole shared pod table with the GIL released: off the event loop
        while True:
            await asyncio.sleep(period)
            gone = await loop.run_in_executor(None, self.state.sweep_nominations, self.cfg.nomination_ttl_s)
            if gone:
                log.info("released %d nominations no bind adopted", len(gone))
            removed = self.state.retry_removals()
            if removed:
                log.info("removed deleted nodes once their last shares went: %s", ", ".join(removed))
            if loop.time() < next_res:
                continue
            next_res = loop.time() + max(1.0, self.cfg.reservation_ttl_s / 4)
            stale = await loop.run_in_executor(None, self.state.sweep_reservations, self.cfg.reservation_ttl_s)
            if stale:
                log.warning("released %d stale reservations", len(stale))
            if self.poller is not None:
                self.poller.sweep_stale()

    async def stop(self) -> None:
        if self.elector is not None:
            await self.elector.release()
        if self.native is not None:
            await self.native.stop()
        if self.runner is not None:
            await self.runner.cleanup()
        for c in self.controllers:
            if hasattr(c, "stop"):
                await c.stop()
        if self.poller is not None:
            await self.poller.stop()
        for t in self.tasks:
            t.cancel()
        for t in self.tasks:
            try:
                await t
            except (asyncio.CancelledError, Exception):
                pass
        for inf in (self.node_informer, self.pod_informer):
            if inf is not None:
                await inf.stop()
        if self.extender is not None:
            await self.extender.drain()
        if self.api is not None and hasattr(self.api, "close"):
            await self.api.close()


def tune_gc(gen0: int = 100_000) -> None:
    """Fewer, cheaper cyclic-GC passes for a long-lived server: the request path allocates
    many short-lived dicts (JSON bodies, watch events) while the informer caches hold a
    large, stable object graph that every default-threshold full collection would rescan.
    Objects alive after start-up are frozen out of collection."""
    import gc

    gc.collect()
    gc.freeze()
    gc.set_threshold(gen0, 50, 100)


async def serve_forever(cfg: Config, worker: int = 0) -> int:
    rt = Runtime(cfg, worker)
    loop = asyncio.get_running_loop()
    stop = asyncio.Event()
    hits = {"n": 0}

    def on_signal():
        hits["n"] += 1
        if hits["n"] > 1:
            os._exit(1)
        stop.set()

    for sig in (signal.SIGINT, signal.SIGTERM):
        loop.add_signal_handler(sig, on_signal)
    await rt.start()
    tune_gc()
    await stop.wait()
    await rt.stop()
    return 0


def pin_worker(cfg: Config, worker: int) -> list[int]:
    """--cpu-affinity: `auto` gives each worker process its own L3 domain (nanogpu.affinity),
    an explicit list ("0-7,16") pins every worker to it; `none` leaves placement to the OS."""
    from . import affinity

    if cfg.cpu_affinity in ("", "none"):
        return []
    if cfg.cpu_affinity == "auto":
        cpus = affinity.pick_cpus(-1, worker, [-1] * cfg.workers if cfg.workers > 1 else None)
    else:
        cpus = affinity._parse_list(cfg.cpu_affinity)
    if affinity.apply(cpus):
        log.info("worker %d pinned to CPUs %s", worker, cpus)
        return cpus
    return []


def _drop_stale_region(path: str) -> None:
    """The server owns its region. One left behind by a previous incarnation (SIGKILL, OOM:
    /dev/shm outlives a container restart, and pid 1 names the same path again) holds pods
    that may have been deleted meanwhile, and nothing would ever release them: start clean.
    The ledger is rebuilt from the API server (the checkpoint) before serving."""
    try:
        os.unlink(path)
        log.warning("removed a stale ledger region at %s", path)
    except FileNotFoundError:
        pass


def guard_busy_poll(cfg: Config) -> None:
    """--busy-poll-us is switched off when the replica's CPUs cannot hold every spinning
    front-door thread (`affinity.busy_poll_fits`)."""
    from . import affinity

    if cfg.busy_poll_us <= 0 or cfg.frontend != "native":
        return
    cores = affinity.available_cores()
    if not affinity.busy_poll_fits(cfg.workers, cfg.frontend_threads, cores):
        log.warning("busy-poll off: %d worker(s) x %d front-door threads + loops need %d cores, %.1f available",
                    cfg.workers, cfg.frontend_threads, cfg.workers * (cfg.frontend_threads + 1), cores)
        cfg.busy_poll_us = 0
        cfg.busy_poll_prio_us = 0


def check_region_space(path: str, max_nodes: int, max_pods: int) -> None:
    """The shared ledger is a file on a tmpfs (/dev/shm, an emptyDir with medium Memory in the
    deployment): a region larger than the filesystem's free space maps fine and then raises
    SIGBUS on the first page past it. Refuse to start instead, naming the sizes (the region
    grows with --max-nodes and --max-pods: Ledger::region_bytes)."""
    from .native import core

    need = int(core().Ledger.region_bytes(max_nodes, max_pods))
    d = os.path.dirname(os.path.abspath(path)) or "/"
    try:
        st = os.statvfs(d)
    except OSError:
        return
    free = st.f_bavail * st.f_frsize
    if os.path.exists(path):
        free += os.path.getsize(path)   # a stale region of ours is replaced
    if need > free:
        raise SystemExit(f"nano-gpu: the shared ledger needs {need >> 20} MiB (--max-nodes {max_nodes}, "
                         f"--max-pods {max_pods}) but {d} has {free >> 20} MiB free: raise the /dev/shm "
                         f"emptyDir sizeLimit or lower the flags")


def run(cfg: Config) -> int:
    guard_busy_poll(cfg)
    if cfg.ledger_path or cfg.workers > 1:
        check_region_space(cfg.ledger_path or "/dev/shm/nanogpu-ledger", cfg.max_nodes, cfg.max_pods)
    if cfg.workers <= 1:
        if cfg.ledger_path:
            _drop_stale_region(cfg.ledger_path)
        pin_worker(cfg, 0)
        return asyncio.run(serve_forever(cfg, 0))
    if not cfg.ledger_path:
        cfg.ledger_path = f"/dev/shm/nanogpu-ledger-{os.getpid()}"
    _drop_stale_region(cfg.ledger_path)
    # create the shared region before forking so every worker attaches to the same layout
    from .native import core

    led = core().Ledger(cfg.ledger_path, cfg.max_nodes, cfg.max_pods, True)
    if cfg.leader_elect:
        led.serving = False          # no worker schedules before the Lease is won
    del led
    children = []
    for w in range(cfg.workers):
        pid = os.fork()
        if pid == 0:
            try:
                pin_worker(cfg, w)
                code = asyncio.run(serve_forever(cfg, w))
            except BaseException:
                log.exception("worker %d crashed", w)
                code = 1
            os._exit(code)
        children.append(pid)

    def forward(sig, _frame):
        for c in children:
            try:
                os.kill(c, sig)
            except ProcessLookupError:
                pass

    stopping = {"on": False}

    def forward_and_stop(sig, frame):
        stopping["on"] = True
        forward(sig, frame)

    signal.signal(signal.SIGINT, forward_and_stop)
    signal.signal(signal.SIGTERM, forward_and_stop)
    code = supervise(children, stopping)
    try:
        os.unlink(cfg.ledger_path)
    except OSError:
        pass
    return code


def supervise(children: list[int], stopping: dict, grace_s: float = 10.0) -> int:
    """Waits for the workers. A worker that exits while the replica is not shutting down
    (a crash, an OOM kill) takes the replica down: the others are stopped and the exit code
    is non-zero, so the kubelet restarts the pod as a whole — worker 0 runs the pod
    controller, sweeper and leader elector, and half a replica must not keep serving."""
    live = set(children)
    code = 0
    while live:
        try:
            pid, status = os.wait()
        except ChildProcessError:
            break
        except InterruptedError:
            continue
        if pid not in live:
            continue
        live.discard(pid)
        rc = os.waitstatus_to_exitcode(status)
        code = code or rc
        if not stopping["on"] and live:
            log.error("worker pid %d exited (%d): stopping the replica", pid, rc)
            code = code or 1
            stopping["on"] = True
            for c in live:
                try:
                    os.kill(c, signal.SIGTERM)
                except ProcessLookupError:
                    pass
            deadline = time.monotonic() + grace_s
            while live and time.monotonic() < deadline:
                for c in list(live):
                    done, st = os.waitpid(c, os.WNOHANG)
                    if done:
                        live.discard(c)
                time.sleep(0.05)
            for c in live:
                try:
                    os.kill(c, signal.SIGKILL)
                except ProcessLookupError:
                    pass
    return code


def main(argv: list[str] | None = None) -> int:
    from .cli import parse

    cfg = parse(argv)
    return run(cfg)


if __name__ == "__main__":
    sys.exit(main())
