"""A kube-scheduler stand-in that speaks the extender protocol.

Models what kube-scheduler does with an extender configured as in the reference README
(README.md:43-58: urlPrefix .../scheduler, filter/priorities/bind verbs,
nodeCacheCapable=true, managed resource nano-gpu/gpu-percent) [ext]:
  * scheduling cycle, serial per scheduler instance: node-level resource fit
    (NodeResourcesFit on the extended resource) -> POST filter -> POST priorities ->
    select the max-score host (ties broken by a seeded RNG, like selectHost) [ext];
  * binding cycle, asynchronous: POST bind (the extender is the binder);
  * failed pods go back to the queue with exponential backoff.
Transport is real HTTP (aiohttp) or in-process calls on an `Extender`.
"""
from __future__ import annotations

import asyncio
import json
import random
import time
import zlib
from dataclasses import dataclass, field

import aiohttp

from .. import types as T
from ..k8s import podutil as pu
from .kubescore import KubeScoring


class HttpExtenderClient:
    def __init__(self, base_url: str, pool: int = 256):
        self.base = base_url.rstrip("/")
        self.pool = pool
        self.s: aiohttp.ClientSession | None = None

    async def _session(self) -> aiohttp.ClientSession:
        if self.s is None:
            self.s = aiohttp.ClientSession(connector=aiohttp.TCPConnector(limit=self.pool),
                                           timeout=aiohttp.ClientTimeout(total=30))
        return self.s

    async def _post(self, verb: str, body: dict):
        s = await self._session()
        async with s.post(f"{self.base}/scheduler/{verb}", data=json.dumps(body, separators=(",", ":")),
                          headers={"Content-Type": "application/json"}) as r:
            return r.status, await r.json(content_type=None)

    async def filter(self, body):
        return (await self._post("filter", body))[1]

    async def prioritize(self, body):
        return (await self._post("priorities", body))[1]

    async def bind(self, body):
        return (await self._post("bind", body))[1]

    async def close(self):
        if self.s is not None:
            await self.s.close()


class _HttpConn(asyncio.Protocol):
    """One keep-alive HTTP/1.1 connection; responses resolve request futures in order."""

    def __init__(self):
        self.transport = None
        self.buf = bytearray()
        self.waiters: list[asyncio.Future] = []
        self.closed = False

    def connection_made(self, transport):
        self.transport = transport

    def connection_lost(self, exc):
        self.closed = True
        for w in self.waiters:
            if not w.done():
                w.set_exception(ConnectionError("connection lost"))
        self.waiters.clear()

    def data_received(self, data):
        self.buf += data
        while self.waiters:
            he = self.buf.find(b"\r\n\r\n")
            if he < 0:
                return
            head = bytes(self.buf[:he])
            clen = 0
            for line in head.split(b"\r\n")[1:]:
                k, _, v = line.partition(b":")
                if k.strip().lower() == b"content-length":
                    clen = int(v)
            if len(self.buf) < he + 4 + clen:
                return
            status = int(head[9:12])
            body = bytes(self.buf[he + 4:he + 4 + clen])
            del self.buf[:he + 4 + clen]
            w = self.waiters.pop(0)
            if not w.done():
                w.set_result((status, body))


class FastExtenderClient:
    """Lean keep-alive client (asyncio.Protocol, no aiohttp) for driving an extender at
    full speed: kube-scheduler's Go client costs microseconds per request, so the
    stand-in should not be the bottleneck of an extender benchmark."""

    def __init__(self, host: str, port: int, pool: int = 256):
        self.host, self.port = host, port
        self.pool = pool
        self.idle: list[_HttpConn] = []
        self.all: list[_HttpConn] = []
        self._enc = json.JSONEncoder(separators=(",", ":"))
        self._pod_json: dict[str, bytes] = {}
        self._names_json: dict[int, tuple] = {}

    async def _conn(self) -> _HttpConn:
        while self.idle:
            c = self.idle.pop()
            if not c.closed:
                return c
        loop = asyncio.get_running_loop()
        _, c = await loop.create_connection(_HttpConn, self.host, self.port)
        self.all.append(c)
        return c

    async def post(self, path: str, body: bytes) -> tuple[int, bytes]:
        c = await self._conn()
        fut = asyncio.get_running_loop().create_future()
        c.waiters.append(fut)
        c.transport.write(b"POST " + path.encode() + b" HTTP/1.1\r\nHost: extender\r\n"
                          b"Content-Type: application/json\r\nContent-Length: " + str(len(body)).encode() +
                          b"\r\n\r\n" + body)
        try:
            return await fut
        finally:
            if not c.closed:
                self.idle.append(c)

    def _args(self, body: dict) -> bytes:
        pod = body.get("Pod")
        uid = pu.pod_uid(pod) if pod else ""
        pj = self._pod_json.get(uid) if uid else None
        if pj is None:
            pj = self._enc.encode(pod).encode()
            if uid:
                if len(self._pod_json) > 65536:
                    self._pod_json.clear()
                self._pod_json[uid] = pj
        names = body.get("NodeNames")
        if names is not None and body.get("Nodes") is None and len(body) <= 3:
            key = id(names)
            hit = self._names_json.get(key)
            if hit is None or hit[0] is not names:
                hit = (names, self._enc.encode(names).encode())
                if len(self._names_json) > 64:
                    self._names_json.clear()
                self._names_json[key] = hit
            return b'{"Pod":' + pj + b',"Nodes":null,"NodeNames":' + hit[1] + b"}"
        rest = {k: v for k, v in body.items() if k != "Pod"}
        return b'{"Pod":' + pj + b"," + self._enc.encode(rest).encode()[1:]

    async def filter(self, body):
        return json.loads((await self.post("/scheduler/filter", self._args(body)))[1])

    async def prioritize(self, body):
        return json.loads((await self.post("/scheduler/priorities", self._args(body)))[1])

    async def bind(self, body):
        return json.loads((await self.post("/scheduler/bind", self._enc.encode(body).encode()))[1])

    async def close(self):
        for c in self.all:
            if c.transport is not None:
                c.transport.close()


class InProcExtenderClient:
    def __init__(self, ext):
        self.ext = ext

    async def filter(self, body):
        return self.ext.filter(body)

    async def prioritize(self, body):
        return self.ext.prioritize(body)

    async def bind(self, body):
        return await self.ext.bind(body)

    async def close(self):
        return None


@dataclass
class PodRecord:
    pod: dict
    t_enqueue: float = 0.0
    t_first_attempt: float = 0.0
    t_bound: float = 0.0
    bind_latency: float = 0.0
    node: str = ""
    attempts: int = 0
    error: str = ""


@dataclass
class DriverStats:
    scheduled: int = 0
    failed: int = 0
    unschedulable_attempts: int = 0
    bind_errors: int = 0
    bind_latencies: list = field(default_factory=list)
    e2e_latencies: list = field(default_factory=list)
    t_first_filter: float = 0.0
    t_last_bind: float = 0.0
    cycle_max_s: float = 0.0
    cycle_sum_s: float = 0.0
    cycle_wire_s: float = 0.0
    nodes_sent_filter: int = 0     # node names sent to the extender's filter, summed over cycles
    cycles: int = 0

    def summary(self) -> dict:
        span = max(1e-9, self.t_last_bind - self.t_first_filter)
        bl = sorted(self.bind_latencies)
        e2e = sorted(self.e2e_latencies)

        def pct(a, q):
            return a[min(len(a) - 1, int(q * len(a)))] if a else 0.0

        def median(a):   # of a sorted list
            n = len(a)
            return 0.0 if not n else (a[n // 2] if n % 2 else 0.5 * (a[n // 2 - 1] + a[n // 2]))

        return {"scheduled": self.scheduled, "failed": self.failed, "bind_errors": self.bind_errors,
                "unschedulable_attempts": self.unschedulable_attempts,
                "pods_per_s": self.scheduled / span if self.scheduled else 0.0, "span_s": span,
                "bind_p50_ms": 1e3 * median(bl),
                "bind_p99_ms": 1e3 * pct(bl, 0.99),
                "bind_max_ms": 1e3 * (bl[-1] if bl else 0.0),
                "cycle_max_ms": 1e3 * self.cycle_max_s,
                "cycle_sum_ms": 1e3 * self.cycle_sum_s,
                "cycle_wire_ms": 1e3 * self.cycle_wire_s,
                "nodes_sent_filter": self.nodes_sent_filter, "cycles": self.cycles,
                "e2e_p50_ms": 1e3 * median(e2e),
                # the burst's window on the monotonic clock (comparable across processes of a node)
                "t_first_filter": self.t_first_filter, "t_last_bind": self.t_last_bind,
                # every POST /scheduler/bind as the scheduler saw it (request written -> reply
                # read), in seconds, unrounded
                "bind_s_all": self.bind_latencies}


class SchedulerDriver:
    def __init__(self, client, api, node_names: list[str], node_capacity: dict[str, int] | None = None,
                 max_inflight_binds: int = 64, seed: int = 0, max_attempts: int = 8,
                 backoff_s: float = 0.001, resource_fit: bool = True, send_nodes: bool = False,
                 node_objects: dict[str, dict] | None = None, kube: KubeScoring | None = None):
        self.client = client
        # kube-scheduler score combining (nanogpu/sim/kubescore.py); None: extender arg-max
        self.kube = kube
        self.used: dict[str, tuple[int, int]] = {n: (0, 0) for n in node_names}
        self.api = api
        self.nodes = list(node_names)
        self.node_objects = node_objects or {}
        self.send_nodes = send_nodes
        self.capacity = dict(node_capacity or {})
        self.requested: dict[str, int] = {n: 0 for n in self.nodes}
        self.resource_fit = resource_fit and bool(self.capacity)
        self.rng = random.Random(seed)
        self.sem = asyncio.Semaphore(max_inflight_binds)
        self.max_attempts = max_attempts
        self.backoff_s = backoff_s
        self.stats = DriverStats()
        self._binds: set[asyncio.Task] = set()
        self.placements: dict[str, str] = {}

    def _select(self, prios: list[dict], pod: dict) -> str:
        """selectHost [ext]: uniform among the max-total hosts; the total is the extender's
        score alone, or kube-scheduler's plugin + weighted extender sum (self.kube)."""
        if self.kube is None:
            totals = [hp["Score"] for hp in prios]
        else:
            req = self.kube.pod_requests(pu.pod_demand(pod))
            totals = [self.kube.total(hp["Score"], self.used.get(hp["Host"], (0, 0)), req) for hp in prios]
        best = max(totals)
        ties = [hp["Host"] for hp, t in zip(prios, totals) if t == best]
        return ties[0] if len(ties) == 1 else ties[self.rng.randrange(len(ties))]

    def _use(self, host: str, pod: dict, sign: int) -> None:
        if self.kube is not None:
            c, m = self.kube.pod_requests(pu.pod_demand(pod))
            u = self.used.get(host, (0, 0))
            self.used[host] = (u[0] + sign * c, u[1] + sign * m)

    def _candidates(self, need: int) -> list[str]:
        if not self.resource_fit:
            return self.nodes
        req, cap = self.requested, self.capacity
        out = [n for n in self.nodes if req.get(n, 0) + need <= cap.get(n, 0)]
        return self.nodes if len(out) == len(self.nodes) else out   # same object: encodings cached

    async def schedule_one(self, rec: PodRecord) -> bool:
        """One scheduling cycle. Returns True when a bind was issued."""
        pod = rec.pod
        need = sum(p for p, _ in pu.pod_demand(pod))
        cands = self._candidates(need)
        rec.attempts += 1
        if not rec.t_first_attempt:
            rec.t_first_attempt = time.perf_counter()
            if not self.stats.t_first_filter:
                self.stats.t_first_filter = rec.t_first_attempt
        if not cands:
            self.stats.unschedulable_attempts += 1
            return False
        if self.send_nodes:
            args = {"Pod": pod, "Nodes": {"items": [self.node_objects[n] for n in cands]}, "NodeNames": None}
        else:
            args = {"Pod": pod, "Nodes": None, "NodeNames": cands}
        fr = await self.client.filter(args)
        if fr.get("Error"):
            rec.error = fr["Error"]
            return False
        fit = fr.get("NodeNames")
        if fit is None and fr.get("Nodes"):
            fit = [pu.meta(n).get("name") for n in fr["Nodes"].get("items", [])]
        if not fit:
            self.stats.unschedulable_attempts += 1
            return False
        if len(fit) == len(cands):
            fit = cands            # all passed, same order: reuse the cached NodeNames encoding
        if len(fit) == 1:
            host = fit[0]
        else:
            args2 = {"Pod": pod, "Nodes": None, "NodeNames": fit}
            prios = await self.client.prioritize(args2)
            host = self._select(prios, pod)
        # kube-scheduler "assumes" the pod in its cache before binding asynchronously
        self.requested[host] = self.requested.get(host, 0) + need
        self._use(host, pod, +1)
        await self.sem.acquire()
        t = asyncio.ensure_future(self._bind(rec, host, need))
        self._binds.add(t)
        t.add_done_callback(self._binds.discard)
        return True

    async def _bind(self, rec: PodRecord, host: str, need: int) -> None:
        ns, name = pu.pod_ns_name(rec.pod)
        t0 = time.perf_counter()
        try:
            res = await self.client.bind({"PodName": name, "PodNamespace": ns, "PodUID": pu.pod_uid(rec.pod),
                                          "Node": host})
        finally:
            self.sem.release()
        t1 = time.perf_counter()
        if res.get("Error"):
            self.requested[host] -= need
            self.stats.bind_errors += 1
            rec.error = res["Error"]
            if rec.attempts < self.max_attempts:
                await asyncio.sleep(self.backoff_s * (2 ** rec.attempts))
                await self._queue.put(rec)
            else:
                self.stats.failed += 1
                self._done.release()
            return
        rec.t_bound = t1
        rec.bind_latency = t1 - t0
        rec.node = host
        self.placements[pu.pod_uid(rec.pod)] = host
        self.stats.scheduled += 1
        self.stats.bind_latencies.append(rec.bind_latency)
        self.stats.e2e_latencies.append(t1 - rec.t_enqueue)
        self.stats.t_last_bind = max(self.stats.t_last_bind, t1)
        self._done.release()

    def release(self, pod: dict) -> None:
        """Scheduler cache update when a bound pod goes away."""
        host = self.placements.pop(pu.pod_uid(pod), None)
        if host:
            self.requested[host] -= sum(p for p, _ in pu.pod_demand(pod))
            self._use(host, pod, -1)

    async def run(self, pods: list[dict], create: bool = True) -> DriverStats:
        """Creates `pods` through the API (if `create`) and schedules all of them."""
        self._queue: asyncio.Queue[PodRecord] = asyncio.Queue()
        self._done = asyncio.Semaphore(0)
        now = time.perf_counter()
        for p in pods:
            if create:
                await self.api.create_pod(p)
            await self._queue.put(PodRecord(p, t_enqueue=now))
        remaining = len(pods)

        async def loop():
            while True:
                rec = await self._queue.get()
                ok = False
                try:
                    ok = await self.schedule_one(rec)
                except (aiohttp.ClientError, asyncio.TimeoutError, ConnectionError) as e:
                    rec.error = str(e)
                if not ok:
                    if rec.attempts < self.max_attempts:
                        asyncio.get_running_loop().call_later(self.backoff_s * (2 ** rec.attempts),
                                                              self._queue.put_nowait, rec)
                    else:
                        self.stats.failed += 1
                        self._done.release()

        task = asyncio.ensure_future(loop())
        try:
            for _ in range(remaining):
                await self._done.acquire()
        finally:
            task.cancel()
            try:
                await task
            except asyncio.CancelledError:
                pass
        return self.stats


def node_capacities(nodes: list[dict]) -> dict[str, int]:
    return {pu.meta(n)["name"]: pu.node_capacity_percent(n) for n in nodes}


__all__ = ["SchedulerDriver", "HttpExtenderClient", "FastExtenderClient", "InProcExtenderClient", "node_capacities", "T"]


# ----------------------------------------------------------------------------- threaded driver
class BlockingHttp:
    """One blocking keep-alive HTTP/1.1 connection (the scheduling cycle is serial)."""

    def __init__(self, host: str, port: int):
        import socket

        self.sock = socket.create_connection((host, port))
        self.sock.setsockopt(socket.IPPROTO_TCP, socket.TCP_NODELAY, 1)
        self.buf = b""

    def post(self, path: bytes, body: bytes) -> tuple[int, bytes]:
        self.sock.sendall(b"POST " + path + b" HTTP/1.1\r\nHost: extender\r\nContent-Type: application/json\r\n"
                          b"Content-Length: " + str(len(body)).encode() + b"\r\n\r\n" + body)
        buf = self.buf
        while True:
            he = buf.find(b"\r\n\r\n")
            if he >= 0:
                head = buf[:he]
                i = head.lower().find(b"content-length:")
                clen = int(head[i + 15:head.find(b"\r\n", i) if head.find(b"\r\n", i) > 0 else len(head)])
                end = he + 4 + clen
                if len(buf) >= end:
                    self.buf = buf[end:]
                    return int(head[9:12]), buf[he + 4:end]
            chunk = self.sock.recv(262144)
            if not chunk:
                raise ConnectionError("extender closed the connection")
            buf += chunk

    def close(self) -> None:
        self.sock.close()


class ThreadedSchedulerDriver:
    """kube-scheduler stand-in without an event loop: the scheduling cycle (filter ->
    priorities -> select host) runs serially on one blocking connection, binds run
    concurrently on a thread pool with one connection per thread (kube-scheduler's
    binding goroutines). Same semantics as SchedulerDriver; lower per-cycle latency."""

    def __init__(self, host: str, port: int, node_names: list[str], node_capacity: dict[str, int] | None = None,
                 bind_threads: int = 16, seed: int = 0, max_attempts: int = 8, backoff_s: float = 0.001):
        import threading

        self.host, self.port = host, port
        self.nodes = list(node_names)
        self.capacity = dict(node_capacity or {})
        self.requested: dict[str, int] = {n: 0 for n in self.nodes}
        self.resource_fit = bool(self.capacity)
        self.rng = random.Random(seed)
        self.max_attempts = max_attempts
        self.backoff_s = backoff_s
        self.bind_threads = bind_threads
        self.stats = DriverStats()
        self.lock = threading.Lock()
        self.cv = threading.Condition(self.lock)
        self._enc = json.JSONEncoder(separators=(",", ":"))
        self._names = self._enc.encode(self.nodes).encode()
        self._local = threading.local()
        self.cycle = BlockingHttp(host, port)

    def _conn(self) -> BlockingHttp:
        c = getattr(self._local, "c", None)
        if c is None:
            c = self._local.c = BlockingHttp(self.host, self.port)
        return c

    def _candidates(self, need: int) -> tuple[list[str], bytes]:
        if not self.resource_fit:
            return self.nodes, self._names
        with self.lock:
            out = [n for n in self.nodes if self.requested.get(n, 0) + need <= self.capacity.get(n, 0)]
        if len(out) == len(self.nodes):
            return self.nodes, self._names
        return out, self._enc.encode(out).encode()

    def run(self, pods: list[dict]) -> DriverStats:
        import heapq
        from concurrent.futures import ThreadPoolExecutor

        now = time.perf_counter()
        recs = [PodRecord(p, t_enqueue=now) for p in pods]
        pod_json = {id(r): self._enc.encode(r.pod).encode() for r in recs}
        ready: list[tuple[float, int, PodRecord]] = [(0.0, i, r) for i, r in enumerate(recs)]
        seq = len(recs)
        remaining = len(recs)
        st = self.stats

        def requeue(rec: PodRecord) -> None:
            nonlocal seq, remaining
            if rec.attempts < self.max_attempts:
                heapq.heappush(ready, (time.perf_counter() + self.backoff_s * (2 ** rec.attempts), seq, rec))
                seq += 1
            else:
                st.failed += 1
                remaining -= 1
            self.cv.notify_all()

        def bind(rec: PodRecord, host: str, need: int) -> None:
            nonlocal remaining
            ns, name = pu.pod_ns_name(rec.pod)
            body = self._enc.encode({"PodName": name, "PodNamespace": ns, "PodUID": pu.pod_uid(rec.pod),
                                     "Node": host}).encode()
            t0 = time.perf_counter()
            try:
                _, out = self._conn().post(b"/scheduler/bind", body)
                err = json.loads(out).get("Error")
            except (OSError, ValueError) as e:
                err = str(e) or "bind failed"
            t1 = time.perf_counter()
            with self.lock:
                if err:
                    self.requested[host] -= need
                    st.bind_errors += 1
                    rec.error = err
                    requeue(rec)
                    return
                rec.t_bound, rec.bind_latency, rec.node = t1, t1 - t0, host
                st.scheduled += 1
                st.bind_latencies.append(t1 - t0)
                st.e2e_latencies.append(t1 - rec.t_enqueue)
                st.t_last_bind = max(st.t_last_bind, t1)
                remaining -= 1
                self.cv.notify_all()

        with ThreadPoolExecutor(self.bind_threads) as pool:
            while True:
                with self.lock:
                    while remaining > 0 and (not ready or ready[0][0] > time.perf_counter()):
                        self.cv.wait(max(0.0, ready[0][0] - time.perf_counter()) if ready else 0.05)
                    if remaining == 0:
                        break
                    _, _, rec = heapq.heappop(ready)
                rec.attempts += 1
                if not st.t_first_filter:
                    st.t_first_filter = time.perf_counter()
                need = sum(p for p, _ in pu.pod_demand(rec.pod))
                cands, cands_json = self._candidates(need)
                host = None
                if cands:
                    head = b'{"Pod":' + pod_json[id(rec)] + b',"Nodes":null,"NodeNames":'
                    _, out = self.cycle.post(b"/scheduler/filter", head + cands_json + b"}")
                    fit = json.loads(out).get("NodeNames") or []
                    if len(fit) == 1:
                        host = fit[0]
                    elif fit:
                        fj = cands_json if len(fit) == len(cands) else self._enc.encode(fit).encode()
                        _, out = self.cycle.post(b"/scheduler/priorities", head + fj + b"}")
                        prios = json.loads(out)
                        best = max(hp["Score"] for hp in prios)
                        ties = [hp["Host"] for hp in prios if hp["Score"] == best]
                        host = ties[0] if len(ties) == 1 else ties[self.rng.randrange(len(ties))]
                if host is None:
                    with self.lock:
                        st.unschedulable_attempts += 1
                        requeue(rec)
                    continue
                with self.lock:
                    self.requested[host] = self.requested.get(host, 0) + need
                pool.submit(bind, rec, host, need)
        return st

    def close(self) -> None:
        self.cycle.close()


def owner_index(pod: dict) -> int:
    """The pod's controlling owner as the stand-in's int id (PodTopologySpread's selector),
    -1 for none. kube-scheduler only applies its system default spread constraints to pods a
    ReplicaSet / StatefulSet / ReplicationController / Service selects."""
    refs = [r for r in (pu.meta(pod).get("ownerReferences") or []) if isinstance(r, dict)]
    ctl = next((r for r in refs if r.get("controller") is True), None)
    if ctl is None or ctl.get("kind") not in ("ReplicaSet", "StatefulSet", "ReplicationController"):
        return -1
    return zlib.crc32(str(ctl.get("uid", "")).encode()) & 0x7FFFFFFF


class NativeSchedulerDriver:
    """ThreadedSchedulerDriver's protocol loop in C++ (native/src/schedsim.cpp): the same
    serial filter -> priorities -> select-host cycle and asynchronous bind pool, without
    the interpreter's ~150 us per pod, so the measured rate is the extender's, not the
    stand-in's. kube-scheduler itself is compiled Go, so this is the closer model of it.
    Tie-breaks draw from a different random stream than the Python drivers."""

    def __init__(self, host: str, port: int, node_names: list[str], node_capacity: dict[str, int] | None = None,
                 bind_threads: int = 256, seed: int = 0, max_attempts: int = 8, backoff_s: float = 0.001,
                 session=None, kube: KubeScoring | None = None, bind_ports: list[int] | None = None):
        self.host, self.port = host, port
        self.bind_ports = list(bind_ports or [])   # several extender workers behind one Service
        self.kube = kube     # combining in C++ (same model as nanogpu/sim/kubescore.py)
        self.session = session      # core().SchedulerSession(): keep-alive connections across runs
        self.nodes = list(node_names)
        self.capacity = [int(node_capacity.get(n, 0)) for n in self.nodes] if node_capacity else []
        self.bind_threads = bind_threads
        self.seed = seed
        self.max_attempts = max_attempts
        self.backoff_s = backoff_s
        self.stats = DriverStats()
        self._placed: list = []    # (pod tuples, node per pod) of each run

    @property
    def placements(self) -> dict[str, str]:
        """ns/name -> node of every pod these runs scheduled (built when asked for)."""
        return {f"{ns}/{name}": node for args, nodes in self._placed
                for (_, ns, name, *_), node in zip(args, nodes) if node}

    @staticmethod
    def prepare_native(pods: list[dict], kube: KubeScoring | None = None):
        """`prepare`, then converted to the native loop's own pod records once
        (core().SimBurst): a run takes them without per-run conversion."""
        from ..native import core

        args = NativeSchedulerDriver.prepare(pods, kube)
        return args, core().SimBurst(args)

    @staticmethod
    def prepare(pods: list[dict], kube: KubeScoring | None = None) -> list[tuple]:
        """The pods as the native loop takes them (kube-scheduler has them decoded from its
        informer before a scheduling cycle starts; this is harness-side work), with the
        CPU / memory requests kube-scheduler's own score plugins see."""
        enc = json.JSONEncoder(separators=(",", ":"))
        ks = kube or KubeScoring()
        args = []
        for p in pods:
            ns, name = pu.pod_ns_name(p)
            d = pu.pod_demand(p)
            cpu, mem = ks.pod_requests(d)
            args.append((enc.encode(p).encode(), ns, name, pu.pod_uid(p), sum(c for c, _ in d), cpu, mem,
                         owner_index(p)))
        return args

    def run(self, pods: list[dict] | None = None, prepared: list[tuple] | None = None,
            live: list[tuple] | None = None) -> DriverStats:
        """`live`: pods bound before this run, (node index, need, cpu_m, mem, owner) each, as
        kube-scheduler's cache holds them (steady-state churn)."""
        from ..native import core

        args = prepared if prepared is not None else self.prepare(pods or [])
        native = None
        if isinstance(args, tuple):   # prepare_native: (pod tuples, SimBurst)
            args, native = args
        k = self.kube
        r = core().drive_scheduler(self.host, self.port, native if native is not None else args,
                                   self.nodes, self.capacity, self.bind_threads,
                                   self.seed, self.max_attempts, self.backoff_s, self.session,
                                   kube_combine=int(k is not None),
                                   extender_weight=k.extender_weight if k else 1,
                                   sample_nodes=int(k.sample_nodes) if k else 1,
                                   percentage_of_nodes_to_score=k.percentage_of_nodes_to_score if k else 0,
                                   spread_weight=k.spread_weight if k else 0,
                                   live=live or [], bind_ports=self.bind_ports)
        self.stats.nodes_sent_filter = r["nodes_sent_filter"]
        self.stats.cycles = r["cycles"]
        st = self.stats
        st.scheduled, st.failed = r["scheduled"], r["failed"]
        st.bind_errors, st.unschedulable_attempts = r["bind_errors"], r["unschedulable_attempts"]
        st.bind_latencies, st.e2e_latencies = r["bind_latencies"], r["e2e_latencies"]
        st.t_first_filter, st.t_last_bind = r["t_first_filter"], r["t_last_bind"]
        st.cycle_max_s = r.get("cycle_max_s", 0.0)
        st.cycle_sum_s = r.get("cycle_sum_s", 0.0)
        st.cycle_wire_s = r.get("cycle_wire_s", 0.0)
        self._placed.append((args, r["node_of"]))
        return st

    def close(self) -> None:
        pass

