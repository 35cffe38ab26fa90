"""`--workers N`: SO_REUSEPORT extender processes sharing one /dev/shm ledger.

The fake API server runs over HTTP in the test process; `python -m nanogpu --workers 2`
serves on one port from two forked workers (native front doors, shared ledger). Many
concurrent clients hit both workers; binds on either worker debit the same devices, so
the cluster never over-commits and /status agrees from every connection."""
import asyncio
import json
import os
import signal
import socket
import subprocess
import sys
import time
from pathlib import Path

import pytest

from nanogpu.k8s import podutil as pu
from nanogpu.k8s.fake_apiserver import FakeKubeStore, serve
from nanogpu.sim.driver import FastExtenderClient, SchedulerDriver, node_capacities
from nanogpu.topology.model import synthetic_mi355x

ROOT = Path(__file__).resolve().parent.parent


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.mark.parametrize("decisive", [False, True])
def test_two_workers_share_one_ledger(decisive):
    """(decisive: --decisive-filter, filter answers one node and kube-scheduler binds it at
    once; with two workers the filter publishes its pod before answering, so a bind on the
    other worker finds it)"""
    async def main():
        store = FakeKubeStore()
        nodes = [pu.make_node(f"n{i}", 2, synthetic_mi355x(2).to_json()) for i in range(3)]
        for n in nodes:
            store.add_node(n)
        runner, api_port = await serve(store)
        port = _free_port()
        ledger = f"/dev/shm/nanogpu-test-workers-{os.getpid()}"
        proc = subprocess.Popen([sys.executable, "-m", "nanogpu", "--kube-api", f"http://127.0.0.1:{api_port}",
                                 "--workers", "2", "--host", "127.0.0.1", "--ledger-path", ledger,
                                 "--policyConfigPath", "/nonexistent"] + (["--decisive-filter"] if decisive else []),
                                env=dict(os.environ, PORT=str(port)), cwd=str(ROOT),
                                stdout=subprocess.PIPE, stderr=subprocess.STDOUT, start_new_session=True)
        try:
            loop = asyncio.get_running_loop()
            deadline = time.time() + 60
            while True:
                try:
                    r, w = await asyncio.open_connection("127.0.0.1", port)
                    w.close()
                    break
                except OSError:
                    assert time.time() < deadline and proc.poll() is None
                    await asyncio.sleep(0.2)
            await asyncio.sleep(1.0)     # both workers listening
            pods = [pu.make_pod(f"p{i}", [("c", 30)]) for i in range(40)]
            clients = [FastExtenderClient("127.0.0.1", port, pool=8) for _ in range(4)]
            from nanogpu.k8s.fake_apiserver import InProcKube

            drivers = [SchedulerDriver(c, InProcKube(store), [pu.meta(n)["name"] for n in nodes],
                                       node_capacities(nodes), seed=k, max_attempts=4, resource_fit=False)
                       for k, c in enumerate(clients)]
            stats = await asyncio.gather(*[d.run(pods[k::4]) for k, d in enumerate(drivers)])
            bound = sum(s.scheduled for s in stats)
            # 3 nodes x 2 devices x 3 shares of 30 % = 18 pods fit
            assert bound == 18, [s.summary() for s in stats]
            used = {}
            for p in store.pods.values():
                if pu.node_name_of(p):
                    k = (pu.node_name_of(p), pu.container_assignment(p, "c")[0])
                    used[k] = used.get(k, 0) + 30
            assert max(used.values()) <= 100
            for c in clients:
                await c.close()
            # every connection sees the same shared ledger
            views = set()
            for _ in range(6):
                r, w = await asyncio.open_connection("127.0.0.1", port)
                w.write(b"GET /status HTTP/1.1\r\nHost: x\r\nConnection: close\r\n\r\n")
                data = await r.read()
                w.close()
                body = json.loads(data.split(b"\r\n\r\n", 1)[1])
                views.add(json.dumps({n: [g["Percent"] for g in v["GPUs"]] for n, v in body.items()}, sort_keys=True))
            assert len(views) == 1
            free = json.loads(views.pop())
            assert sum(100 - x for v in free.values() for x in v) == 30 * bound
            # with two workers on the ledger, every filter publishes its pod for a bind that
            # lands on the other worker (the shared-ledger handoff)
            published = 0
            for _ in range(8):
                r, w = await asyncio.open_connection("127.0.0.1", port)
                w.write(b"GET /metrics HTTP/1.1\r\nHost: x\r\nConnection: close\r\n\r\n")
                text = (await r.read()).decode()
                w.close()
                for line in text.splitlines():
                    if line.startswith("nanogpu_native_pods_published_total "):
                        published = max(published, float(line.split()[1]))
            assert published > 0
        finally:
            os.killpg(proc.pid, signal.SIGTERM)
            try:
                proc.wait(timeout=15)
            except subprocess.TimeoutExpired:
                os.killpg(proc.pid, signal.SIGKILL)
            await runner.cleanup()
            try:
                os.unlink(ledger)
            except FileNotFoundError:
                pass

    asyncio.run(main())


def test_ledger_refuses_a_short_or_foreign_region(tmp_path):
    """Attaching to a /dev/shm file of another geometry, another layout version, or one whose
    creator died before sizing it must fail cleanly (not SIGBUS past the end of the file)."""
    import pytest

    from nanogpu import _native as N

    short = f"/dev/shm/nanogpu-test-short-{os.getpid()}"
    other = f"/dev/shm/nanogpu-test-other-{os.getpid()}"
    try:
        open(short, "wb").close()                       # creator died before ftruncate
        with pytest.raises(RuntimeError, match="smaller"):
            N.Ledger(short, 16, 64, False)
        a = N.Ledger(other, 16, 64, True)               # live region, other geometry
        with pytest.raises(RuntimeError):
            N.Ledger(other, 32, 64, False)
        b = N.Ledger(other, 16, 64, False)              # same geometry attaches
        del a, b
    finally:
        for p in (short, other):
            if os.path.exists(p):
                os.unlink(p)


def _die_with_parent():
    """The replica runs in a session of its own (the test signals its whole group); if the test
    process is killed before its `finally` (an interrupted `pytest -x -n`), the replica gets
    SIGTERM instead of living on as an orphan."""
    import ctypes

    ctypes.CDLL(None, use_errno=True).prctl(1, signal.SIGTERM)   # PR_SET_PDEATHSIG


async def _start_replica(api_port, port, ledger, *extra):
    proc = subprocess.Popen([sys.executable, "-m", "nanogpu", "--kube-api", f"http://127.0.0.1:{api_port}",
                             "--workers", "2", "--host", "127.0.0.1", "--ledger-path", ledger,
                             "--policyConfigPath", "/nonexistent", *extra],
                            env=dict(os.environ, PORT=str(port)), cwd=str(ROOT),
                            stdout=subprocess.PIPE, stderr=subprocess.STDOUT, start_new_session=True,
                            preexec_fn=_die_with_parent)
    deadline = time.time() + 60
    while True:
        try:
            r, w = await asyncio.open_connection("127.0.0.1", port)
            w.close()
            break
        except OSError:
            assert time.time() < deadline and proc.poll() is None
            await asyncio.sleep(0.2)
    await asyncio.sleep(1.0)     # both workers listening
    return proc


def _stop(proc):
    try:
        os.killpg(proc.pid, signal.SIGTERM)
    except ProcessLookupError:
        return
    try:
        proc.wait(timeout=15)
    except subprocess.TimeoutExpired:
        os.killpg(proc.pid, signal.SIGKILL)


async def _statuses(port, method, path, body=b"", n=16):
    """`n` fresh connections (SO_REUSEPORT spreads them over the workers)."""
    out = []
    for _ in range(n):
        r, w = await asyncio.open_connection("127.0.0.1", port)
        w.write(f"{method} {path} HTTP/1.1\r\nHost: x\r\nConnection: close\r\nContent-Length: {len(body)}\r\n\r\n"
                .encode() + body)
        data = await r.read()
        w.close()
        out.append(int(data.split(b" ", 2)[1]))
    return out


def test_standby_replica_answers_503_on_every_worker_until_it_wins_the_lease():
    """with --workers 2 --leader-elect only worker 0 runs the elector; every worker
    must follow it (shared flag in the ledger), or a standby replica schedules against its
    own ledger next to the leader's."""
    from datetime import datetime, timedelta, timezone

    async def main():
        store = FakeKubeStore()
        node = pu.make_node("n0", 2, synthetic_mi355x(2).to_json())
        store.add_node(node)
        fmt = "%Y-%m-%dT%H:%M:%S.%fZ"
        now = datetime.now(timezone.utc)
        store.create_lease("kube-system", {"metadata": {"name": "nano-gpu-scheduler"}, "spec": {
            "holderIdentity": "someone-else", "leaseDurationSeconds": 4,
            "acquireTime": now.strftime(fmt), "renewTime": now.strftime(fmt), "leaseTransitions": 0}})
        runner, api_port = await serve(store)
        port = _free_port()
        ledger = f"/dev/shm/nanogpu-test-standby-{os.getpid()}"
        proc = await _start_replica(api_port, port, ledger, "--leader-elect", "--identity", "me")
        try:
            pod = store.create_pod(pu.make_pod("p", [("c", 30)]))
            body = json.dumps({"Pod": pod, "NodeNames": ["n0"]}).encode()
            assert set(await _statuses(port, "POST", "/scheduler/filter", body)) == {503}
            assert set(await _statuses(port, "GET", "/readyz")) == {503}
            # the other holder stops renewing: after the lease expires this replica leads, and
            # every worker serves
            deadline = time.time() + 20
            while time.time() < deadline:
                if set(await _statuses(port, "GET", "/readyz", n=8)) == {200}:
                    break
                await asyncio.sleep(0.3)
            assert set(await _statuses(port, "POST", "/scheduler/filter", body)) == {200}
            assert store.get_lease("kube-system", "nano-gpu-scheduler")["spec"]["holderIdentity"] == "me"
        finally:
            _stop(proc)
            await runner.cleanup()
            if os.path.exists(ledger):
                os.unlink(ledger)

    asyncio.run(main())


def test_a_crashed_worker_takes_the_replica_down_and_a_stale_region_is_not_reused():
    async def main():
        store = FakeKubeStore()
        store.add_node(pu.make_node("n0", 2, synthetic_mi355x(2).to_json()))
        runner, api_port = await serve(store)
        port = _free_port()
        ledger = f"/dev/shm/nanogpu-test-crash-{os.getpid()}"
        from nanogpu import _native as N

        # a region left by a killed incarnation, holding a pod that no longer exists
        stale = N.Ledger(ledger, 4096, 131072, True)
        t = synthetic_mi355x(2)
        nid = stale.upsert_node("n0", t.ledger_devices(True), t.ledger_topo())
        assert stale.allocate_plan(nid, "ghost", [(60, 0)], [[0]]) == N.OK
        del stale
        proc = await _start_replica(api_port, port, ledger)
        try:
            r, w = await asyncio.open_connection("127.0.0.1", port)
            w.write(b"GET /status HTTP/1.1\r\nHost: x\r\nConnection: close\r\n\r\n")
            status = json.loads((await r.read()).split(b"\r\n\r\n", 1)[1])
            w.close()
            assert [g["Percent"] for g in status["n0"]["GPUs"]] == [100, 100]   # the ghost is gone
            workers = [int(p) for p in subprocess.check_output(["pgrep", "-P", str(proc.pid)]).split()]
            assert len(workers) == 2
            os.kill(workers[1], signal.SIGKILL)
            assert proc.wait(timeout=20) != 0                 # the whole replica exits non-zero
            for w_pid in workers:
                assert not os.path.exists(f"/proc/{w_pid}") or \
                    open(f"/proc/{w_pid}/stat").read().split()[2] == "Z"
        finally:
            _stop(proc)
            await runner.cleanup()
            if os.path.exists(ledger):
                os.unlink(ledger)

    asyncio.run(main())
