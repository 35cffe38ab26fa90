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


def test_two_workers_share_one_ledger():
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
                                 "--policyConfigPath", "/nonexistent"],
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
