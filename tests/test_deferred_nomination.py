"""Nominations deferred past the answer with several worker processes.

A worker with one front-door thread makes a filter's / priorities' nomination after writing its
answer (Frontend::run_deferred), off kube-scheduler's cycle. kube-scheduler's next filter can
reach another worker process over another connection: that worker must not read the ledger
before the nomination exists, or it may answer the same tight device for a second pod. The
ledger counts deferred nominations begun and made; a verb on any worker waits (bounded) until
they match (Ledger::wait_deferred_nominations).
"""
from __future__ import annotations

import json
import threading
import time

from nanogpu import _native as N
from nanogpu.k8s import podutil as pu
from nanogpu.topology.model import synthetic_mi355x


def test_ledger_wait_returns_once_the_deferred_nomination_is_made(tmp_shm):
    L = N.Ledger(tmp_shm, 16, 256, True)
    assert L.wait_deferred_nominations(1_000)          # nothing pending: at once
    L.deferred_nomination_begin()
    t0 = time.perf_counter()
    assert not L.wait_deferred_nominations(200_000)    # never made: bounded (200 us)
    assert time.perf_counter() - t0 < 0.05
    th = threading.Timer(0.002, L.deferred_nomination_end)
    th.start()
    t0 = time.perf_counter()
    assert L.wait_deferred_nominations(2_000_000_000)
    assert 0.0015 < time.perf_counter() - t0 < 1.0
    th.join()


def test_the_verb_waits_for_a_deferred_nomination_made_within_its_bound(tmp_shm):
    """The common case: the deferred nomination lands microseconds after the answer, well
    inside the verb's 100 us bound: the other worker's filter waits and sees it, no retry."""
    led1 = N.Ledger(tmp_shm, 16, 256, True)
    led2 = N.Ledger(tmp_shm, 16, 256, False)
    t = synthetic_mi355x(1)
    n0 = led1.upsert_node("n0", t.ledger_devices(True), t.ledger_topo())
    led1.upsert_node("n1", t.ledger_devices(True), t.ledger_topo())
    assert led1.allocate_plan(n0, "base", [(50, 0)], [[0]], True) == N.OK
    opts = N.Options(N.Policy.BINPACK)
    fe2 = N.Frontend(led2, "127.0.0.1", 0, 1)
    fe2.set_options(opts, False, True, True, 100)
    a = pu.make_pod("a", [("c", 50)])
    b = pu.make_pod("b", [("c", 50)])
    body = json.dumps({"Pod": b, "Nodes": None, "NodeNames": ["n0", "n1"]}, separators=(",", ":")).encode()
    wins = 0
    try:
        for k in range(20):
            uid = f"{pu.pod_uid(a)}-{k}"
            led1.deferred_nomination_begin()
            go = threading.Event()

            def make():
                go.wait()
                led1.nominate(n0, uid, [(50, 0)], opts)
                led1.deferred_nomination_end()

            th = threading.Thread(target=make)
            th.start()
            go.set()
            ok, ans = fe2.verb(body, False)
            th.join()
            wins += json.loads(ans)["NodeNames"] == ["n1"]
            led1.drop_nomination(uid)
            led2.drop_nomination(pu.pod_uid(b))
        # without the wait the verb answers before the other thread nominates: 0 of 20. A
        # thread's wake-up can exceed the 100 us bound on a loaded host (this container is a VM
        # whose hypervisor steals up to 9 % of the CPU time under load: 16 of 20 seen there)
        assert wins >= 12, wins
    finally:
        fe2.stop()
