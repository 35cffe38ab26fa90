"""Pods with any number of containers (reference allocate.go:54-62 and rater.go:74-110 place
one demand slot per container, without a limit).

A ledger record holds 64 containers (16 inline in the pod's slot, more in an overflow record);
larger pods keep only their GPU-requesting containers there (podutil.ledger_view). Every verb answers in the extender protocol whatever the pod
looks like: filter reports unplaceable pods in FailedNodes, never as an HTTP error.
"""
import asyncio
import json
import random

from nanogpu import types as T
from nanogpu.k8s import podutil as pu

from nanogpu.app import Config, Runtime
from nanogpu.k8s.fake_apiserver import FakeKubeStore, InProcKube
from nanogpu.topology.model import synthetic_mi355x
from test_control_plane import annotated, runtime, wait_for
from test_control_plane import node as mknode
from test_frontend import _dumps, _http


async def _runtime(n_nodes, **kw):
    store = FakeKubeStore()
    for i in range(n_nodes):
        store.add_node(mknode(f"n{i}"))
    rt = Runtime(Config(port=0, host="127.0.0.1", policy_config_path="/nonexistent", **kw), api=InProcKube(store))
    await rt.start()
    assert (rt.native is not None) == (kw.get("frontend", "native") == "native")
    return store, rt


def _sidecar_pod(name, n_containers, gpu_at, pct=20):
    cs = [(f"c{k}", pct if k in gpu_at else 0, 0) for k in range(n_containers)]
    return pu.make_pod(name, cs)


def _schedule(rt, store, pod, nodes):
    """filter -> priorities -> bind over HTTP on the extender; returns the three responses."""
    m = pu.meta(pod)
    res = _http(rt.bound_port, [
        ("POST", "/scheduler/filter", _dumps({"Pod": pod, "NodeNames": nodes})),
        ("POST", "/scheduler/priorities", _dumps({"Pod": pod, "NodeNames": nodes}))])
    fit = json.loads(res[0][1])["NodeNames"] or []
    if not fit:
        return res + [None]
    bind = _http(rt.bound_port, [("POST", "/scheduler/bind", _dumps(
        {"PodName": m["name"], "PodNamespace": m["namespace"], "PodUID": m["uid"], "Node": fit[0]}))])
    return res + bind


def test_forty_container_pod_schedules_through_both_front_doors():
    for frontend in ("native", "aiohttp"):
        async def main():
            store, rt = await _runtime(2, frontend=frontend)
            loop = asyncio.get_running_loop()
            try:
                pod = store.create_pod(_sidecar_pod("big", 40, {25}, pct=30))
                f, p, b = await loop.run_in_executor(None, _schedule, rt, store, pod, ["n0", "n1"])
                assert f[0] == 200 and json.loads(f[1])["NodeNames"], (frontend, f)
                assert p[0] == 200 and len(json.loads(p[1])) == 2
                assert b == (200, b'{"Error":""}'), (frontend, b)
                ann = store.get_pod("default", "big")["metadata"]["annotations"]
                assert ann[T.container_annotation("c25")] != "-1"
                assert all(ann[T.container_annotation(f"c{k}")] == "-1" for k in range(40) if k != 25)
                node = pu.node_name_of(store.get_pod("default", "big"))
                dev = int(ann[T.container_annotation("c25")])
                assert rt.state.status()[node]["GPUs"][dev]["Percent"] == 70
                store.delete_pod("default", "big")
                assert await wait_for(lambda: rt.state.status()[node]["GPUs"][dev]["Percent"] == 100)
            finally:
                await rt.stop()

        asyncio.run(main())


def test_pods_with_more_gpu_containers_than_a_ledger_record_place():
    """The reference places any container count (allocate.go:54-62, rater.go:74-110). A pod with
    66 GPU containers (more than the ledger record's 64 entries) is placed in Python
    (podutil.wide_place) and accounted folded per device (podutil.fold_plan): every container
    gets its device, the device's share is their sum, and deleting the pod gives it all back.
    One that cannot fit fails its nodes with the reason, never a 5xx."""
    for frontend in ("native", "aiohttp"):
        async def main():
            store, rt = await _runtime(2, frontend=frontend)
            loop = asyncio.get_running_loop()
            try:
                pod = store.create_pod(_sidecar_pod("huge", 70, set(range(66)), pct=1))
                f, p, b = await loop.run_in_executor(None, _schedule, rt, store, pod, ["n0", "n1"])
                body = json.loads(f[1])
                assert f[0] == 200 and body["NodeNames"] == ["n0", "n1"] and body["Error"] == "", body
                assert p[0] == 200 and all(h["Score"] > 0 for h in json.loads(p[1]))
                assert b == (200, b'{"Error":""}'), (frontend, b)
                got = store.get_pod("default", "huge")
                ann = got["metadata"]["annotations"]
                devs = [int(ann[T.container_annotation(f"c{k}")]) for k in range(66)]
                assert all(ann[T.container_annotation(f"c{k}")] == "-1" for k in range(66, 70))
                node = pu.node_name_of(got)
                gpus = rt.state.status()[node]["GPUs"]
                used = [100 - g["Percent"] for g in gpus]
                assert sum(used) == 66 and all(used[d] > 0 for d in devs)   # binpack: on as few as fit
                assert rt.state.ledger.lookup(pu.pod_uid(pod))["state"] == "committed"
                store.delete_pod("default", "huge")
                assert await wait_for(lambda: all(g["Percent"] == 100 for g in rt.state.status()[node]["GPUs"]))
                # more than the node holds: 200 x 10 % on 8-GPU nodes
                big = store.create_pod(_sidecar_pod("toobig", 200, set(range(200)), pct=10))
                f, p, b = await loop.run_in_executor(None, _schedule, rt, store, big, ["n0", "n1"])
                body = json.loads(f[1])
                assert f[0] == 200 and not body["NodeNames"] and body["Error"] == ""
                assert all("can't allocate 200 GPU containers" in r for r in body["FailedNodes"].values()), body
                assert p[0] == 200 and [h["Score"] for h in json.loads(p[1])] == [0, 0] and b is None
            finally:
                await rt.stop()

        asyncio.run(main())


def test_a_wide_pod_found_at_restart_is_accounted_from_its_annotations():
    """Checkpoint/resume for a wide pod: the annotations written at bind fold into one ledger
    record on a fresh extender (allocate_existing), the same per-device shares as before."""
    from nanogpu.state.cluster import ClusterState

    st = ClusterState()
    st.register_node(pu.make_node("n0", 8, synthetic_mi355x(8).to_json()))
    pod = _sidecar_pod("wide", 80, set(range(80)), pct=5)
    pod["metadata"]["uid"] = "wide-uid"
    plan, fresh = st.reserve(pod, "n0")
    assert fresh and len(plan) == 80 and all(len(x) == 1 and x[0] >= 0 for x in plan)
    st.commit("wide-uid")
    before = [g["Percent"] for g in st.status()["n0"]["GPUs"]]
    assert sum(100 - x for x in before) == 400
    pod["spec"]["nodeName"] = "n0"
    pod["metadata"]["annotations"] = dict(pu.placement_annotations([f"c{k}" for k in range(80)], plan))
    fresh_state = ClusterState()
    fresh_state.register_node(pu.make_node("n0", 8, synthetic_mi355x(8).to_json()))
    assert fresh_state.allocate_existing(pod)
    assert [g["Percent"] for g in fresh_state.status()["n0"]["GPUs"]] == before
    assert fresh_state.release(pod) and all(g["Percent"] == 100 for g in fresh_state.status()["n0"]["GPUs"])


def test_a_wide_pods_retried_bind_on_another_worker_gets_the_ledger_plan(tmp_shm):
    """ADVICE r04 / VERDICT r04 #5: a wide pod's per-container plan lives in the shared ledger
    (Ledger::reserve_wide), not in one worker's memory. Reserved on worker A, its bind retried on
    worker B (another ClusterState on the same /dev/shm ledger, as the deployment's second
    worker process) answers A's plan, not a new one, with one ledger record and no double
    accounting; a restart (a third state) reads it back; release frees the wide record."""
    from nanogpu.state.cluster import ClusterState

    topo = synthetic_mi355x(8).to_json()
    a = ClusterState(ledger_path=tmp_shm, max_nodes=16, max_pods=4096)
    b = ClusterState(ledger_path=tmp_shm, max_nodes=16, max_pods=4096)
    for st in (a, b):
        st.register_node(pu.make_node("n0", 8, topo))
    pod = _sidecar_pod("wide70", 70, set(range(70)), pct=7)
    pod["metadata"]["uid"] = "wide70-uid"
    # another tenant first, so that a placement recomputed after A's reservation would differ
    other = _sidecar_pod("other", 1, {0}, pct=30)
    other["metadata"]["uid"] = "other-uid"
    a.reserve(other, "n0")
    plan_a, fresh_a = a.reserve(pod, "n0")
    assert fresh_a and len(plan_a) == 70
    used = [100 - g["Percent"] for g in a.status()["n0"]["GPUs"]]
    assert sum(used) == 30 + 70 * 7
    # worker B never saw the pod: its retried bind recovers A's plan from the ledger
    plan_b, fresh_b = b.reserve(pod, "n0")
    assert (plan_b, fresh_b) == (plan_a, False)
    assert [100 - g["Percent"] for g in b.status()["n0"]["GPUs"]] == used     # accounted once
    assert b.ledger.wide_records_used == 1
    # and B committing / A retrying again changes nothing
    b.commit("wide70-uid")
    assert a.reserve(pod, "n0") == (plan_a, False)
    assert a.ledger.lookup("wide70-uid")["state"] == "committed"
    # a pod reserved on n0 retried for another node is refused, not placed twice
    b.register_node(pu.make_node("n1", 8, topo))
    import pytest
    from nanogpu.state.cluster import SchedulingError

    with pytest.raises(SchedulingError):
        b.reserve(pod, "n1")
    # restart: a fresh worker on the same ledger reads the plan back
    c = ClusterState(ledger_path=tmp_shm, max_nodes=16, max_pods=4096)
    c.register_node(pu.make_node("n0", 8, topo))
    assert c.ledger.wide_plan("wide70-uid") == plan_a
    assert c.release_uid("wide70-uid")
    assert c.ledger.wide_plan("wide70-uid") is None and c.ledger.wide_records_used == 0
    assert [100 - g["Percent"] for g in c.status()["n0"]["GPUs"]] == [30] + [0] * 7


def test_wide_pods_in_compat_mode_follow_the_reference_choose():
    """`--compat` keeps the reference's placement for every pod: a wide pod (more GPU containers
    than a ledger record) is placed by the reference's Choose (its executable spec,
    nanogpu.sim.oracle, Go 1.16 sort included) and scored by its Rate on the node as it is."""
    from nanogpu.sim import oracle
    from nanogpu.state.cluster import ClusterState

    for policy in ("binpack", "spread"):
        st = ClusterState(policy=policy, compat=True)
        st.register_node(pu.make_node("n0", 8, synthetic_mi355x(8).to_json()))
        st.register_node(pu.make_node("n1", 8, synthetic_mi355x(8).to_json()))
        pre = _sidecar_pod("pre", 3, {0, 1, 2}, pct=30)
        pre["metadata"]["uid"] = f"pre-{policy}"
        st.reserve(pre, "n0")
        pod = _sidecar_pod(f"wide-{policy}", 100, set(range(0, 100, 4)) | set(range(1, 100, 2)), pct=3)
        pod["metadata"]["uid"] = f"wide-{policy}"
        full = st.pod_demand(pod)
        assert pu.is_wide(full)
        devs = st.ledger.snapshot(st.node_entry("n0").id)["devices"]
        gpus = [oracle.G(int(d["pct_free"]), int(d["pct_total"])) for d in devs]
        want = oracle.choose(gpus, [p for p, _ in full], spread=policy == "spread")
        scores = st.score(pod, ["n0", "n1"])
        assert scores[0] == (oracle.rate_spread if policy == "spread" else oracle.rate_binpack)(gpus)
        plan, fresh = st.reserve(pod, "n0")
        assert fresh and plan == [[i] for i in want], policy
        used = [100 - g["Percent"] for g in st.status()["n0"]["GPUs"]]
        assert sum(used) == 90 + 3 * sum(1 for p, _ in full if p)


def test_fuzz_container_counts_never_answer_5xx():
    async def main():
        store, rt = await _runtime(4)
        loop = asyncio.get_running_loop()
        rng = random.Random(11)
        try:
            for i in range(40):
                n = rng.randint(0, 80)
                gpu = set(rng.sample(range(n), min(n, rng.choice([0, 1, 2, 5, 17, 24, 65])))) if n else set()
                pod = store.create_pod(_sidecar_pod(f"f{i}", n, gpu, pct=rng.choice([1, 2, 5])))
                f, p, b = await loop.run_in_executor(None, _schedule, rt, store, pod, ["n0", "n1", "n2", "n3"])
                assert f[0] == 200 and p[0] == 200, (n, len(gpu), f, p)
                fit = json.loads(f[1])["NodeNames"]
                # the pods are small (at most 65 x 5 % on four 8-GPU nodes): every one fits, the
                # ones with more GPU containers than a ledger record included
                assert fit, (n, len(gpu), f)
                if b is not None:
                    assert b == (200, b'{"Error":""}'), (n, len(gpu), b)
        finally:
            await rt.stop()

    asyncio.run(main())


def test_twenty_four_gpu_containers_schedule_through_both_front_doors_and_rebuild():
    """the reference places any number of GPU containers
    (allocate.go:54-62). 24 containers of 5 % each (over the 16 a pod slot holds inline) take
    an overflow record, schedule through the native and the Python front door, release on
    delete and come back from their annotations after a restart."""
    for frontend in ("native", "aiohttp"):
        async def main():
            store, rt = await _runtime(2, frontend=frontend)
            loop = asyncio.get_running_loop()
            try:
                pod = store.create_pod(_sidecar_pod("wide24", 24, set(range(24)), pct=5))
                f, p, b = await loop.run_in_executor(None, _schedule, rt, store, pod, ["n0", "n1"])
                assert f[0] == 200 and json.loads(f[1])["NodeNames"], (frontend, f)
                assert b == (200, b'{"Error":""}'), (frontend, b)
                got = store.get_pod("default", "wide24")
                ann = got["metadata"]["annotations"]
                devs = [int(ann[T.container_annotation(f"c{k}")]) for k in range(24)]
                node = pu.node_name_of(got)
                used = {d: devs.count(d) * 5 for d in set(devs)}
                gpus = rt.state.status()[node]["GPUs"]
                assert all(gpus[d]["Percent"] == 100 - u for d, u in used.items())
                led = rt.state.ledger
                rec = led.lookup(pu.pod_uid(got))
                assert len(rec["demand"]) == 24 and [x[0] for x in rec["plan"]] == devs
                assert led.overflow_records_used == 1
                # restart: a fresh runtime rebuilds the wide pod from its annotations
                rt2 = await runtime(store)
                try:
                    g2 = rt2.state.status()[node]["GPUs"]
                    assert all(g2[d]["Percent"] == 100 - u for d, u in used.items())
                    assert rt2.state.ledger.lookup(pu.pod_uid(got))["plan"] == rec["plan"]
                finally:
                    await rt2.stop()
                store.delete_pod("default", "wide24")
                assert await wait_for(lambda: led.lookup(pu.pod_uid(got)) is None)
                assert led.overflow_records_used == 0
                assert all(g["Percent"] == 100 for g in rt.state.status()[node]["GPUs"])
            finally:
                await rt.stop()

        asyncio.run(main())


def test_restart_rebuilds_a_pod_with_more_than_16_containers():
    async def main():
        store = FakeKubeStore()
        store.add_node(mknode("n0"))
        plan = [[-1]] * 20
        plan[3], plan[17] = [2], [5]
        p = annotated("wide", "n0", plan, pct=0)
        for k in (3, 17):
            p["spec"]["containers"][k]["resources"]["limits"][T.RESOURCE_GPU_PERCENT] = "40"
        store.create_pod(p)
        rt = await runtime(store)
        try:
            gpus = rt.state.status()["n0"]["GPUs"]
            assert gpus[2]["Percent"] == 60 and gpus[5]["Percent"] == 60
            assert rt.state.ledger.n_pods == 1
        finally:
            await rt.stop()

    asyncio.run(main())


def test_node_with_more_devices_than_a_slot_holds_fails_alone():
    """A 10-GPU CPX node exposes 80 schedulable devices (a ledger slot holds 64): it is
    reported in FailedNodes with the reason while the other nodes keep scheduling."""
    from nanogpu.topology.model import synthetic_mi355x

    async def main():
        store, rt = await _runtime(1)
        big = synthetic_mi355x(10, "CPX")
        store.add_node(pu.make_node("wide", len(big.devices), big.to_json(), {"amd.com/gpu.present": "true"}))
        loop = asyncio.get_running_loop()
        try:
            pod = store.create_pod(_sidecar_pod("p", 1, {0}, pct=10))
            f, p, b = await loop.run_in_executor(None, _schedule, rt, store, pod, ["wide", "n0"])
            body = json.loads(f[1])
            assert f[0] == 200 and body["NodeNames"] == ["n0"], body
            assert "too many devices" in body["FailedNodes"]["wide"], body
            assert b == (200, b'{"Error":""}')
        finally:
            await rt.stop()

    asyncio.run(main())


from hypothesis import given, settings   # noqa: E402
from hypothesis import strategies as st   # noqa: E402


@settings(max_examples=150, deadline=None)
@given(st.lists(st.tuples(st.sampled_from([0, 1, 2, 5, 10, 25, 100, 200]), st.sampled_from([0, 512, 4096])),
                min_size=65, max_size=160),
       st.booleans(), st.lists(st.integers(0, 100), min_size=8, max_size=8))
def test_wide_placement_never_overcommits_and_folds_exactly(demand, spread, used):
    """podutil.wide_place / fold_plan on any wide demand over a partly used 8-device node: a
    placement never overcommits a device's percent or HBM, whole-device containers get devices
    nobody else uses, and the folded record holds each device's exact sum (a device filled to
    100 % is held whole); the ledger accepts the folded record and gives everything back."""
    devs = [{"pct_free": 100 - u, "pct_total": 100, "mib_free": 262144 - 1024 * u, "mib_total": 262144,
             "healthy": True, "pool": -1} for u in used]
    plan = pu.wide_place(devs, demand, spread=spread)
    if plan is None:
        return
    assert len(plan) == len(demand)
    pct = [0] * 8
    mib = [0] * 8
    whole = set()
    for (p, m), idx in zip(demand, plan):
        if p <= 0 and m <= 0:
            assert idx == [-1]
            continue
        if p >= 100 and p % 100 == 0:
            assert len(idx) == p // 100 and not whole.intersection(idx)
            whole.update(idx)
            for j in idx:
                pct[j] += 100
        else:
            (j,) = idx
            pct[j] += p
            mib[j] += m
    for j in range(8):
        assert pct[j] <= devs[j]["pct_free"] and mib[j] <= devs[j]["mib_free"]
        if j in whole:
            assert pct[j] == 100 and devs[j]["pct_free"] == 100
    folded, fplan = pu.fold_plan(demand, plan)
    assert len(folded) <= 8 and sorted(x[0] for x in fplan) == [j for j in range(8) if pct[j] or mib[j]]
    for (fp, fm), (j,) in zip(folded, fplan):
        assert fp == min(100, pct[j]) and (fm == mib[j] or j in whole)
    from nanogpu.state.cluster import ClusterState

    st_ = ClusterState()
    node = pu.make_node("n0", 8, synthetic_mi355x(8, hbm_mib=262144).to_json())
    e = st_.register_node(node)
    for j, u in enumerate(used):    # the same pre-existing load
        if u:
            assert st_.ledger.allocate_plan(e.id, f"pre{j}", [(u, 1024 * u)], [[j]], True) == 0
    assert st_.ledger.allocate_plan(e.id, "wide", folded, fplan, True) == 0
    assert st_.ledger.release("wide") == 0
