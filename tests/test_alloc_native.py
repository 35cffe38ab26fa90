"""Native (MI355X) placement mode of the C++ allocator: properties and topology behaviour.

Compat mode is pinned bit-for-bit to the reference oracle in test_parity.py /
test_alloc_golden.py; these tests pin what the native mode adds: the HBM dimension,
partition / xGMI / NUMA-aware multi-container placement and the ledger invariants.
"""
import os
import random

from hypothesis import given, settings
from hypothesis import strategies as st

from nanogpu import _native as N
from nanogpu.topology.model import synthetic_mi355x

BIN = N.Options(N.Policy.BINPACK)
SPR = N.Options(N.Policy.SPREAD)


def ledger_with(topo, n_nodes=1, track_hbm=True):
    L = N.Ledger("", 16, 4096, True)
    ids = [L.upsert_node(f"n{i}", topo.ledger_devices(track_hbm), topo.ledger_topo()) for i in range(n_nodes)]
    return L, ids


def devices_of(plan):
    return [i for idx in plan for i in idx if i >= 0]


def test_tp4_whole_gpus_stay_on_one_socket_and_fast_links():
    t = synthetic_mi355x(8)
    t.link_bw[0][1] = t.link_bw[1][0] = 38.0
    L, (nid,) = ledger_with(t)
    rc, _ = L.reserve(nid, "pre", [(50, 0)], BIN)       # GPU 0 half used
    assert rc == N.OK
    for opts in (BIN, SPR):
        rc, plan, _ = L.assume(nid, [(100, 0)] * 4, opts)
        assert rc == N.OK
        gpus = {t.devices[i].gpu for i in devices_of(plan)}
        assert gpus == {4, 5, 6, 7}, (opts, plan)       # NUMA 1, no degraded link


def test_spread_share_pod_avoids_degraded_link():
    t = synthetic_mi355x(8)
    for a, b in ((0, 1), (4, 5)):
        t.link_bw[a][b] = t.link_bw[b][a] = 20.0
    L, (nid,) = ledger_with(t)
    rc, plan, _ = L.assume(nid, [(25, 0)] * 4, SPR)
    gpus = [t.devices[i].gpu for i in devices_of(plan)]
    # every 4-GPU set inside one socket contains a 20 GB/s link here; xGMI joins all 8 GPUs
    # directly, so the ring's slowest link matters more than the socket boundary
    assert len(set(gpus)) == 4
    assert all(t.link_bw[a][b] > 20.0 for a in gpus for b in gpus if a != b)


def test_cpx_spread_uses_distinct_physical_gpus_binpack_uses_siblings():
    t = synthetic_mi355x(8, "CPX")
    L, (nid,) = ledger_with(t)
    rc, plan, _ = L.assume(nid, [(50, 0)] * 4, SPR)
    assert len({t.devices[i].gpu for i in devices_of(plan)}) == 4
    rc, plan, _ = L.assume(nid, [(100, 0)] * 4, BIN)
    assert len({t.devices[i].gpu for i in devices_of(plan)}) == 1   # four XCD partitions of one GPU
    rc, plan, _ = L.assume(nid, [(200, 0)], BIN)                     # 2-device container
    assert rc == N.OK and len(devices_of(plan)) == 2
    assert len({t.devices[i].gpu for i in devices_of(plan)}) == 1


def test_binpack_fills_one_device_before_the_next():
    L, (nid,) = ledger_with(synthetic_mi355x(8))
    devs = []
    for k in range(10):
        rc, plan = L.reserve(nid, f"p{k}", [(20, 0)], BIN)
        assert rc == N.OK
        devs.append(plan[0][0])
    assert devs[:5] == [devs[0]] * 5 and devs[5:] == [devs[5]] * 5 and devs[0] != devs[5]


def test_hbm_limits_colocation():
    t = synthetic_mi355x(1)
    L, (nid,) = ledger_with(t)
    ok = sum(L.reserve(nid, f"p{k}", [(10, 64 * 1024)], BIN)[0] == N.OK for k in range(10))
    assert ok == t.devices[0].hbm_mib // (64 * 1024)      # 4 x 64 GiB in 288 GB
    L2, (nid2,) = ledger_with(t, track_hbm=False)
    assert sum(L2.reserve(nid2, f"p{k}", [(10, 64 * 1024)], BIN)[0] == N.OK for k in range(10)) == 10


_demand = st.lists(st.tuples(st.sampled_from([0, 5, 10, 20, 25, 33, 50, 100, 200]),
                             st.sampled_from([0, 0, 1024, 16384, 65536])), min_size=1, max_size=4)


@settings(max_examples=60, deadline=None)
@given(st.lists(_demand, min_size=1, max_size=40), st.sampled_from(["SPX", "QPX", "CPX"]),
       st.sampled_from([N.Policy.BINPACK, N.Policy.SPREAD, N.Policy.RANDOM, N.Policy.FIRSTFIT]), st.integers(0, 99))
def test_ledger_invariants_under_random_churn(demands, mode, policy, seed):
    t = synthetic_mi355x(8, mode)
    L, ids = ledger_with(t, 2)
    o = N.Options(policy, seed=seed)
    rng = random.Random(seed)
    live = []
    for k, d in enumerate(demands):
        nid = rng.choice(ids)
        rc, plan = L.reserve(nid, f"p{k}", d, o)
        if rc == N.OK:
            assert len(plan) == len(d)
            for (pct, mib), idx in zip(d, plan):
                assert (idx == [-1]) == (pct == 0 and mib == 0)   # an HBM-only container needs a device
                if pct > 100:
                    assert len(idx) == pct // 100 and len(set(idx)) == len(idx)
            L.commit(f"p{k}")
            live.append(f"p{k}")
        if live and rng.random() < 0.3:
            L.release(live.pop(rng.randrange(len(live))))
        for nid in ids:
            for dv in L.snapshot(nid)["devices"]:
                assert 0 <= dv["pct_free"] <= dv["pct_total"]
                assert 0 <= dv["mib_free"] <= dv["mib_total"]
    for u in live:
        assert L.release(u) == N.OK
    for nid in ids:   # allocate -> release is the identity
        for dv in L.snapshot(nid)["devices"]:
            assert dv["pct_free"] == dv["pct_total"] and dv["mib_free"] == dv["mib_total"]


@settings(max_examples=60, deadline=None)
@given(_demand, st.sampled_from(["SPX", "CPX"]), st.sampled_from([N.Policy.BINPACK, N.Policy.SPREAD]),
       st.booleans(), st.lists(st.tuples(st.sampled_from([10, 30, 60]), st.just(0)), max_size=6), st.randoms())
def test_container_order_does_not_change_the_placement(d, mode, policy, compat, pre, rnd):
    """SURVEY §4 property: containers are placed largest-first and mapped back, so a
    permutation of a pod's containers lands the same (demand, devices) multiset. (First-fit
    is the reference's SampleRater, rater.go:29-50, which places in container order.)"""
    o = N.Options(policy, compat=compat)
    perm = list(d)
    rnd.shuffle(perm)
    results = []
    for demand in (d, perm):
        L, (nid,) = ledger_with(synthetic_mi355x(2, mode))
        for k, p in enumerate(pre):            # the same partly used node both times
            L.reserve(nid, f"pre{k}", [p], o)
        rc, plan = L.reserve(nid, "pod", demand, o)
        # compat mode ignores HBM as the reference does: containers of equal percent are
        # interchangeable there, so only the percent identifies a container
        key = (lambda c: c[0]) if compat else (lambda c: c)
        results.append((rc, sorted((key(c), tuple(ix)) for c, ix in zip(demand, plan)) if rc == N.OK else None))
    assert results[0] == results[1]


def test_partial_plan_failure_restores_exactly_D5():
    """Reference allocate.go:108-113 restores Demand[i] (not [j]) and does not skip -1
    indices when a multi-container allocation fails half way; here the debit is undone
    exactly."""
    L, (nid,) = ledger_with(synthetic_mi355x(2))
    assert L.allocate_plan(nid, "a", [(70, 0)], [[1]], True) == N.OK
    before = L.snapshot(nid)["devices"]
    # container 0 fits on device 0, container 1 (40 %) does not fit on device 1 (30 % free)
    rc = L.allocate_plan(nid, "b", [(50, 0), (0, 0), (40, 0)], [[0], [-1], [1]], True)
    assert rc != N.OK
    assert L.snapshot(nid)["devices"] == before and L.lookup("b") is None


# ----------------------------------------------------------------------------- HBM pools
def _pool_views(L, nid):
    by = {}
    for d in L.snapshot(nid)["devices"]:
        if d["pool"] >= 0:
            by.setdefault(d["pool"], set()).add((d["mib_free"], d["mib_total"]))
    return by


def test_cpx_partitions_share_the_gpu_hbm_pool():
    """NPS1 + CPX: the 8 XCD partitions of a GPU draw from one 288 GB pool, so a 1-XCD pod can
    take 100 GiB (a static 1/8 split would cap it at 36 GiB) while the pool is never
    over-committed across siblings."""
    t = synthetic_mi355x(1, "CPX")
    pool = t.devices[0].hbm_mib
    L, (nid,) = ledger_with(t)
    big = 100 * 1024
    placed = []
    for k in range(3):
        rc, plan = L.reserve(nid, f"m{k}", [(10, big)], BIN)
        if rc == N.OK:
            placed.append(plan[0][0])
    assert len(placed) == 2                       # 2 x 100 GiB fit in 288 GB, the third does not
    views = _pool_views(L, nid)
    assert views == {0: {(pool - 2 * big, pool)}}  # every member mirrors the pool
    f = L.frag(0)
    assert f["mib_free_total"] == pool - 2 * big        # the pool is counted once, not 8 times
    assert f["mib_free_partial"] == pool - 2 * big      # and it is partial (two members in use)
    # a whole-partition grant (2 devices) takes 2 x (pool / 8)
    rc, plan = L.reserve(nid, "w", [(200, 0)], BIN)
    assert rc == N.OK and len(plan[0]) == 2
    assert _pool_views(L, nid) == {0: {(pool - 2 * big - 2 * (pool // 8), pool)}}
    for u in ("m0", "m1", "w"):
        assert L.release(u) == N.OK
    assert _pool_views(L, nid) == {0: {(pool, pool)}}


@settings(max_examples=40, deadline=None)
@given(st.lists(_demand, min_size=1, max_size=40), st.sampled_from([("CPX", "NPS1"), ("CPX", "NPS2"),
                                                                    ("QPX", "NPS1"), ("DPX", "NPS2")]),
       st.sampled_from([N.Policy.BINPACK, N.Policy.SPREAD, N.Policy.FIRSTFIT]), st.booleans(), st.integers(0, 99))
def test_pool_mirrors_stay_consistent_under_churn(demands, modes, policy, compat, seed):
    t = synthetic_mi355x(2, *modes)
    L, (nid,) = ledger_with(t)
    o = N.Options(policy, compat=compat, seed=seed)
    rng = random.Random(seed)
    live = []
    for k, d in enumerate(demands):
        if L.reserve(nid, f"p{k}", d, o)[0] == N.OK:
            live.append(f"p{k}")
        if live and rng.random() < 0.3:
            L.release(live.pop(rng.randrange(len(live))))
        for views in _pool_views(L, nid).values():
            assert len(views) == 1                        # all members agree
            (free, total), = views
            assert 0 <= free <= total
    for u in live:
        L.release(u)
    for d in L.snapshot(nid)["devices"]:
        assert d["mib_free"] == d["mib_total"] and d["pct_free"] == d["pct_total"]


def test_nomination_lifecycle():
    """Ledger::nominate: tentative at priorities, adopted by reserve on the same node, moved
    by a reserve elsewhere, dropped only while still a nomination, swept when stale."""
    t = synthetic_mi355x(8)
    L, (a, b) = ledger_with(t, 2)
    free = lambda nid: sum(d["pct_free"] for d in L.snapshot(nid)["devices"])   # noqa: E731
    assert L.nominate(a, "p", [(50, 0)], BIN) == N.OK
    assert L.lookup("p")["state"] == "nominated" and free(a) == 750
    assert L.nominate(a, "p", [(50, 0)], BIN) == N.OK_EXISTING            # repeated priorities
    rc, plan = L.reserve(a, "p", [(50, 0)], BIN)
    assert rc == N.OK and L.lookup("p")["state"] == "reserved" and free(a) == 750   # adopted, owned
    assert L.drop_nomination("p") == N.OK_EXISTING and free(a) == 750            # bound: left alone
    assert L.nominate(a, "p", [(50, 0)], BIN) == N.OK_EXISTING                  # bound: left alone
    # nominated on a, bound on b: a is freed
    assert L.nominate(a, "q", [(100, 0)], BIN) == N.OK and free(a) == 650
    rc, _ = L.reserve(b, "q", [(100, 0)], BIN)
    assert rc == N.OK and L.lookup("q")["node"] == b and free(a) == 750 and free(b) == 700
    # a newer priorities call moves the nomination
    assert L.nominate(a, "r", [(30, 0)], BIN) == N.OK and L.nominate(b, "r", [(30, 0)], BIN) == N.OK
    assert free(a) == 750 and free(b) == 670
    assert L.drop_nomination("r") == N.OK and L.lookup("r") is None and free(b) == 700
    assert L.drop_nomination("r") == N.ERR_UNKNOWN_POD
    # stale nominations are swept, reservations are not
    assert L.nominate(a, "s", [(10, 0)], BIN) == N.OK
    assert L.expired_nominations(-1.0) == ["s"] and "s" not in L.expired_reservations(-1.0)
    # annotations of a pod bound elsewhere win over our nomination
    assert L.allocate_plan(b, "s", [(10, 0)], [[3]], True) == N.OK
    assert L.lookup("s")["node"] == b and free(a) == 750 and free(b) == 690


def test_memory_bound_shares_pair_with_compute_bound_neighbours():
    """CU masks do not split HBM bandwidth (profiles/gpu_calibration.md: a lone 25 % tenant
    streams at 51 % of the device, two streaming tenants split it 25/75). Binpack therefore
    places a memory-bound share (nano-gpu/memory-bound) on the device with the fewest
    memory-bound tenants first; compute-bound shares still pack as before."""
    from nanogpu.k8s.podutil import Req

    t = synthetic_mi355x(2)
    L, (nid,) = ledger_with(t)
    mb = [Req(25, 0, N.FLAG_MEM_BOUND)]
    rc, p1 = L.reserve(nid, "mb1", mb, BIN)
    assert rc == N.OK and devices_of(p1) == [0]
    rc, p2 = L.reserve(nid, "mb2", mb, BIN)          # plain binpack would stack it on device 0
    assert rc == N.OK and devices_of(p2) == [1]
    rc, p3 = L.reserve(nid, "cb", [(25, 0)], BIN)     # compute-bound: best fit, either device
    assert rc == N.OK
    assert [d["mem_bound"] for d in L.snapshot(nid)["devices"]] == [1, 1]
    rc, p4 = L.reserve(nid, "mb3", mb, BIN)           # both hold one: best fit decides
    assert rc == N.OK and devices_of(p4) == devices_of(p3)
    assert L.release("mb2") == N.OK
    assert sorted(d["mem_bound"] for d in L.snapshot(nid)["devices"]) == [0, 2]
    # without the flag the same stream stacks on device 0 (the reference's behaviour)
    L2, (n2,) = ledger_with(t)
    assert [devices_of(L2.reserve(n2, f"p{i}", [(25, 0)], BIN)[1]) for i in range(2)] == [[0], [0]]


def test_priorities_prefer_a_node_without_memory_bound_tenants():
    from nanogpu.k8s.podutil import Req

    t = synthetic_mi355x(1)
    L, (a, b) = ledger_with(t, n_nodes=2)
    assert L.reserve(a, "x", [Req(30, 0, N.FLAG_MEM_BOUND)], BIN)[0] == N.OK
    assert L.reserve(b, "y", [(30, 0)], BIN)[0] == N.OK
    sa, sb = L.score([a, b], [Req(30, 0, N.FLAG_MEM_BOUND)], BIN)
    assert sb > sa                                    # pair with the compute-bound tenant
    ca, cb = L.score([a, b], [(30, 0)], BIN)
    assert ca == cb                                   # no preference for plain shares


def test_stream_owner_learning_needs_a_lone_committed_tenant():
    """Ledger::learn_stream_owners: only a hot device holding exactly one committed pod with a
    known owner teaches anything (HBM activity is a device counter); reserved (not yet bound)
    pods and shared devices teach nothing; a whole-device pod is alone on each of its devices."""
    t = synthetic_mi355x(4)
    L, (nid,) = ledger_with(t)
    for key, owner, demand, plan in (("p1", "o1", [(30, 0)], [[0]]), ("p2", "o2", [(30, 0)], [[1]]),
                                     ("p3", "o3", [(30, 0)], [[1]]), ("p4", "o4", [(200, 0)], [[2, 3]])):
        assert L.allocate_plan(nid, key, demand, plan, True) == N.OK
        assert L.set_pod_owner(key, owner) == N.OK
    assert L.reserve(nid, "p5", [(30, 0)], BIN)[0] == N.OK           # reserved only
    assert L.set_pod_owner("p5", "o5") == N.OK
    assert L.set_pod_owner("nope", "o9") == N.ERR_UNKNOWN_POD
    for dev in range(4):
        assert L.set_mem_hot(nid, dev, True) == N.OK
    learned, forgotten = L.learn_stream_owners(True)
    assert (learned, forgotten) == (2, 0)
    assert [L.is_stream_owner(o) for o in ("o1", "o2", "o3", "o4", "o5")] == [True, False, False, True, False]
    assert L.learn_stream_owners(True) == (0, 0)                     # already known
    assert L.set_mem_hot(nid, 0, False) == N.OK
    assert L.learn_stream_owners(False) == (0, 0) and L.is_stream_owner("o1")   # no forgetting asked
    assert L.learn_stream_owners(True) == (0, 1) and not L.is_stream_owner("o1")
    # a released pod's slot reused by a new pod does not inherit the old owner
    assert L.release("p1") == N.OK
    assert L.allocate_plan(nid, "p1", [(30, 0)], [[0]], True) == N.OK
    assert L.lookup("p1")["owner"] == 0


def test_stream_owner_learning_decides_per_owner_and_forgets_slowly():
    """one owner with a lone replica on a hot device and another on a cool device is
    learned and stays learned (the decision is per owner, not per device in hash order); a
    learned owner is forgotten only after `forget_after` passes in a row with every lone
    replica cool."""
    t = synthetic_mi355x(4)
    L, (nid,) = ledger_with(t)
    for key, dev in (("r1", 0), ("r2", 1)):
        assert L.allocate_plan(nid, key, [(30, 0)], [[dev]], True) == N.OK
        assert L.set_pod_owner(key, "rs") == N.OK
    assert L.set_mem_hot(nid, 0, True) == N.OK            # r1's device hot, r2's cool
    for _ in range(5):
        assert L.learn_stream_owners(True, forget_after=1) in ((1, 0), (0, 0))
        assert L.is_stream_owner("rs")
    assert L.set_mem_hot(nid, 0, False) == N.OK           # both cool now
    assert L.learn_stream_owners(True, forget_after=3) == (0, 0) and L.is_stream_owner("rs")
    assert L.learn_stream_owners(True, forget_after=3) == (0, 0) and L.is_stream_owner("rs")
    assert L.set_mem_hot(nid, 1, True) == N.OK            # hot again: the streak starts over
    assert L.learn_stream_owners(True, forget_after=3) == (0, 0)
    assert L.set_mem_hot(nid, 1, False) == N.OK
    for _ in range(2):
        assert L.learn_stream_owners(True, forget_after=3) == (0, 0) and L.is_stream_owner("rs")
    assert L.learn_stream_owners(True, forget_after=3) == (0, 1) and not L.is_stream_owner("rs")


def test_a_pod_that_replaced_a_streaming_tenant_is_not_blamed_for_its_mark():
    """the HBM-hot mark averages a window of past samples; a pod recorded after that
    window began (it replaced the streaming tenant that heated the device) is not attributed."""
    t = synthetic_mi355x(2)
    L, (nid,) = ledger_with(t)
    assert L.allocate_plan(nid, "streamer", [(50, 0)], [[0]], True) == N.OK
    assert L.set_pod_owner("streamer", "hot-job") == N.OK
    assert L.set_mem_hot(nid, 0, True) == N.OK
    assert L.release("streamer") == N.OK                   # the tenant ends, the mark lingers
    cutoff = N.mono_now()                                  # start of the mark's window
    assert L.allocate_plan(nid, "newcomer", [(50, 0)], [[0]], True) == N.OK
    assert L.set_pod_owner("newcomer", "compute-job") == N.OK
    assert L.learn_stream_owners(True, reserved_before=cutoff) == (0, 0)
    assert not L.is_stream_owner("compute-job")
    # once a whole window has passed with it alone there, the mark is its own
    assert L.learn_stream_owners(True, reserved_before=N.mono_now()) == (1, 0)
    assert L.is_stream_owner("compute-job")


def test_overflow_records_hold_wide_pods_and_are_reused():
    """Pods over 16 containers spill into the ledger's overflow records: lookups return the
    whole demand and plan, a release frees the record for the next wide pod."""
    t = synthetic_mi355x(8)
    L = N.Ledger("", 4, 64, True)           # 64 pods -> 64 overflow records
    nid = L.upsert_node("n0", t.ledger_devices(True), t.ledger_topo())
    wide = [(2, 0)] * 40
    rc, plan = L.reserve(nid, "w0", wide, BIN)
    assert rc == N.OK and len(plan) == 40
    rec = L.lookup("w0")
    assert rec["demand"] == [(2, 0)] * 40 and rec["plan"] == plan
    assert L.overflow_records_used == 1
    assert L.release("w0") == N.OK and L.overflow_records_used == 0
    keys = []
    for i in range(64):
        rc, _ = L.reserve(nid, f"w{i}", [(1, 0)] * 17, BIN)
        if rc != N.OK:
            break
        keys.append(f"w{i}")
    assert L.overflow_records_used == len(keys) == 47      # 800 % / 17 % per pod
    for k in keys:
        assert L.release(k) == N.OK
    assert L.overflow_records_used == 0 and L.n_pods == 0
    assert all(d["pct_free"] == 100 for d in L.snapshot(nid)["devices"])


def test_share_aware_learner_threshold_follows_the_streaming_curve():
    """with a curve the learner compares a lone pod's device activity with
    the curve at that pod's share. The default curve (types.HBM_STREAMING_CURVE, measured on
    the box) halved: 12.5 % -> 5.5, 25 % -> 15, 75 % -> 20 (capped at the device threshold, 0.20)."""
    from nanogpu.config.policy import PolicySpec

    curve = PolicySpec().learn_curve()
    t = synthetic_mi355x(4)
    L, (nid,) = ledger_with(t)
    for key, owner, pct, dev, busy in (("a", "o-small", 12, 0, 10), ("b", "o-quarter", 25, 1, 30),
                                       ("c", "o-big-cool", 75, 2, 18), ("d", "o-big-hot", 75, 3, 40)):
        assert L.allocate_plan(nid, key, [(pct, 0)], [[dev]], True) == N.OK
        L.set_pod_owner(key, owner)
        assert L.set_mem_busy(nid, dev, busy) == N.OK
    assert [d["mem_busy"] for d in L.snapshot(nid)["devices"]] == [10, 30, 18, 40]
    assert L.learn_stream_owners(True, N.mono_now(), 1, curve) == (3, 0)
    assert [L.is_stream_owner(o) for o in ("o-small", "o-quarter", "o-big-cool", "o-big-hot")] == \
        [True, True, False, True]
    # without a curve the device mark decides (none set here)
    L2, (nid2,) = ledger_with(t)
    assert L2.allocate_plan(nid2, "b", [(25, 0)], [[1]], True) == N.OK
    L2.set_pod_owner("b", "o-quarter")
    L2.set_mem_busy(nid2, 1, 30)
    assert L2.learn_stream_owners(True) == (0, 0)


def test_bind_handoff_slots_put_take_and_size_limit(tmp_path):
    """Ledger::put_pod_info / take_pod_info: a blob stored under a pod key is taken once by any
    process attached to the region; one too large for a slot is refused (the bind then goes
    the slow way)."""
    path = f"/dev/shm/nanogpu-test-info-{os.getpid()}"
    try:
        a = N.Ledger(path, 8, 1024, True)
        b = N.Ledger(path, 8, 1024, True)        # a second worker attaching
        assert a.attached == 2 and b.attached == 2
        assert a.put_pod_info("uid-1", b"\x01\x02payload")
        assert b.take_pod_info("uid-2") is None
        assert b.take_pod_info("uid-1") == b"\x01\x02payload"
        assert a.take_pod_info("uid-1") is None  # taken once
        assert not a.put_pod_info("uid-3", b"x" * 5000)
        # 4-way buckets: 300 pods in flight over 1024 slots all survive but a handful (a
        # direct-mapped table would lose about one in eight to collisions)
        keys = [f"pod-{i:04d}" for i in range(300)]
        for k in keys:
            assert a.put_pod_info(k, k.encode())
        got = sum(b.take_pod_info(k) == k.encode() for k in keys)
        assert got >= 290, got
        del b
        assert a.attached == 1
    finally:
        try:
            os.unlink(path)
        except FileNotFoundError:
            pass


def test_pod_keys_are_views_and_keys_no_slot_holds_never_match():
    """The ledger's key APIs take string views (a stack copy of the key, no heap string): a
    63-character key is held and found; an empty key or one of 64 characters or more is refused
    by reserve and, where a call does not check sizes, reads as the empty key, which no slot
    holds. A longer key that starts with a held key's text never finds that pod."""
    L, (nid,) = ledger_with(synthetic_mi355x(8))
    k63 = "u" * 63
    rc, _ = L.reserve(nid, k63, [(10, 0)], BIN)
    assert rc == N.OK and L.lookup(k63) is not None
    assert L.lookup(k63 + "x") is None and L.lookup(k63 + "x" * 40) is None
    assert L.release(k63 + "x") != N.OK and L.lookup(k63) is not None
    for bad in ("", "v" * 64, "w" * 200):
        rc, _ = L.reserve(nid, bad, [(10, 0)], BIN)
        assert rc != N.OK and L.lookup(bad) is None
    assert L.release(k63) == N.OK and L.lookup(k63) is None


def test_holds_any_matches_lookup_over_a_key_list():
    """holds_any (the bench's release check: one call for a burst's keys) is true exactly when
    lookup finds one of the keys; bad keys never match."""
    L, (nid,) = ledger_with(synthetic_mi355x(8))
    keys = [f"h{i}" for i in range(40)]
    for k in keys[::3]:
        assert L.reserve(nid, k, [(5, 0)], BIN)[0] == N.OK
    assert L.holds_any(keys) and L.holds_any(keys[:1]) and not L.holds_any(keys[1:3])
    assert not L.holds_any([]) and not L.holds_any(["", "z" * 64])
    for k in keys[::3]:
        assert L.release(k) == N.OK
    assert not L.holds_any(keys) and all(L.lookup(k) is None for k in keys)


@settings(max_examples=60, deadline=None)
@given(st.lists(st.tuples(st.booleans(), st.integers(0, 199)), min_size=50, max_size=600))
def test_pod_table_stays_exact_under_churn_with_tombstone_cleanup(ops):
    """The pod table is open addressing with linear probing per shard: a freed slot becomes
    empty when the next one is (with the dead tombstones before it), and a shard rehashes once
    tombstones are a quarter of it. Over any reserve / release sequence on a table small enough
    to collide constantly (4 slots a shard: chains wrap round), every key is found exactly when
    it is held (a full shard refuses the reserve; the model follows)."""
    L = N.Ledger("", 2, 256, True)
    nid = L.upsert_node("n0", synthetic_mi355x(8).ledger_devices(False), synthetic_mi355x(8).ledger_topo())
    live = set()
    for add, k in ops:
        key = f"p{k}"
        if add and key not in live:
            if L.reserve(nid, key, [(0, 0)], BIN)[0] == N.OK:
                live.add(key)
        elif not add and key in live:
            assert L.release(key) == N.OK
            live.discard(key)
    for k in range(200):
        key = f"p{k}"
        assert (L.lookup(key) is not None) == (key in live), key
    assert L.holds_any(sorted(live)) == bool(live) and L.n_pods == len(live)


# ----------------------------------------------------------------------------- memo re-validation
_share = st.tuples(st.sampled_from([5, 10, 25, 50, 100]), st.sampled_from([0, 0, 8192, 32768, 100 * 1024]),
                   st.sampled_from([0, 0, 1]))


@settings(max_examples=120, deadline=None)
@given(st.lists(st.tuples(st.sampled_from(["reserve", "reserve", "reserve", "release", "hot", "health", "reup"]),
                          _share, st.integers(0, 3), st.integers(0, 63)), min_size=5, max_size=80),
       st.lists(_share, min_size=1, max_size=4), st.sampled_from(["SPX", "CPX", "QPX"]),
       st.sampled_from([N.Policy.BINPACK, N.Policy.SPREAD]), st.booleans())
def test_memo_revalidation_agrees_with_a_fresh_choose(ops, probes, mode, policy, hbm):
    """assume_many (the front door's filter path) keeps a per-thread memo of each node's answer
    and, when the node changed, re-validates it against the devices the changes touched
    (Ledger::changed_since + alloc revalidate) instead of re-running choose(). Whatever the
    history of reserves, releases, health and HBM-activity flips, its (rc, score) per node is
    what a fresh choose() on the node's current state gives (the plan cache cleared)."""
    t = synthetic_mi355x(2, mode)
    L, ids = ledger_with(t, 4, track_hbm=hbm)
    o = N.Options(policy)
    live = []
    N.io_tally_reset()
    N.io_tally_enable(True)   # (the timers only; the paths are the same either way)
    try:
        for k, (op, d, node, dev) in enumerate(ops):
            nid = ids[node]
            if op == "reserve":
                if L.reserve(nid, f"p{k}", [d], o)[0] == N.OK:
                    live.append(f"p{k}")
            elif op == "release" and live:
                L.release(live.pop(dev % len(live)))
            elif op == "hot":
                L.set_mem_hot(nid, dev % len(t.devices), bool(k % 2))
            elif op == "health":
                L.set_health(nid, dev % len(t.devices), dev % 5 != 0)
            elif op == "reup":   # the node registered again (every device marked changed)
                assert L.upsert_node(f"n{node}", t.ledger_devices(hbm), t.ledger_topo()) == nid
            for p in probes:
                rcs, scores = L.assume_many(ids, [p], o)
                dh = N.demand_hash([p])
                # the plan each node's answer was cached with (by the memo path: the device too)
                plans = {nid2: [pl for h, _, rc_, pl, _ in L.cached_plans(nid2) if h == dh and rc_ == N.OK]
                         for nid2 in ids}
                L.clear_cache()
                for nid2, rc, sc in zip(ids, rcs, scores):
                    rc2, plan2, sc2 = L.assume(nid2, [p], o)
                    assert (rc, sc if rc == N.OK else 0) == (rc2, sc2 if rc2 == N.OK else 0), (k, op, p, nid2)
                    if rc == N.OK and plans[nid2]:
                        assert plans[nid2][0] == plan2, (k, op, p, nid2)
                L.clear_cache()
    finally:
        N.io_tally_enable(False)


def test_memo_revalidation_skips_most_recomputation_on_a_binpack_burst():
    """A burst like the bench's: 1-container pods of a dozen shapes reserved one after another
    on 64 nodes, every pod's filter over all nodes. Once each shape has been seen (the first
    filter of a shape computes every node), a node that changed is answered from its memo entry
    and the devices the change touched, not by choose() (5.7 plan computations a
    pod; at most 2 wanted)."""
    t = synthetic_mi355x(8)
    L = N.Ledger("", 64, 4096, True)
    ids = [L.upsert_node(f"n{i}", t.ledger_devices(True), t.ledger_topo()) for i in range(64)]
    o = N.Options(N.Policy.BINPACK)
    rng = random.Random(5)
    shapes = [(p, m) for p in (10, 25, 50) for m in (8192, 16384, 32768, 65536)]
    N.io_tally_enable(True)
    try:
        for k in range(700):
            if k == 100:
                N.io_tally_reset()
            d = [rng.choice(shapes)]
            rcs, scores = L.assume_many(ids, d, o)
            best = max((s, -i) for i, (rc, s) in enumerate(zip(rcs, scores)) if rc == N.OK)
            assert L.reserve(ids[-best[1]], f"p{k}", d, o)[0] == N.OK
        tally = N.io_tally()
    finally:
        N.io_tally_enable(False)
    # full placement computations (the general choose() and the one-share fast scan) against
    # answers re-validated from the memo and the changed devices alone
    full = tally.get("ledger_choose", (0, 0))[0] + tally.get("ledger_scan", (0, 0))[0]
    reval = tally.get("ledger_revalidate", (0, 0))[0]
    assert reval > 0 and full / 600 <= 2.0, (full, reval, tally)
