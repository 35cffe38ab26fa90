"""Placement quality: native binpack against the reference algorithm on frag%.

The reference binpack (/root/reference/pkg/dealer/rater.go:59-110) scores a node by its
utilisation and takes the lowest-free device that fits. Native binpack scores the fit of the
plan and avoids turning fillable holes into dead ones (alloc.h SizeSet / Options::waste). These
tests replay reduced versions of the bench burst and BASELINE config 5 through both
(nanogpu.sim.fragsim) and pin that native is at least as good on percent and HBM
fragmentation, schedules as many pods, and never over-commits HBM.
"""
from nanogpu import _native as N
from nanogpu.sim import fragsim
from nanogpu.topology.model import synthetic_mi355x

BIN = N.Options(N.Policy.BINPACK)


def test_waste_table_marks_dead_holes_for_the_request_mix():
    o = N.Options(N.Policy.BINPACK, request_sizes=[10, 25, 50])
    assert o.request_sizes == [10, 25, 50]
    dead = {h for h, w in enumerate(o.waste) if w}
    assert 5 in dead and 15 in dead
    assert not {0, 10, 20, 25, 35, 45, 50, 75, 100} & dead
    assert o.waste[15] == 5 and o.waste[95] == 0
    assert all(w == 0 for w in N.Options(N.Policy.BINPACK).waste)


def _ledger(n_nodes=1):
    t = synthetic_mi355x(8)
    L = N.Ledger("", 16, 4096, True)
    return L, [L.upsert_node(f"n{i}", t.ledger_devices(True), t.ledger_topo()) for i in range(n_nodes)]


def test_binpack_keeps_a_25_hole_for_the_next_25():
    # GPU0 has a 25 % hole, GPU1 a 75 % hole. Best fit alone puts a 10 % share in the
    # 25 % hole (leaving a dead 15 %); with 10/25/50 requests common, binpack takes the 75 %.
    L, (nid,) = _ledger()
    assert L.allocate_plan(nid, "a", [(75, 0)], [[0]]) == N.OK
    assert L.allocate_plan(nid, "b", [(25, 0)], [[1]]) == N.OK
    for q in (10, 25, 50) * 20:
        L.note_request([(q, 0)])
    assert {10, 25, 50} <= set(L.learned_sizes())
    rc, plan, _ = L.assume(nid, [(10, 0)], BIN)
    assert rc == N.OK and plan == [[1]]
    # with learning off and no fixed sizes, plain best fit
    rc, plan, _ = L.assume(nid, [(10, 0)], N.Options(N.Policy.BINPACK, learn_sizes=False))
    assert plan == [[0]]
    # a 25 % share fills the 25 % hole exactly
    rc, plan, _ = L.assume(nid, [(25, 0)], BIN)
    assert plan == [[0]]


def test_binpack_node_score_prefers_the_tight_fit_over_the_busy_node():
    L, (busy, tight) = _ledger(2)
    assert L.reserve(busy, "x", [(100, 0)] * 6 + [(20, 0)], BIN)[0] == N.OK   # 6.2 of 8 GPUs used
    assert L.reserve(tight, "y", [(70, 0)], BIN)[0] == N.OK                   # one 30 % hole
    s_busy, s_tight = L.score([busy, tight], [(30, 0)], BIN)
    assert s_tight > s_busy          # the 30 % share closes tight's hole exactly
    assert s_tight == 100


def test_learned_sizes_decay_and_drop_rare_sizes():
    L, _ = _ledger()
    for _ in range(3000):
        L.note_request([(20, 0)])
    assert L.learned_sizes() == [20]
    for _ in range(4000):
        L.note_request([(30, 0)])
    assert L.learned_sizes() == [20, 30]
    for _ in range(12000):              # counts halve every ~2k requests
        L.note_request([(30, 0)])
    assert L.learned_sizes() == [30]    # 20 % decayed below 1 %


def test_headline_burst_native_beats_reference_frag():
    nat = fragsim.headline(False, steps=3)
    ref = fragsim.headline(True, steps=3)
    assert nat["unschedulable"] == ref["unschedulable"] == 0
    assert nat["frag_pct"] <= ref["frag_pct"] / 3, (nat, ref)
    assert nat["frag_hbm_pct"] <= ref["frag_hbm_pct"], (nat, ref)
    assert nat["hbm_overcommit_mib"] == 0


def test_config5_churn_native_beats_reference_frag():
    for sriov, pods in ((False, 1000), (True, 125)):
        nat = fragsim.config5(False, reps=3, sriov=sriov, pods_n=pods)
        ref = fragsim.config5(True, reps=3, sriov=sriov, pods_n=pods)
        assert nat["unschedulable"] <= ref["unschedulable"], (sriov, nat, ref)
        assert nat["frag_pct"] <= ref["frag_pct"], (sriov, nat, ref)
        assert nat["hbm_overcommit_mib"] == 0


def _stacked_streamers(mode: str, opts=BIN) -> int:
    """Streaming pods that share a device with another streaming pod, after a deployment of
    streaming replicas (owner "s") and one of compute-bound replicas (owner "c") scale up
    together on one 8-GPU node. The first streaming replica ran alone for one HBM-activity
    period. mode: "none" (no annotation, no learning: the reference's view), "learn" (the
    device counter marks the lone replica's device hot and the owner is learned), "declared"
    (every streaming pod annotated)."""
    from nanogpu.k8s.podutil import Req

    L, (nid,) = _ledger()
    truth: dict[int, int] = {}           # device -> streaming tenants (ground truth)

    def place(key: str, owner: str):
        streams = owner == "s"
        flagged = streams and (mode == "declared" or (mode == "learn" and L.is_stream_owner(owner)))
        d = [Req(25, 0, N.FLAG_MEM_BOUND)] if flagged else [(25, 0)]
        rc, plan = L.reserve(nid, key, d, opts)
        assert rc == N.OK
        L.commit(key)
        L.set_pod_owner(key, owner)
        (dev,) = plan[0]
        truth[dev] = truth.get(dev, 0) + (1 if streams else 0)

    def period():                        # the device counter: hot where a streamer runs
        for dev in range(8):
            L.set_mem_hot(nid, dev, truth.get(dev, 0) > 0)
        if mode == "learn":
            L.learn_stream_owners(True)

    place("s0", "s")
    period()
    for i in range(1, 8):             # 8 streaming replicas: one per GPU is possible
        place(f"s{i}", "s")
        place(f"c{i}", "c")
        if i % 4 == 0:
            period()
    return sum(n for n in truth.values() if n > 1)


def test_learned_streaming_owner_stops_streamers_stacking():
    """With the owner learned from its first replica's device counter, later replicas stop
    stacking on streaming devices, as when every pod is declared; without it, best fit packs
    the streamers together."""
    none, learn, declared = (_stacked_streamers(m) for m in ("none", "learn", "declared"))
    assert none >= 6
    assert learn == declared == 0
    assert _stacked_streamers("none", N.Options(N.Policy.BINPACK, compat=True)) == none   # the reference's


def test_steady_state_churn_native_frag_at_most_the_reference_models():
    """VERDICT r2 item 4 on a reduced stream: the cluster is filled once, then every step deletes
    30 % of the live pods and creates as many (nanogpu.sim.workload.steady), behind the
    kube-scheduler model. Native binpack's fragmentation stays at or below the reference
    algorithm's (compat mode) on the same stream."""
    from nanogpu.sim import fragsim

    kw = dict(steps=10, nodes=16, initial=250, kube=True)
    nat, ref = fragsim.steady_state(False, **kw), fragsim.steady_state(True, **kw)
    assert nat["unschedulable"] == 0 and ref["unschedulable"] == 0
    assert nat["frag_pct"] <= ref["frag_pct"], (nat, ref)
    assert nat["frag_hbm_pct"] <= ref["frag_hbm_pct"], (nat, ref)


def test_kube_scheduler_model_samples_nodes_and_spreads_owned_pods():
    """numFeasibleNodesToFind (all nodes below 100; 42 % of 1,000; at least 100) with a rotating
    start, and PodTopologySpread's normalised hostname score (fewer of the owner's pods on a
    node scores higher)."""
    from nanogpu import _native as NN
    from nanogpu.sim.kubescore import KubeScoring, num_feasible_nodes_to_find, spread_scores

    for n, want in ((64, 64), (99, 99), (100, 100), (200, 100), (1000, 420), (5000, 500), (10000, 500)):
        assert num_feasible_nodes_to_find(n) == want == NN.num_feasible_nodes_to_find(n)
    assert num_feasible_nodes_to_find(1000, 100) == 1000 and num_feasible_nodes_to_find(1000, 20) == 200
    k = KubeScoring()
    first = k.feasible(1000, lambda i: True)
    second = k.feasible(1000, lambda i: True)
    assert len(first) == len(second) == 420 and first[0] == 0 and second[0] == 420
    odd = k.feasible(1000, lambda i: i % 2 == 1)         # processed nodes include the failures
    assert len(odd) == 420 and odd[0] == 841 and k.next_start == (840 + 840) % 1000
    assert spread_scores([0, 0, 0]) == [100, 100, 100]
    s = spread_scores([3, 0, 1])
    assert s[1] == max(s) and s[0] == min(s)
