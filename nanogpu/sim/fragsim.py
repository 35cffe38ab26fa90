"""Offline placement-quality simulator: replays the bench / BASELINE-config pod streams
through the native ledger (filter -> score -> arg-max with random tie-break -> reserve ->
commit), with no HTTP, so a policy change can be judged on frag% in seconds.

It models a serial kube-scheduler cycle that takes the extender's arg-max (what the bench
stand-in does). The reference algorithm runs in compat mode (bit-exact with the Go raters,
tests/test_parity.py) without the HBM dimension, as the reference has none.

    python -m nanogpu.sim.fragsim                       # every scenario, native vs reference
    python -m nanogpu.sim.fragsim --scenario headline
"""
from __future__ import annotations

import argparse
import json
import random
import statistics
import sys

from nanogpu.native import core
from nanogpu.sim import workload as W
from nanogpu.sim.kubescore import KubeScoring, spread_scores
from nanogpu.topology.model import synthetic_mi355x, synthetic_sriov_guest

N = core()
POL = {"binpack": N.Policy.BINPACK, "spread": N.Policy.SPREAD}


class Cluster:
    def __init__(self, topo, n_nodes: int, compat: bool, track_hbm: bool, policy: str = "binpack", seed: int = 0,
                 kube: KubeScoring | None = None):
        self.L = N.Ledger("", max(64, n_nodes), 1 << 16, True)
        self.ids = [self.L.upsert_node(f"n{i:03d}", topo.ledger_devices(track_hbm), topo.ledger_topo())
                    for i in range(n_nodes)]
        self.opts = N.Options(POL[policy], compat=compat)
        self.track_hbm = track_hbm
        self.rng = random.Random(seed)
        self.live: dict[str, int] = {}
        self.unsched = 0
        # kube-scheduler (None: the extender's arg-max over every node, random ties). With it:
        # NodeResourcesFit on the gpu-percent capacity, node sampling from a rotating start,
        # then LeastAllocated + BalancedAllocation + PodTopologySpread + 10 x extender
        self.kube = kube
        if kube is not None:
            kube.rng.seed(seed)
            kube.next_start = 0
        self.capacity = 100 * len(topo.devices)
        self.pct_used = {i: 0 for i in self.ids}
        self.requested = {i: (0, 0) for i in self.ids}
        self.pod_req: dict[str, tuple[int, int, int, int]] = {}   # uid -> (cpu, mem, pct, owner)
        self.owner_cnt: dict[tuple[int, int], int] = {}
        self.nodes_sent = 0
        self.cycles = 0

    def place(self, uid: str, demand: list, owner: int = -1) -> bool:
        if not self.track_hbm:
            demand = [(p, 0) for p, _ in demand]
        need = sum(p for p, _ in demand)
        if self.kube is not None:
            cand = [self.ids[k] for k in self.kube.feasible(
                len(self.ids), lambda k: self.pct_used[self.ids[k]] + need <= self.capacity)]
        else:
            cand = self.ids
        self.cycles += 1
        self.nodes_sent += len(cand)
        rcs = self.L.filter(cand, demand, self.opts) if cand else []
        fit = [i for i, rc in zip(cand, rcs) if rc == 0]
        if not fit:
            self.unsched += 1
            return False
        req = self.kube.pod_requests(demand) if self.kube is not None else (0, 0)
        if len(fit) == 1:
            host = fit[0]
        elif self.kube is not None:
            scores = self.L.score(fit, demand, self.opts)
            spread = spread_scores([self.owner_cnt.get((owner, i), 0) for i in fit], self.kube.spread_max_skew) \
                if owner >= 0 else [0] * len(fit)
            host = fit[self.kube.select([self.kube.total(s, self.requested[i], req, sp)
                                         for s, i, sp in zip(scores, fit, spread)])]
        else:
            scores = self.L.score(fit, demand, self.opts)
            best = max(scores)
            host = self.rng.choice([i for i, s in zip(fit, scores) if s == best])
        rc, _ = self.L.reserve(host, uid, demand, self.opts)
        assert rc == 0, rc
        self.L.commit(uid)
        self.live[uid] = host
        u = self.requested[host]
        self.requested[host] = (u[0] + req[0], u[1] + req[1])
        self.pct_used[host] += need
        if owner >= 0:
            self.owner_cnt[(owner, host)] = self.owner_cnt.get((owner, host), 0) + 1
        self.pod_req[uid] = (req[0], req[1], need, owner)
        return True

    def delete(self, uid: str) -> None:
        host = self.live.pop(uid, None)
        if host is not None:
            self.L.release(uid)
            cpu, mem, need, owner = self.pod_req.pop(uid, (0, 0, 0, -1))
            u = self.requested[host]
            self.requested[host] = (u[0] - cpu, u[1] - mem)
            self.pct_used[host] -= need
            if owner >= 0:
                self.owner_cnt[(owner, host)] -= 1

    def frag(self, min_req: int) -> dict:
        return self.L.frag(min_req)

    def hbm_overcommit(self) -> int:
        """MiB granted beyond a device's (or pool's) HBM, summed over the cluster."""
        over = 0
        for i in self.ids:
            for d in self.L.snapshot(i)["devices"]:
                over += max(0, -d["mib_free"])
        return over


def headline(compat: bool, steps: int = 20, nodes: int = 64, hbm_mib: int = 294_896, pods: int = 1000,
             step0: int = 0, kube: bool = False, **_) -> dict:
    """bench.py's workload: a 1000-pod burst of {10,25,50} % x {8,16,32,64} GiB on 64 SPX nodes,
    frag measured at peak occupancy, then the burst is deleted (bench.burst's RNG stream).
    The reference model sees the HBM requests too (the bench runs it with --compat)."""
    topo = synthetic_mi355x(8, "SPX", hbm_mib=hbm_mib)
    c = Cluster(topo, nodes, compat, track_hbm=True, seed=1, kube=KubeScoring() if kube else None)
    out = []
    for step in range(step0, step0 + steps):
        uids = []
        for spec in W.burst_specs(step, pods):
            uid = f"s{step}-{spec.key}"
            if c.place(uid, [(spec.pct, spec.gib * 1024)], spec.owner):
                uids.append(uid)
        out.append(c.frag(10))
        for u in uids:
            c.delete(u)
    return summarize(out, c)


def steady_state(compat: bool, steps: int = 20, nodes: int = 64, hbm_mib: int = 294_896, initial: int = 1000,
                 churn: float = 0.3, kube: bool = True, seed: int = 11, first: int | None = None, **_) -> dict:
    """Steady-state churn (nanogpu.sim.workload.steady): an initial fill, then each step deletes
    a random 30 % of the live pods and creates as many; frag measured after each step's creates,
    averaged over the steps from `first` on (default: the second half; the cluster is never
    emptied). bench.py's steady pass runs the same stream live."""
    topo = synthetic_mi355x(8, "SPX", hbm_mib=hbm_mib)
    c = Cluster(topo, nodes, compat, track_hbm=True, seed=seed, kube=KubeScoring() if kube else None)
    out = []
    for k, st in enumerate(W.steady(steps, initial, churn, seed)):
        for key in st.deletes:
            c.delete(f"k{key}")
        for spec in st.creates:
            c.place(f"k{spec.key}", [(spec.pct, spec.gib * 1024)], spec.owner)
        out.append(c.frag(10))
    return summarize(out[len(out) // 2 if first is None else first:], c)


def steady_protocol(lag: int, lead: int = 0, steps: int = 9, nodes: int = 64, hbm_mib: int = 294_896,
                    initial: int = 1000, churn: float = 0.3, seed: int = 11, first: int | None = None,
                    nominate: bool = True) -> dict:
    """The steady-churn stream through the extender's own verbs (the native front door's filter
    and priorities, with their nominations, Frontend.verb) and kube-scheduler's model, with every
    bind reserving `lag` scheduling cycles after its own: kube-scheduler starts the next pod's
    cycle without waiting for a bind (binding is asynchronous there), so its next filters can
    reach the extender before the bind does. In a deployment `lag` is set by timing (which worker
    the bind reaches, how soon its thread runs); here it is fixed, so the replay is exact and a
    policy's sensitivity to it is measured, not sampled. `lead`: Frontend.set_options(lead=...)
    (nanogpu.types.PRIORITY_LEAD). frag is averaged over the steps from `first` (default: the
    second half), as steady_state; also the nominations made / adopted / moved."""
    import collections
    from collections import deque

    from nanogpu.sim.driver import owner_index

    topo = synthetic_mi355x(8, "SPX", hbm_mib=hbm_mib)
    L = N.Ledger("", max(64, nodes), 1 << 16, True)
    names = [f"n{i:03d}" for i in range(nodes)]
    index = {n: i for i, n in enumerate(names)}
    ids = [L.upsert_node(n, topo.ledger_devices(True), topo.ledger_topo()) for n in names]
    opts = N.Options(N.Policy.BINPACK)
    fe = N.Frontend(L, "127.0.0.1", 0, 1)
    fe.set_options(opts, False, nominate, False, lead)
    kube = KubeScoring()
    kube.rng.seed(seed)
    cap = 100 * len(topo.devices)
    pct_used = [0] * nodes
    requested = [(0, 0)] * nodes
    owner_cnt: collections.Counter = collections.Counter()
    live: dict[int, tuple] = {}
    enc = json.JSONEncoder(separators=(",", ":"))
    out = []
    failed = [0]
    try:
        for k, st in enumerate(W.steady(steps, initial, churn, seed)):
            for key in st.deletes:
                rec = live.pop(key, None)
                if rec is None:
                    continue
                h, need, req, owner, uid = rec
                L.release(uid)
                pct_used[h] -= need
                requested[h] = (requested[h][0] - req[0], requested[h][1] - req[1])
                if owner >= 0:
                    owner_cnt[(owner, h)] -= 1
            pending: deque = deque()

            def bind_oldest() -> None:
                key, h, dem, uid = pending.popleft()
                rc, _ = L.reserve(ids[h], uid, dem, opts)
                if rc in (N.OK, N.OK_EXISTING):
                    L.commit(uid)
                    return
                # the node filled up under it: kube-scheduler's bind fails and the pod goes back
                # to its queue (counted here, not retried)
                failed[0] += 1
                _, need, req, owner, _ = live.pop(key)
                pct_used[h] -= need
                requested[h] = (requested[h][0] - req[0], requested[h][1] - req[1])
                if owner >= 0:
                    owner_cnt[(owner, h)] -= 1

            for spec in st.creates:
                pod = W.steady_pod(spec)   # bench.py's steady pods (same UIDs: same tie-breaks)
                uid = pod["metadata"]["uid"]
                dem = [(spec.pct, spec.gib * 1024)]
                req = kube.pod_requests(dem)
                owner = owner_index(pod)
                cand = kube.feasible(nodes, lambda i: pct_used[i] + spec.pct <= cap)
                text = enc.encode(pod)

                def verb(node_list: list[int], prio: bool):
                    body = '{"Pod":' + text + ',"Nodes":null,"NodeNames":' + enc.encode([names[i] for i in node_list]) + "}"
                    ok, ans = fe.verb(body.encode(), prio)
                    assert ok
                    return json.loads(ans)

                fits = [index[n] for n in verb(cand, False)["NodeNames"]] if cand else []
                if not fits:
                    continue
                host = fits[0]
                if len(fits) > 1:
                    sc = {index[e["Host"]]: e["Score"] for e in verb(fits, True)}
                    spread = spread_scores([owner_cnt.get((owner, i), 0) for i in fits], kube.spread_max_skew) \
                        if owner >= 0 else [0] * len(fits)
                    host = fits[kube.select([kube.total(sc[i], requested[i], req, sp) for i, sp in zip(fits, spread)])]
                pct_used[host] += spec.pct
                requested[host] = (requested[host][0] + req[0], requested[host][1] + req[1])
                if owner >= 0:
                    owner_cnt[(owner, host)] += 1
                live[spec.key] = (host, spec.pct, req, owner, uid)
                pending.append((spec.key, host, dem, uid))
                while len(pending) > lag:
                    bind_oldest()
            while pending:
                bind_oldest()
            out.append(L.frag(10))
    finally:
        fe.stop()
    res = summarize(out[len(out) // 2 if first is None else first:], None, 0)
    res["frag_pct_each_step"] = [round(f["frag_pct"], 3) for f in out]
    res["nominations"] = L.nomination_counts()
    res["bind_failures"] = failed[0]
    return res


def config5(compat: bool, rounds: int = 5, pods_n: int = 1000, nodes_n: int = 8, sriov: bool = False,
            reps: int = 10, kube: bool = False, **_) -> dict:
    """BASELINE config 5: CPX nodes (or SR-IOV guests), 1000-pod create/delete churn, binpack.
    The reference model has no HBM dimension (as in nanogpu.sim.configs)."""
    frs, unsched = [], 0
    for rep in range(reps):
        if sriov:
            topo, n = synthetic_sriov_guest(4), nodes_n * 2
        else:
            topo, n = synthetic_mi355x(8, "CPX"), nodes_n
        c = Cluster(topo, n, compat, track_hbm=not compat, seed=rep, kube=KubeScoring() if kube else None)
        rng = random.Random(5 + rep)
        live: list[str] = []
        for r in range(rounds):
            prng = random.Random(100 + r + 1000 * rep)
            for i in range(pods_n // rounds):
                uid = f"r{rep}-{r}-{i}"
                if c.place(uid, [(prng.choice((10, 25, 50, 100)), prng.choice((0, 8, 16, 32)) * 1024)]):
                    live.append(uid)
            frs.append(c.frag(10))
            rng.shuffle(live)
            half, live = live[: len(live) // 2], live[len(live) // 2:]
            for u in half:
                c.delete(u)
        unsched += c.unsched
    return summarize(frs, None, unsched)


def summarize(frs: list[dict], c: Cluster | None, unsched: int | None = None) -> dict:
    return {"frag_pct": round(statistics.mean(f["frag_pct"] for f in frs), 3),
            "frag_hbm_pct": round(statistics.mean(f["frag_mib"] for f in frs), 3),
            "stranded_pct": round(statistics.mean(f["stranded_pct"] for f in frs), 3),
            "unschedulable": c.unsched if c is not None else unsched,
            "hbm_overcommit_mib": c.hbm_overcommit() if c is not None else 0}


SCENARIOS = {
    "headline": headline,
    "steady": steady_state,
    "config5": config5,
    "config5_sriov": lambda compat, **kw: config5(compat, sriov=True, pods_n=125, **kw),
}


def run(names=None, kube: bool = False) -> dict:
    res = {}
    for name in names or SCENARIOS:
        fn = SCENARIOS[name]
        res[name] = {"native": fn(False, kube=kube), "reference_model": fn(True, kube=kube)}
    return res


def main(argv=None) -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--scenario", action="append", choices=sorted(SCENARIOS))
    ap.add_argument("--kube", action="store_true", help="kube-scheduler score combining (nanogpu.sim.kubescore)")
    args = ap.parse_args(argv)
    print(json.dumps(run(args.scenario, args.kube), indent=1))
    return 0


if __name__ == "__main__":
    sys.exit(main())
