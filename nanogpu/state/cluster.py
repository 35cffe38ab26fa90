"""Cluster GPU state: node registry + pod ledger over the native core.

Reference: pkg/dealer/dealer.go (DealerImpl, 20-method Dealer interface :23-43) and
pkg/dealer/node.go (NodeInfo + PlanCache). Differences by design:
  * no global lock: the native ledger has per-node locks and per-node generations, and the
    plan cache is keyed by generation instead of being wiped on every filter (node.go:96-98);
  * bind is reserve -> (API I/O, no lock) -> commit | rollback (fixes D1/D2);
  * delete events release (fixes D3); completed pods are skipped at rebuild (fixes D14);
    terminating pods keep their share until they stop (compat: reference release at deletion);
  * G = 0 nodes are unfit instead of a divide-by-zero panic (fixes D6);
  * nodes re-register when capacity/topology change (fixes D20).
"""
from __future__ import annotations

import hashlib
import logging
import threading
import time
from collections import OrderedDict
from dataclasses import dataclass
from typing import Callable

from .. import types as T
from ..k8s import podutil as pu
from ..native import core
from ..topology.model import NodeTopology, from_node

log = logging.getLogger(__name__)
N = core()

POLICY_ENUM = {
    T.PRIORITY_BINPACK: N.Policy.BINPACK,
    T.PRIORITY_SPREAD: N.Policy.SPREAD,
    T.PRIORITY_RANDOM: N.Policy.RANDOM,
    T.PRIORITY_FIRSTFIT: N.Policy.FIRSTFIT,
}


class SchedulingError(Exception):
    pass


@dataclass
class NodeEntry:
    id: int
    name: str
    topology: NodeTopology
    fingerprint: str


def demand_hash_compat(demand) -> str:
    """Reference PlanCache key: sha256 of "(p0)(p1)..." truncated to 8 hex (allocate.go:64-75)."""
    s = "".join(f"({p})" for p, _ in demand)
    return hashlib.sha256(s.encode()).hexdigest()[:8]


class ClusterState:
    def __init__(self, policy: str = T.PRIORITY_BINPACK, compat: bool = False,
                 load_aware: bool = False, topo_weight: float = 1.0, seed: int = 0,
                 ledger_path: str = "", max_nodes: int = 4096, max_pods: int = 131072,
                 track_hbm: bool = True, node_source: Callable[[str], dict | None] | None = None,
                 score_normalize: bool = False, nominate: bool = True, request_sizes: list[int] | None = None,
                 learn_sizes: bool = True, decisive_filter: bool = False, priority_lead: int = T.PRIORITY_LEAD):
        self.ledger = N.Ledger(ledger_path, max_nodes, max_pods, True)
        self._nominate = bool(nominate)
        self._lead = max(0, int(priority_lead))
        self._decisive = bool(decisive_filter)
        self.track_hbm = track_hbm
        self._listeners: list[Callable[[], None]] = []
        self._score_normalize = bool(score_normalize)
        self.node_source = node_source
        self._nodes: dict[str, NodeEntry] = {}
        self._nodes_mu = threading.Lock()
        self._released: OrderedDict[str, None] = OrderedDict()   # reference ReleasedPodMap
        self._rejected: dict[str, str] = {}     # nodes the ledger cannot hold, with the reason
        self._pending_removal: dict[str, int] = {}   # deleted nodes whose slot still holds shares
        self._released_cap = 65536
        self._reaccount_wait: dict[str, dict] = {}   # uid -> pod waiting for its partner (reaccount)
        self.set_policy(policy, compat=compat, load_aware=load_aware, topo_weight=topo_weight, seed=seed,
                        request_sizes=request_sizes or [], learn_sizes=learn_sizes)

    # ------------------------------------------------------------------ policy
    def add_listener(self, fn: Callable[[], None]) -> None:
        """Called after every policy / option change (the native front door mirrors them)."""
        self._listeners.append(fn)

    def remove_listener(self, fn: Callable[[], None]) -> None:
        if fn in self._listeners:
            self._listeners.remove(fn)

    def _changed(self) -> None:
        for fn in list(self._listeners):
            fn()

    @property
    def score_normalize(self) -> bool:
        return self._score_normalize

    @score_normalize.setter
    def score_normalize(self, v: bool) -> None:
        self._score_normalize = bool(v)
        self._changed()

    @property
    def nominate(self) -> bool:
        """Priorities nominate the unique top-scored node (Ledger::nominate). Off in compat
        mode: the reference keeps no state between prioritize and bind."""
        return self._nominate and not self.options.compat

    @nominate.setter
    def nominate(self, v: bool) -> None:
        self._nominate = bool(v)
        self._changed()

    @property
    def priority_lead(self) -> int:
        """Priorities answer the nominated node this many points above every other fitting node
        (normalised scores: 10 and 0), so kube-scheduler's own score plugins do not move the pod
        off the devices the ledger holds for it (frontend.cpp, priorities). 0: off."""
        return self._lead

    @priority_lead.setter
    def priority_lead(self, v: int) -> None:
        self._lead = max(0, int(v))
        self._changed()

    @property
    def decisive_filter(self) -> bool:
        """Filter answers only the node priorities would rank first (and nominates it), so
        kube-scheduler, left one feasible node, skips scoring and the priorities call: one
        round trip a pod instead of two. Its own score plugins then have no say. Off in compat
        mode and for wide pods. Off by default (the reference's filter answers every fitting
        node)."""
        return self._decisive and not self.options.compat

    @decisive_filter.setter
    def decisive_filter(self, v: bool) -> None:
        self._decisive = bool(v)
        self._changed()

    def set_policy(self, policy: str, compat: bool | None = None, load_aware: bool | None = None,
                   topo_weight: float | None = None, seed: int | None = None,
                   request_sizes: list[int] | None = None, learn_sizes: bool | None = None) -> None:
        """`request_sizes` fixes share sizes (percent) binpack treats as common; with
        `learn_sizes` the ledger adds the sizes it sees requested (alloc.h SizeSet)."""
        if policy not in POLICY_ENUM:
            raise ValueError(f"Priority algorithm {policy} is not supported")
        old = getattr(self, "options", None)
        self.policy = policy
        self.options = N.Options(
            POLICY_ENUM[policy],
            compat=bool(compat if compat is not None else (old.compat if old else False)),
            load_aware=bool(load_aware if load_aware is not None else (old.load_aware if old else False)),
            topo_weight=float(topo_weight if topo_weight is not None else (old.topo_weight if old else 1.0)),
            seed=int(seed if seed is not None else (old.seed if old else 0)),
            request_sizes=list(request_sizes if request_sizes is not None else (old.request_sizes if old else [])),
            learn_sizes=bool(learn_sizes if learn_sizes is not None else (old.learn_sizes if old else True)))
        self._changed()

    # ------------------------------------------------------------------ nodes
    def register_node(self, node: dict) -> NodeEntry:
        """Registers/refreshes a Node object (capacity + `nano-gpu/topology` annotation)."""
        name = pu.meta(node).get("name", "")
        topo = from_node(node)
        devices = topo.ledger_devices(self.track_hbm)
        fp = hashlib.blake2b(repr((devices, topo.link_bw)).encode(), digest_size=8).hexdigest()
        with self._nodes_mu:
            cur = self._nodes.get(name)
            if cur and cur.fingerprint == fp:
                return cur
        nid = self.ledger.upsert_node(name, devices, topo.ledger_topo()) if devices else \
            self.ledger.upsert_node(name, [], None)
        entry = NodeEntry(nid, name, topo, fp)
        with self._nodes_mu:
            self._nodes[name] = entry
        return entry

    def try_register_node(self, node: dict) -> NodeEntry | None:
        """register_node for a node that may not fit a ledger slot (more than 64 schedulable
        devices, 16 physical GPUs): logged once, reported as the node's filter failure."""
        name = pu.meta(node).get("name", "")
        try:
            e = self.register_node(node)
        except ValueError as err:
            if self._rejected.get(name) != str(err):
                log.warning("node %s not schedulable: %s", name, err)
            self._rejected[name] = str(err)
            return None
        self._rejected.pop(name, None)
        return e

    def forget_node(self, name: str) -> bool:
        """A deleted Node: its ledger slot goes once nothing holds a share on it. Nominations
        there are dropped at once (nobody will bind to a deleted node); reservations and
        committed pods keep the slot until they are released, and `retry_removals` (the
        sweeper) finishes the removal then, so the slot is not left behind."""
        with self._nodes_mu:
            e = self._nodes.pop(name, None)
        if not e:
            return False
        if self._remove_slot(e.id):
            self._pending_removal.pop(name, None)
            return True
        self._pending_removal[name] = e.id
        return False

    def _remove_slot(self, node_id: int) -> bool:
        for rec in self.ledger.pods_on(node_id):
            if rec["state"] == "nominated":
                self.ledger.drop_nomination(rec["key"])
        return self.ledger.remove_node(node_id)

    def retry_removals(self) -> list[str]:
        """Deleted nodes whose slot could not go yet (pods held shares): removed now if they
        are empty; a node registered again under the same name meanwhile is left alone."""
        done = []
        for name, nid in list(self._pending_removal.items()):
            if name in self._nodes or self.ledger.node_name(nid) != name:
                self._pending_removal.pop(name, None)
                continue
            if self._remove_slot(nid):
                self._pending_removal.pop(name, None)
                done.append(name)
        return done

    def node_entry(self, name: str) -> NodeEntry | None:
        e = self._nodes.get(name)
        if e is not None:
            return e
        # another worker (shared ledger) may have registered it; otherwise ask the lister
        if self.node_source is not None:
            node = self.node_source(name)
            if node is not None:
                return self.try_register_node(node)
        nid = self.ledger.find_node(name)
        if nid >= 0:
            snap = self.ledger.snapshot(nid)
            topo = NodeTopology.from_dict({"devices": [{"gpu": d["gpu"], "part": d["part"], "cus": d["cus"],
                                                        "xcds": d["xcds"], "hbm_mib": d["mib_total"]}
                                                       for d in snap["devices"]],
                                           "gpus": [], "link_bw": snap["topo"]["link_bw"]})
            entry = NodeEntry(nid, name, topo, "shared")
            with self._nodes_mu:
                self._nodes[name] = entry
            return entry
        return None

    def node_ids(self, names: list[str]) -> list[int]:
        out = []
        for n in names:
            e = self.node_entry(n)
            out.append(e.id if e else -1)
        return out

    def pod_demand(self, pod: dict):
        """The pod's demand; an unannotated pod of a learned streaming owner is memory-bound."""
        return pu.pod_demand(pod, self.ledger.is_stream_owner)

    # ------------------------------------------------------------------ verbs
    def filter(self, pod: dict, node_names: list[str]) -> tuple[list[str], dict[str, str]]:
        """Reference Dealer.Assume (dealer.go:89-136) + Predicate.Handler (predicate.go:19-41)."""
        if self.nominate:
            self._drop_own_nomination(pod)
        full = self.pod_demand(pod)
        if pu.is_wide(full):
            return self._wide_filter(full, node_names)
        demand, _ = pu.ledger_view(full)
        ids = self.node_ids(node_names)
        rcs = self.ledger.filter(ids, demand, self.options)
        wants = self.nominate and pu.pod_uid(pod) and any(p > 0 or m > 0 for p, m in demand)
        if self.decisive_filter and any(rc == N.OK for rc in rcs):
            scores = self.ledger.score(ids, demand, self.options)
            pick = self._top_pick(pu.pod_uid(pod), scores, rcs)
            if wants:
                self.ledger.nominate(ids[pick], pu.pod_uid(pod), demand, self.options)
            rcs = [rc if rc != N.OK or k == pick else None for k, rc in enumerate(rcs)]
        elif wants and sum(1 for rc in rcs if rc == N.OK) == 1:
            # one fitting node: kube-scheduler binds it without a priorities call (frontend.cpp)
            self.ledger.nominate(ids[rcs.index(N.OK)], pu.pod_uid(pod), demand, self.options)
        ok, failed = [], {}
        for name, nid, rc in zip(node_names, ids, rcs):
            if rc is None:    # fits, not the decisive pick: neither answered nor failed
                continue
            if rc == N.OK:
                ok.append(name)
            elif nid < 0:
                failed[name] = (f"nano gpu scheduler get node failed: node {name}: {self._rejected[name]}"
                                if name in self._rejected else
                                f"nano gpu scheduler get node failed: node {name} not found")
            else:
                failed[name] = f"can't allocate {self._demand_str(demand)} on node {name}: {N.err_str(rc)}"
        return ok, failed

    def score(self, pod: dict, node_names: list[str]) -> list[int]:
        """Reference Dealer.Score (dealer.go:138-153); ScoreMin (0) for unknown/unfit nodes."""
        if self.nominate:
            self._drop_own_nomination(pod)
        full = self.pod_demand(pod)
        if pu.is_wide(full):
            return self._wide_scores(full, node_names)
        demand, _ = pu.ledger_view(full)
        ids = self.node_ids(node_names)
        scores = self.ledger.score(ids, demand, self.options)
        if self.nominate and scores:
            scores = self._nominate_best(pod, demand, ids, scores)
        if self.score_normalize and scores:
            scores = self._normalize(scores)
        return scores

    def _drop_own_nomination(self, pod: dict) -> None:
        uid = pu.pod_uid(pod)
        if uid:
            self.ledger.drop_nomination(uid)

    @staticmethod
    def _top_pick(uid: str, scores: list[int], rcs: list[int]) -> int:
        """frontend.cpp top_pick: the fitting node with the top score; a tie goes to the tied
        node (in the request's order) the pod's UID hash picks."""
        cand = [k for k, rc in enumerate(rcs) if rc == N.OK]
        best = max(scores[k] for k in cand)
        top = [k for k in cand if scores[k] == best]
        return top[N.Ledger.owner_hash(uid) % len(top)] if len(top) > 1 and uid else top[0]

    def _nominate_best(self, pod: dict, demand, ids: list[int], scores: list[int]) -> list[int]:
        """Same rule as the native front door (frontend.cpp, priorities): a unique best fitting
        node is nominated; a tie at the top is broken by one point, for the tied node (in the
        request's order) that the pod's UID hash picks, while the nomination margin is 0.
        Returns the scores to answer."""
        uid = pu.pod_uid(pod)
        fits = self.ledger.filter(ids, demand, self.options)
        cand = [(s, k) for k, (s, i, rc) in enumerate(zip(scores, ids, fits)) if rc == N.OK and i >= 0]
        if not cand or not uid:
            return scores
        best = max(s for s, _ in cand)
        top = [k for s, k in cand if s == best]
        rest = [s for s, _ in cand if s != best]
        margin = self.ledger.nomination_margin
        if len(top) > 1 and margin == 0:
            pick = top[N.Ledger.owner_hash(uid) % len(top)]
            scores = list(scores)
            scores[pick] += 1
            rest, top = [best], [pick]
            best += 1
        # the lead must survive kube-scheduler's own plugins (Ledger::nomination_margin)
        if (len(top) == 1 and (not rest or best - max(rest) >= margin)
                and any(p > 0 or m > 0 for p, m in demand)):
            self.ledger.nominate(ids[top[0]], uid, demand, self.options)
            if self._lead > 0 and rest:
                # the nominated node leads every other fitting node by `priority_lead`
                # (normalised: 10 and 0, _normalize maps 100 to 10)
                scores = list(scores)
                if self.score_normalize:
                    scores = [100 if k == top[0] else 0 for k in range(len(scores))]
                elif best - max(rest) < self._lead:
                    scores[top[0]] = max(rest) + self._lead
        return scores

    def _normalize(self, scores: list[int]) -> list[int]:
        """Maps to kube-scheduler's extender range [0, 10] (MaxExtenderPriority) [ext]."""
        if self.options.compat:
            lo, hi = min(scores), max(scores)
            if hi == lo:
                return [10 if hi > 0 else 0 for _ in scores]
            return [int(round(10 * (s - lo) / (hi - lo))) for s in scores]
        return [max(0, min(10, int(round(s / 10)))) for s in scores]

    def reserve(self, pod: dict, node_name: str) -> tuple[list[list[int]], bool]:
        """First half of bind: allocate on the ledger (node.go:70-84 + allocate.go:102-118).

        Returns (plan, fresh); fresh is False when the pod was already allocated on that
        node (a retried bind), in which case a later failure must not roll it back."""
        e = self.node_entry(node_name)
        if e is None:
            raise SchedulingError(f"node {node_name} not found")
        uid = pu.pod_uid(pod)
        full = self.pod_demand(pod)
        if pu.is_wide(full):
            return self._wide_reserve(e, uid, full)
        demand, idx = pu.ledger_view(full)
        rc, plan = self.ledger.reserve(e.id, uid, demand, self.options)
        if rc not in (N.OK, N.OK_EXISTING):
            raise self.reserve_error(demand, node_name, rc)
        owner = pu.controller_uid(pod)
        if owner:                     # what the streaming-owner learner reads (learn_stream_owners)
            self.ledger.set_pod_owner(uid, owner)
        return pu.full_plan(plan, idx, len(full)), rc == N.OK

    # ------------------------------------------------------------------ wide pods
    # More GPU containers than a ledger record holds (pu.is_wide): placed in Python on the
    # node's snapshot (pu.wide_place), accounted as one record folded per device (pu.fold_plan)
    # with the per-container plan beside it in the shared ledger (Ledger::reserve_wide), so any
    # worker process answers a retried bind with the plan the ledger holds (reference
    # dealer.go:200 keeps every pod's plan in its dealer; allocate.go:29-50).
    # The native front door hands such pods to this path (its demand parser stops at 64).
    def _wide_plan(self, nid: int, full) -> list | None:
        if nid < 0:
            return None
        snap = self.ledger.snapshot(nid)
        if self.options.compat and self.policy in ("binpack", "spread"):
            # the reference's Choose places any container count (rater.go:74-163): its executable
            # spec (nanogpu.sim.oracle, bit-exact with Go 1.16's sort) on the node's percents
            from ..sim import oracle

            gpus = [oracle.G(int(d["pct_free"]) if d.get("healthy", True) else -1, int(d["pct_total"]))
                    for d in snap["devices"]]
            idx = oracle.choose(gpus, [int(pct) for pct, _ in full], spread=self.policy == "spread")
            return None if idx is None else [[i] for i in idx]
        return pu.wide_place(snap["devices"], full, spread=self.policy == "spread")

    def _wide_filter(self, full, node_names: list[str]) -> tuple[list[str], dict[str, str]]:
        ok, failed = [], {}
        n = pu.gpu_container_count(full)
        for name, nid in zip(node_names, self.node_ids(node_names)):
            if nid < 0:
                failed[name] = f"nano gpu scheduler get node failed: node {name} not found"
            elif self._wide_plan(nid, full) is None:
                failed[name] = f"can't allocate {n} GPU containers on node {name}: {N.err_str(N.ERR_NO_FIT)}"
            else:
                ok.append(name)
        return ok, failed

    def _wide_scores(self, full, node_names: list[str]) -> list[int]:
        """Utilisation after the placement (binpack: fuller is better; spread: emptier); in
        compat mode the reference's Rate on the node as it is (rater.go:59-70, 113-123)."""
        out = []
        if self.options.compat and self.policy in ("binpack", "spread"):
            from ..sim import oracle

            for nid in self.node_ids(node_names):
                if nid < 0 or self._wide_plan(nid, full) is None:
                    out.append(0)
                    continue
                gpus = [oracle.G(int(d["pct_free"]), int(d["pct_total"])) for d in self.ledger.snapshot(nid)["devices"]]
                out.append((oracle.rate_spread if self.policy == "spread" else oracle.rate_binpack)(gpus))
            return self._normalize(out) if self.score_normalize and out else out
        for nid in self.node_ids(node_names):
            plan = self._wide_plan(nid, full)
            if plan is None:
                out.append(0)
                continue
            devs = self.ledger.snapshot(nid)["devices"]
            total = sum(int(d["pct_total"]) for d in devs) or 1
            used = total - sum(int(d["pct_free"]) for d in devs)
            folded, _ = pu.fold_plan(full, plan)
            u = int(100 * (used + sum(p for p, _ in folded)) / total)
            out.append(100 - u if self.policy == "spread" else u)
        if self.score_normalize and out:
            out = self._normalize(out)
        return out

    def _wide_reserve(self, e, uid: str, full) -> tuple[list[list[int]], bool]:
        rec = self.ledger.lookup(uid)
        if rec is not None and rec["state"] != "nominated":
            # a retried bind (on this worker or another): the plan the ledger holds, never a new one
            return self._wide_held(e, uid, rec), False
        plan = self._wide_plan(e.id, full)
        if plan is None:
            raise SchedulingError(f"assume {pu.gpu_container_count(full)} GPU containers on {e.name} failed: "
                                  f"{N.err_str(N.ERR_NO_FIT)}")
        folded, fplan = pu.fold_plan(full, plan)
        rc, held = self.ledger.reserve_wide(e.id, uid, folded, fplan, plan, False)
        if rc == N.OK_EXISTING:          # another worker reserved it meanwhile
            return self._wide_held(e, uid, self.ledger.lookup(uid), held), False
        if rc != N.OK:
            raise self.reserve_error(folded, e.name, rc)
        return plan, True

    def _wide_held(self, e, uid: str, rec: dict | None, held: list | None = None) -> list[list[int]]:
        if rec is None or rec["node"] != e.id:
            raise SchedulingError(f"pod {uid} is already placed on another node")
        held = held if held is not None else self.ledger.wide_plan(uid)
        if held is None:
            raise SchedulingError(f"pod {uid} is reserved on {e.name} without its per-container plan")
        return [list(x) for x in held]

    def reserve_error(self, demand, node_name: str, rc: int) -> SchedulingError:
        return SchedulingError(f"assume {self._demand_str(demand)} on {node_name} failed: {N.err_str(rc)}")

    def commit(self, uid: str) -> None:
        self.ledger.commit(uid)

    def rollback(self, uid: str) -> None:
        self.ledger.release(uid)

    def allocate_existing(self, pod: dict, quiet: bool = False) -> bool:
        """Account a pod placed by someone else / found at restart (dealer.go:205-228)."""
        node = pu.node_name_of(pod)
        if not node:
            return False
        plan = pu.plan_from_pod(pod)
        if plan is None:
            return False
        e = self.node_entry(node)
        if e is None:
            log.warning("allocate %s: node %s unknown", pu.pod_key(pod), node)
            return False
        full = self.pod_demand(pod)
        if len(plan) != len(full):
            log.warning("allocate %s: %d assignments for %d containers", pu.pod_key(pod), len(plan), len(full))
            return False
        if pu.is_wide(full):
            demand, lplan = pu.fold_plan(full, plan)
            rc, _ = self.ledger.reserve_wide(e.id, pu.pod_uid(pod), demand, lplan, plan, True)
            rc = N.OK if rc == N.OK_EXISTING else rc   # already accounted (dealer.go:214-216)
        else:
            demand, idx = pu.ledger_view(full)
            lplan = pu.ledger_plan(plan, idx)
            rc = self.ledger.allocate_plan(e.id, pu.pod_uid(pod), demand, lplan, True)
        if rc != N.OK:
            if not quiet:
                log.warning("allocate %s on %s failed: %s", pu.pod_key(pod), node, N.err_str(rc))
            return False
        owner = pu.controller_uid(pod)
        if owner:
            self.ledger.set_pod_owner(pu.pod_uid(pod), owner)
        return True

    def reaccount(self, pod: dict) -> bool:
        """A bound pod whose placement annotations changed (the node agent's reconciliation
        with kubelet): its share moves to the annotated devices. True if it moved.

        Swapped containers are re-accounted one at a time, so the first one's new devices are
        often still held by its partner: its share is dropped and it waits (`_reaccount_wait`)
        until the partner has moved; every move retries the waiting ones."""
        uid = pu.pod_uid(pod)
        rec = self.ledger.lookup(uid)
        plan = pu.plan_from_pod(pod)
        if rec is None and uid in self._reaccount_wait:
            self._reaccount_wait[uid] = pod
            return self._retry_reaccount()
        if rec is None or plan is None or rec["state"] != "committed":
            return False
        full = self.pod_demand(pod)
        if pu.is_wide(full):
            _, lplan = pu.fold_plan(full, plan) if len(plan) == len(full) else (None, None)
        else:
            _, idx = pu.ledger_view(full)
            lplan = pu.ledger_plan(plan, idx)
        if lplan is None or [list(x) for x in lplan] == [list(x) for x in rec["plan"]]:
            return False
        if self.ledger.drop_committed(uid) != N.OK:
            return False
        if not self.allocate_existing(pod, quiet=True):
            self._reaccount_wait[uid] = pod     # its new devices are still taken: wait
            return False
        self._retry_reaccount()
        return True

    def _retry_reaccount(self) -> bool:
        moved = False
        for uid, pod in list(self._reaccount_wait.items()):
            if self.allocate_existing(pod, quiet=True):
                del self._reaccount_wait[uid]
                moved = True
        return moved

    def forget_reaccount(self, uid: str) -> None:
        self._reaccount_wait.pop(uid, None)

    def release(self, pod: dict) -> bool:
        return self.release_uid(pu.pod_uid(pod))

    def release_uid(self, uid: str) -> bool:
        rc = self.ledger.release(uid)
        if rc == N.OK:
            self._released[uid] = None
            if len(self._released) > self._released_cap:
                self._released.popitem(last=False)
            return True
        return False

    def reconcile(self, live_uids: list[str], before: float) -> list[str]:
        """After a pod LIST: releases committed shares recorded before `before` whose pod is
        not among `live_uids` (Ledger::reconcile). Returns the UIDs released."""
        gone = self.reconcile_native("\n".join(live_uids), before)
        self.note_released(gone)
        return gone

    def reconcile_native(self, joined_uids: str, before: float) -> list[str]:
        """The ledger half of `reconcile` (thread-safe, runs without the GIL: the pod
        controller calls it from an executor thread); `joined_uids` newline-separated."""
        return self.ledger.reconcile_joined(joined_uids, float(before))

    def note_released(self, uids: list[str]) -> None:
        for uid in uids:
            self._released[uid] = None
        while len(self._released) > self._released_cap:
            self._released.popitem(last=False)

    def known(self, uid: str) -> bool:
        return self.ledger.lookup(uid) is not None

    def released(self, uid: str) -> bool:
        return uid in self._released

    def forget(self, uid: str) -> None:
        self._released.pop(uid, None)

    def rebuild(self, pods: list[dict]) -> int:
        """Checkpoint/resume: the API server is the checkpoint (dealer.go:58-72, 279-299)."""
        n = 0
        for p in pods:
            if pu.is_assumed(p) and pu.node_name_of(p) and not pu.share_gone(p, self.options.compat):
                n += int(self.allocate_existing(p))
        return n

    def sweep_reservations(self, ttl_s: float) -> list[str]:
        """Releases reservations whose bind never committed (crashed worker, lost request)."""
        stale = self.ledger.expired_reservations(ttl_s)
        # only while still reserved: a bind may commit between the scan and the release
        return [uid for uid in stale if self.ledger.drop_reservation(uid) == N.OK]

    def sweep_nominations(self, ttl_s: float) -> list[str]:
        """Releases nominations no bind adopted (kube-scheduler chose another node, or the
        pod was never bound)."""
        stale = self.ledger.expired_nominations(ttl_s)
        # only while still nominated: a bind may adopt it between the scan and the release
        return [uid for uid in stale if self.ledger.drop_nomination(uid) == N.OK]

    # ------------------------------------------------------------------ telemetry
    def set_load(self, node_name: str, device: int, usage: float) -> bool:
        e = self._nodes.get(node_name)
        return bool(e) and self.ledger.set_load(e.id, device, float(usage)) == N.OK

    def set_mem_hot(self, node_name: str, device: int, hot: bool) -> bool:
        """Measured HBM activity above the threshold (telemetry): the device counts as
        holding a streaming tenant for memory-bound placement (alloc.h Device::mem_hot)."""
        e = self._nodes.get(node_name)
        return bool(e) and self.ledger.set_mem_hot(e.id, device, bool(hot)) == N.OK

    def set_mem_busy(self, node_name: str, device: int, activity: float) -> bool:
        """The averaged HBM activity (0..1) the streaming-owner learner reads (Device::mem_busy)."""
        e = self._nodes.get(node_name)
        return bool(e) and self.ledger.set_mem_busy(e.id, device, int(round(100 * activity))) == N.OK

    # ------------------------------------------------------------------ introspection
    def frag(self, min_request: int = 0) -> dict:
        return self.ledger.frag(min_request)

    def status(self) -> dict:
        """`/status` body in the reference's shape (NodeInfo JSON: routes.go:212-240)."""
        out = {}
        for name, e in list(self._nodes.items()):
            snap = self.ledger.snapshot(e.id)
            if snap is None:
                continue
            out[name] = {
                "Rater": {},
                "Name": name,
                "GPUs": [{"Percent": d["pct_free"], "PercentTotal": d["pct_total"],
                          "RemainLoad": d["remain_load"], "MemoryMiB": d["mib_free"],
                          "MemoryMiBTotal": d["mib_total"], "MemoryPool": d["pool"], "GPU": d["gpu"],
                          "Partition": d["part"],
                          "Healthy": d["healthy"],
                          # streaming tenants: declared (nano-gpu/memory-bound) and measured
                          "MemoryBoundTenants": d["mem_bound"], "HBMHot": d["mem_hot"],
                          "HBMActivityPct": d["mem_busy"]}
                         for d in snap["devices"]],
                "PlanCache": self._plan_cache(e.id),
                "Generation": snap["generation"],
            }
        return out

    def _plan_cache(self, node_id: int) -> dict:
        """This process's cached plans still valid for the node (the reference dumps
        NodeInfo.PlanCache, node.go:18-23, keyed by a demand hash). Keys are the native
        demand/options hashes; GPUIndexes holds each container's devices ([-1]: no GPU)."""
        out = {}
        for dh, oh, rc, plan, score in self.ledger.cached_plans(node_id):
            out[f"{dh:016x}/{oh:08x}"] = {"GPUIndexes": plan if rc == N.OK else [], "Score": score if rc == N.OK else 0,
                                          "Fits": rc == N.OK}
        return out

    @staticmethod
    def _demand_str(demand) -> str:
        return "".join(f"({p})" if not m else f"({p},{m}Mi)" for p, m in demand)


def now() -> float:
    return time.monotonic()
