"""Pod / node helpers over raw Kubernetes JSON objects (dicts).

Reference: pkg/utils/pod.go:15-100, pkg/utils/node.go:8-14, pkg/dealer/allocate.go:29-62.
"""
from __future__ import annotations

import logging
from typing import Iterable

from .. import types as T
from .quantity import QuantityError, quantity_to_mib, quantity_value

log = logging.getLogger(__name__)

Demand = list  # list[tuple[int, int]]: (gpu-percent, hbm-mib) per container
Plan = list    # list[list[int]]: device indices per container ([-1] = no GPU)


def meta(obj: dict) -> dict:
    return obj.get("metadata") or {}


def pod_uid(pod: dict) -> str:
    return meta(pod).get("uid", "")


def pod_ns_name(pod: dict) -> tuple[str, str]:
    m = meta(pod)
    return m.get("namespace", "default"), m.get("name", "")


def pod_key(pod: dict) -> str:
    ns, name = pod_ns_name(pod)
    return f"{ns}/{name}"


def containers(pod: dict) -> list[dict]:
    return (pod.get("spec") or {}).get("containers") or []


def node_name_of(pod: dict) -> str:
    return (pod.get("spec") or {}).get("nodeName") or ""


def is_completed(pod: dict) -> bool:
    """pod.go:15-24: deletionTimestamp set, or phase Succeeded/Failed."""
    if meta(pod).get("deletionTimestamp"):
        return True
    return ((pod.get("status") or {}).get("phase")) in ("Succeeded", "Failed")


def is_terminated(pod: dict) -> bool:
    """Its containers have stopped: phase Succeeded or Failed. A pod with only a
    deletionTimestamp is still running through its grace period and holds its HBM and CUs;
    kube-scheduler keeps such pods in its node accounting too. The reference releases at the
    deletionTimestamp (is_completed); compat mode keeps that."""
    return ((pod.get("status") or {}).get("phase")) in ("Succeeded", "Failed")


def share_gone(pod: dict, compat: bool = False) -> bool:
    """The pod no longer uses its devices: terminated, or (reference, compat) terminating."""
    return is_completed(pod) if compat else is_terminated(pod)


def _limit(c: dict, res: str):
    lim = ((c.get("resources") or {}).get("limits")) or {}
    return lim.get(res)


def container_percent(c: dict) -> int:
    """pod.go:94-100: Quantity.Value() of limits[nano-gpu/gpu-percent], 0 when absent."""
    v = _limit(c, T.RESOURCE_GPU_PERCENT)
    if v is None:
        return 0
    try:
        return max(0, quantity_value(v))
    except QuantityError:
        log.warning("bad %s quantity %r", T.RESOURCE_GPU_PERCENT, v)
        return 0


def container_mib(c: dict) -> int:
    v = _limit(c, T.RESOURCE_GPU_MEMORY)
    if v is None:
        return 0
    try:
        return max(0, quantity_to_mib(v))
    except QuantityError:
        log.warning("bad %s quantity %r", T.RESOURCE_GPU_MEMORY, v)
        return 0


class Req(tuple):
    """One container's demand with flags: unpacks as (percent, MiB) like the plain tuples and
    carries `flags` (types.FLAG_MEM_BOUND) to the native core (bindings.cpp to_demand). Pods
    without flags keep plain tuples."""

    def __new__(cls, pct: int, mib: int, flags: int = 0):
        r = tuple.__new__(cls, (pct, mib))
        r.flags = flags
        return r

    def __repr__(self) -> str:
        return f"Req({self[0]}, {self[1]}, flags={self.flags})"


_DEMAND_CACHE: dict[str, Demand] = {}
_DEMAND_CACHE_OWNED: dict[str, Demand] = {}   # demands decided with the streaming-owner lookup
_DEMAND_CACHE_CAP = 65536


def controller_uid(pod: dict) -> str:
    """UID of the pod's controlling owner (the first ownerReferences entry with controller:
    true, else the first entry); "" when there is none (frontend.cpp controller_uid)."""
    refs = [r for r in (meta(pod).get("ownerReferences") or []) if isinstance(r, dict) and r.get("uid")]
    for r in refs:
        if r.get("controller") is True:
            return str(r["uid"])
    return str(refs[0]["uid"]) if refs else ""


def pod_demand(pod: dict, is_stream_owner=None) -> Demand:
    """allocate.go:54-62 (+ HBM MiB as the second dimension). Init containers are ignored.

    Container resources are immutable for the life of a pod UID, so the parsed demand is
    memoised per UID (filter, prioritize, bind and the controller all ask for it).
    `is_stream_owner(uid)` (the ledger's learned streaming owners): a pod with no
    nano-gpu/memory-bound annotation whose controlling owner was measured streaming HBM counts
    as memory-bound; "false" opts out. Decided at the pod's first sight, so its filter and its
    bind see the same demand."""
    uid = meta(pod).get("uid")
    cache = _DEMAND_CACHE if is_stream_owner is None else _DEMAND_CACHE_OWNED
    if uid:
        d = cache.get(uid)
        if d is not None:
            return d
    cs = containers(pod)
    mb = (meta(pod).get("annotations") or {}).get(T.ANNOTATION_MEMORY_BOUND)
    if mb is None and is_stream_owner is not None:
        owner = controller_uid(pod)
        if owner and is_stream_owner(owner):
            mb = "true"
    if mb:
        names = None if mb == "true" else {x.strip() for x in mb.split(",") if x.strip()}
        d = [Req(container_percent(c), container_mib(c),
                 T.FLAG_MEM_BOUND if names is None or c.get("name", "") in names else 0) for c in cs]
    else:
        d = [(container_percent(c), container_mib(c)) for c in cs]
    if uid:
        if len(cache) >= _DEMAND_CACHE_CAP:
            cache.clear()
        cache[uid] = d
    return d


# Containers one ledger record holds (native alloc.h kMaxContainers: one per plan index, 64;
# the ledger keeps 16 inline and spills larger pods into overflow records).
def _max_containers() -> int:
    from ..native import core

    return int(core().MAX_CONTAINERS)


LEDGER_MAX_CONTAINERS = _max_containers()


class TooManyGpuContainers(ValueError):
    pass


def ledger_view(demand: Demand) -> tuple[Demand, list[int] | None]:
    """The demand as the native ledger stores it, and the container each entry belongs to.

    The reference places any number of containers (allocate.go:54-62, rater.go:74-110); a
    ledger record holds 64 (every GPU container takes a plan index, and a node has at most
    64 devices' worth of them). A pod within that is passed as is (None: entries ARE containers,
    so compat placements stay bit-exact with the reference). A larger pod keeps only its
    GPU-requesting containers, which is placement-neutral in native mode (zero-demand
    containers take no device and sort last); more than 64 of those raises (the caller places
    such a pod with `wide_place` and accounts it with `fold_plan`)."""
    if len(demand) <= LEDGER_MAX_CONTAINERS:
        return demand, None
    idx = [i for i, d in enumerate(demand) if d[0] > 0 or d[1] > 0]
    if len(idx) > LEDGER_MAX_CONTAINERS:
        raise TooManyGpuContainers(f"pod requests GPUs in {len(idx)} containers; at most "
                                   f"{LEDGER_MAX_CONTAINERS} per pod are supported")
    return [demand[i] for i in idx], idx


def gpu_container_count(demand: Demand) -> int:
    return sum(1 for d in demand if d[0] > 0 or d[1] > 0)


def is_wide(demand: Demand) -> bool:
    """More GPU-requesting containers than one ledger record holds (wide_place / fold_plan)."""
    return len(demand) > LEDGER_MAX_CONTAINERS and gpu_container_count(demand) > LEDGER_MAX_CONTAINERS


def wide_place(devices: list[dict], demand: Demand, spread: bool = False) -> Plan | None:
    """Placement of a pod with more GPU containers than a ledger record holds (the reference
    places any count: allocate.go:54-62, rater.go:74-110). Containers largest first, as the
    reference's Choose does; a share goes to the fitting device with the least free percent
    (binpack: best fit) or the most (spread), HBM checked per memory pool; a k x 100 % container
    takes k devices with nothing used. Returns one entry per container ([-1]: no GPU), or None
    when the pod does not fit. The result is accounted through `fold_plan`."""
    free = [int(d["pct_free"]) if d.get("healthy", True) else -1 for d in devices]
    total = [int(d["pct_total"]) for d in devices]
    pool_of = [int(d.get("pool", -1)) if int(d.get("pool", -1)) >= 0 else -(k + 1) for k, d in enumerate(devices)]
    mib: dict[int, int] = {}
    for k, d in enumerate(devices):
        mib[pool_of[k]] = int(d["mib_free"]) if int(d.get("mib_total", 0)) > 0 else 1 << 62
    plan: Plan = [[-1] for _ in demand]
    order = sorted(range(len(demand)), key=lambda i: (demand[i][0], demand[i][1]), reverse=True)
    for i in order:
        pct, m = int(demand[i][0]), int(demand[i][1])
        if pct <= 0 and m <= 0:
            continue
        if pct >= 100 and pct % 100 == 0:
            k = pct // 100
            cand = [j for j in range(len(devices)) if free[j] == total[j] > 0]
            if len(cand) < k:
                return None
            take = cand[:k]
            for j in take:
                free[j] = 0
                mib[pool_of[j]] = 0 if pool_of[j] < 0 else mib[pool_of[j]]
            plan[i] = take
            continue
        fit = [j for j in range(len(devices)) if free[j] >= pct and mib[pool_of[j]] >= m]
        if not fit:
            return None
        j = (max if spread else min)(fit, key=lambda x: (free[x], -x if spread else x))
        free[j] -= pct
        mib[pool_of[j]] -= m
        if free[j] == 0 and pool_of[j] < 0:
            mib[pool_of[j]] = 0   # folded, a device filled to 100 % is held whole (fold_plan)
        plan[i] = [j]
    return plan


def fold_plan(demand: Demand, plan: Plan) -> tuple[Demand, Plan]:
    """A wide pod as one ledger record: one entry per device it uses, holding the sum of the
    shares placed there (a device its containers fill to 100 % is held whole, HBM included),
    so any container count fits the record's 64 entries (a node has at most 64 devices)."""
    per: dict[int, list[int]] = {}
    for k, idx in enumerate(plan):
        pct, m = int(demand[k][0]), int(demand[k][1])
        flags = getattr(demand[k], "flags", 0)
        if pct <= 0 and m <= 0:
            continue
        whole = pct >= 100 and pct % 100 == 0
        for j in idx:
            if j < 0:
                continue
            acc = per.setdefault(j, [0, 0, 0])
            acc[0] += 100 if whole else pct
            acc[1] += 0 if whole else m
            acc[2] |= flags
    folded: Demand = []
    fplan: Plan = []
    for j in sorted(per):
        pct, m, flags = per[j]
        folded.append(Req(min(pct, 100), m, flags) if flags else (min(pct, 100), m))
        fplan.append([j])
    return folded, fplan


def full_plan(plan: Plan, idx: list[int] | None, n_containers: int) -> Plan:
    """Ledger plan -> one entry per container ([-1]: no GPU)."""
    if idx is None:
        return plan
    out: Plan = [[-1] for _ in range(n_containers)]
    for k, i in enumerate(idx):
        out[i] = plan[k]
    return out


def ledger_plan(plan: Plan, idx: list[int] | None) -> Plan:
    """One entry per container -> the ledger's entries."""
    return plan if idx is None else [plan[i] for i in idx]


def is_gpu_sharing(pod: dict) -> bool:
    """pod.go:27-29 (Σ gpu-percent > 0), extended: an HBM-only request also counts."""
    return any(p > 0 or m > 0 for p, m in pod_demand(pod))


def is_assumed(pod: dict) -> bool:
    return (meta(pod).get("annotations") or {}).get(T.ANNOTATION_GPU_ASSUME) == "true"


def container_assignment(pod: dict, name: str) -> list[int] | None:
    """pod.go:85-92; comma-separated indices for whole-device (multi-GPU) containers."""
    val = (meta(pod).get("annotations") or {}).get(T.container_annotation(name))
    if val is None:
        return None
    try:
        return [int(x) for x in val.split(",") if x.strip() != ""]
    except ValueError:
        return None


def plan_from_pod(pod: dict) -> Plan | None:
    """allocate.go:29-50. A missing/garbled container index defaults to device 0 as in the
    reference (allocate.go:42-45); a zero-demand container keeps -1."""
    if not is_assumed(pod):
        return None
    plan: Plan = []
    for c in containers(pod):
        idx = container_assignment(pod, c.get("name", ""))
        if not idx:
            log.warning("pod %s: container %s has no assignment; defaulting to 0",
                        pod_key(pod), c.get("name"))
            idx = [0]
        plan.append(idx)
    return plan


def placement_patch(pod: dict, plan: Plan, extra: dict | None = None) -> dict:
    """Merge-patch body writing the reference annotation contract (pod.go:65-79)."""
    return placement_patch_names([c.get("name", "") for c in containers(pod)], plan, extra)


def placement_patch_names(names: list[str], plan: Plan, extra: dict | None = None) -> dict:
    return {"metadata": {"annotations": placement_annotations(names, plan, extra),
                         "labels": {T.LABEL_GPU_ASSUME: "true"}}}


def placement_annotations(names: list[str], plan: Plan, extra: dict | None = None) -> dict:
    """The reference's placement annotations (pod.go:65-79): what the Binding carries."""
    ann = {T.container_annotation(n): ",".join(str(i) for i in plan[k]) for k, n in enumerate(names)}
    ann[T.ANNOTATION_GPU_ASSUME] = "true"
    if extra:
        ann.update(extra)
    return ann


def label_patch(node: str) -> dict:
    """The bind's second write: the assume label only (the Binding carried the annotations),
    guarded by spec.nodeName. kube-apiserver refuses a pod patch that would change
    spec.nodeName (422), and restating an unchanged value is a no-op, so the label lands only
    on a pod that is bound to `node`: never on one bound elsewhere or still unbound."""
    return {"metadata": {"labels": {T.LABEL_GPU_ASSUME: "true"}}, "spec": {"nodeName": node}}


def apply_patch(obj: dict, patch: dict) -> dict:
    """RFC 7386 JSON merge patch (what the fake apiserver and our tests use)."""
    if not isinstance(patch, dict):
        return patch
    out = dict(obj) if isinstance(obj, dict) else {}
    for k, v in patch.items():
        if v is None:
            out.pop(k, None)
        elif isinstance(v, dict):
            out[k] = apply_patch(out.get(k) or {}, v)
        else:
            out[k] = v
    return out


def node_capacity_percent(node: dict) -> int:
    cap = ((node.get("status") or {}).get("capacity")) or {}
    v = cap.get(T.RESOURCE_GPU_PERCENT)
    if v is None:
        return 0
    try:
        return quantity_value(v)
    except QuantityError:
        return 0


def node_gpu_count(node: dict) -> int:
    """node.go:8-14: ⌊capacity[gpu-percent] / 100⌋."""
    return node_capacity_percent(node) // T.GPU_PERCENT_EACH_CARD


def node_labels(node: dict) -> dict:
    return meta(node).get("labels") or {}


def make_pod(name: str, containers_spec: Iterable[tuple[str, int] | tuple[str, int, int]],
             namespace: str = "default", uid: str | None = None,
             scheduler_name: str = "default-scheduler") -> dict:
    """Builds a pod object (tests, simulator, bench). containers_spec: (name, pct[, mib])."""
    import uuid

    cs = []
    for spec in containers_spec:
        cname, pct = spec[0], spec[1]
        mib = spec[2] if len(spec) > 2 else 0
        lim = {}
        if pct:
            lim[T.RESOURCE_GPU_PERCENT] = str(pct)
        if mib:
            lim[T.RESOURCE_GPU_MEMORY] = str(mib)
        cs.append({"name": cname, "image": "busybox", "resources": {"limits": lim, "requests": dict(lim)}})
    return {
        "apiVersion": "v1", "kind": "Pod",
        "metadata": {"name": name, "namespace": namespace, "uid": uid or str(uuid.uuid4()),
                     "annotations": {}, "labels": {}},
        "spec": {"containers": cs, "schedulerName": scheduler_name},
        "status": {"phase": "Pending"},
    }


def make_node(name: str, gpus: int, topology_json: str | None = None, labels: dict | None = None) -> dict:
    ann = {}
    if topology_json:
        ann[T.ANNOTATION_TOPOLOGY] = topology_json
    return {
        "apiVersion": "v1", "kind": "Node",
        "metadata": {"name": name, "labels": dict(labels or {}), "annotations": ann},
        "status": {"capacity": {T.RESOURCE_GPU_PERCENT: str(gpus * T.GPU_PERCENT_EACH_CARD)},
                   "allocatable": {T.RESOURCE_GPU_PERCENT: str(gpus * T.GPU_PERCENT_EACH_CARD)}},
    }
