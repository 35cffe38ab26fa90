"""The benchmark's pod streams, shared by bench.py (live, through the extender) and
nanogpu.sim.fragsim (offline replays of the same streams, native and reference algorithm).

Pods: gpu-percent {10, 25, 50} x HBM {8, 16, 32, 64} GiB, one container each. Three in five
belong to one of 16 ReplicaSets (ownerReferences + an `app` label), the rest are bare pods or
Jobs: kube-scheduler applies its system default PodTopologySpread constraints to the owned ones
(nanogpu/sim/kubescore.py), which is what makes its choice differ from the extender's top score.

Two streams:
  * burst(step): `total` pods created at once, all deleted after the step (the headline);
  * steady(): BASELINE config 5's create/delete churn at a steady state. An initial fill,
    then every step deletes a random `churn` share of the live pods and creates as many new
    ones, so the cluster is never emptied. Deletions are drawn from the pods created so far
    (not from where they were placed), so the stream is the same for every scheduler.
"""
from __future__ import annotations

import random
import uuid
from dataclasses import dataclass

SIZES = (10, 25, 50)
HBM_GIB = (8, 16, 32, 64)
N_REPLICASETS = 16


@dataclass(frozen=True)
class PodSpec:
    key: int          # unique within its stream
    pct: int
    gib: int
    owner: int        # ReplicaSet index, -1: none


def owner_of(i: int, step: int) -> int:
    return (i * 7 + step) % N_REPLICASETS if i % 5 < 3 else -1


def burst_specs(step: int, total: int, seed: int = 7) -> list[PodSpec]:
    """bench.py's burst for `step` (the RNG stream of rounds 1-2: sizes first, then HBM)."""
    rng = random.Random(seed * 1000003 + step)
    out = []
    for i in range(total):
        pct, gib = rng.choice(SIZES), rng.choice(HBM_GIB)
        out.append(PodSpec(i, pct, gib, owner_of(i, step)))
    return out


def rs_uid(k: int) -> str:
    return str(uuid.UUID(int=(0x5EED << 96) | k))


def owner_refs(k: int) -> list[dict]:
    return [{"apiVersion": "apps/v1", "kind": "ReplicaSet", "name": f"bench-rs-{k}", "uid": rs_uid(k),
             "controller": True, "blockOwnerDeletion": True}]


def make_pod(spec: PodSpec, name: str, namespace: str, uid: str) -> dict:
    from ..k8s import podutil as pu

    p = pu.make_pod(name, [("main", spec.pct, spec.gib * 1024)], namespace=namespace, uid=uid)
    if spec.owner >= 0:
        p["metadata"]["ownerReferences"] = owner_refs(spec.owner)
        p["metadata"]["labels"]["app"] = f"bench-rs-{spec.owner}"
    return p


STEADY_NAMESPACE = "bench-steady"


def steady_uid(key: int) -> str:
    """A steady-stream pod's UID: the same whichever worker or rank handles it, so a run with N
    extender workers replays exactly the stream one worker sees (the UID breaks ties at the top,
    frontend.cpp top_pick)."""
    return str(uuid.UUID(int=(0x57EAD << 96) | key))


def steady_pod(spec: PodSpec) -> dict:
    return make_pod(spec, f"k{spec.key}", STEADY_NAMESPACE, steady_uid(spec.key))


@dataclass
class SteadyStep:
    deletes: list[int]          # keys of pods created earlier
    creates: list[PodSpec]


def steady(steps: int, initial: int = 1000, churn: float = 0.3, seed: int = 11) -> list[SteadyStep]:
    """Step 0 creates `initial` pods; every later step deletes round(churn x live) of the live
    pods (uniformly at random) and creates as many."""
    rng = random.Random(seed)
    live: list[int] = []
    out = []
    nxt = 0

    def new(n: int, step: int) -> list[PodSpec]:
        nonlocal nxt
        specs = []
        for _ in range(n):
            pct, gib = rng.choice(SIZES), rng.choice(HBM_GIB)
            specs.append(PodSpec(nxt, pct, gib, owner_of(nxt, step)))
            nxt += 1
        return specs

    for step in range(steps):
        if step == 0:
            dels, creates = [], new(initial, 0)
        else:
            k = round(churn * len(live))
            idx = sorted(rng.sample(range(len(live)), k), reverse=True)
            dels = [live[j] for j in idx]
            for j in idx:
                live[j] = live[-1]
                live.pop()
            creates = new(k, step)
        live.extend(s.key for s in creates)
        out.append(SteadyStep(dels, creates))
    return out
