"""kube-scheduler extender wire format (k8s.io/kube-scheduler/extender/v1, v0.18).

The Go structs have no json tags, so keys are the capitalised field names on output and
Go's decoder matches them case-insensitively on input [ext]. Reference use sites:
routes.go:50-51 (ExtenderArgs/ExtenderFilterResult), :99-100 (HostPriorityList),
:133-134 (ExtenderBindingArgs/Result); predicate.go:34-38; priority.go:30-38.
"""
from __future__ import annotations

from typing import Any


def field(obj: dict, name: str, default: Any = None) -> Any:
    """Case-insensitive key lookup (Go encoding/json semantics)."""
    if not isinstance(obj, dict):
        return default
    if name in obj:
        return obj[name]
    low = name.lower()
    for k, v in obj.items():
        if k.lower() == low:
            return v
    return default


class ExtenderArgs:
    __slots__ = ("pod", "nodes", "node_names")

    def __init__(self, pod: dict | None, nodes: list[dict] | None, node_names: list[str] | None):
        self.pod = pod
        self.nodes = nodes
        self.node_names = node_names

    @classmethod
    def decode(cls, body: Any) -> "ExtenderArgs":
        if not isinstance(body, dict):
            raise ValueError("ExtenderArgs must be a JSON object")
        pod = field(body, "Pod")
        nodes = field(body, "Nodes")
        names = field(body, "NodeNames")
        node_items = None
        if isinstance(nodes, dict):
            node_items = nodes.get("items") or []
        if names is not None and not isinstance(names, list):
            raise ValueError("NodeNames must be a list")
        if pod is not None and not isinstance(pod, dict):
            raise ValueError("Pod must be an object")
        return cls(pod or {}, node_items, names)


def filter_result(node_names: list[str] | None, failed: dict[str, str], error: str = "",
                  nodes: list[dict] | None = None) -> dict:
    return {"Nodes": None if nodes is None else {"metadata": {}, "items": nodes},
            "NodeNames": node_names, "FailedNodes": failed, "Error": error}


def priority_list(hosts: list[str], scores: list[int]) -> list[dict]:
    return [{"Host": h, "Score": int(s)} for h, s in zip(hosts, scores)]


class BindingArgs:
    __slots__ = ("pod_name", "pod_namespace", "pod_uid", "node")

    def __init__(self, pod_name: str, pod_namespace: str, pod_uid: str, node: str):
        self.pod_name, self.pod_namespace, self.pod_uid, self.node = pod_name, pod_namespace, pod_uid, node

    @classmethod
    def decode(cls, body: Any) -> "BindingArgs":
        if not isinstance(body, dict):
            raise ValueError("ExtenderBindingArgs must be a JSON object")
        name, node = field(body, "PodName", ""), field(body, "Node", "")
        if not name or not node:
            raise ValueError("ExtenderBindingArgs requires PodName and Node")
        return cls(name, field(body, "PodNamespace", "") or "default", field(body, "PodUID", "") or "", node)


def binding_result(error: str = "") -> dict:
    return {"Error": error}


class PreemptionArgs:
    """ExtenderPreemptionArgs: the preemptor and, per candidate node, the victims
    kube-scheduler chose. With nodeCacheCapable it sends NodeNameToMetaVictims
    ({"Pods": [{"UID"}], "NumPDBViolations"}); otherwise NodeNameToVictims with full pods.
    Not in the reference (it registers no preemptVerb)."""
    __slots__ = ("pod", "victims", "pdb")

    def __init__(self, pod: dict, victims: dict[str, list[str]], pdb: dict[str, int]):
        self.pod, self.victims, self.pdb = pod, victims, pdb

    @classmethod
    def decode(cls, body: Any) -> "PreemptionArgs":
        if not isinstance(body, dict):
            raise ValueError("ExtenderPreemptionArgs must be a JSON object")
        pod = field(body, "Pod") or {}
        if not isinstance(pod, dict):
            raise ValueError("Pod must be an object")
        meta = field(body, "NodeNameToMetaVictims")
        full = field(body, "NodeNameToVictims")
        src = meta if isinstance(meta, dict) else full if isinstance(full, dict) else {}
        victims: dict[str, list[str]] = {}
        pdb: dict[str, int] = {}
        for node, v in src.items():
            pods = field(v, "Pods") or []
            uids = []
            for p in pods:
                if not isinstance(p, dict):
                    continue
                uid = field(p, "UID") if src is meta else ((p.get("metadata") or {}).get("uid"))
                if uid:
                    uids.append(str(uid))
            victims[node] = uids
            pdb[node] = int(field(v, "NumPDBViolations", 0) or 0)
        return cls(pod, victims, pdb)


def preemption_result(victims: dict[str, list[str]], pdb: dict[str, int]) -> dict:
    return {"NodeNameToMetaVictims": {n: {"Pods": [{"UID": u} for u in uids], "NumPDBViolations": pdb.get(n, 0)}
                                      for n, uids in victims.items()}}
