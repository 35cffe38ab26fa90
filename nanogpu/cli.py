"""Command line: reference flag names and env vars, plus MI355X-native options.

Reference: cmd/main.go:63-73 (flags), :27, 93-99 (KUBECONFIG, PORT default 39999 when
not an int, THREADNESS default 1 when < 1 or not an int), :83-91 (priority switch:
anything but binpack/spread logs an error and exits).
"""
from __future__ import annotations

import argparse
import logging
import os

from . import types as T
from .app import Config
from .config.policy import parse_duration


def _int_env(name: str, default: int, minimum: int | None = None) -> int:
    try:
        v = int(os.environ.get(name, ""))
    except ValueError:
        return default
    if minimum is not None and v < minimum:
        return default
    return v


def _bool(s: str) -> bool:
    return str(s).lower() in ("1", "true", "yes", "on")


def build_parser() -> argparse.ArgumentParser:
    p = argparse.ArgumentParser("nano-gpu-scheduler", description="MI355X-native fine-grained GPU scheduler extender")
    # reference flags (Go flag package accepts -flag and --flag; so does this parser)
    p.add_argument("--priority", "-priority", default=T.PRIORITY_BINPACK, help="binpack|spread|random|firstfit")
    p.add_argument("--policyConfigPath", "-policyConfigPath", default=T.DEFAULT_POLICY_PATH)
    p.add_argument("--prometheusUrl", "-prometheusUrl", default=T.DEFAULT_PROMETHEUS_URL)
    p.add_argument("--instancePort", "-instancePort", default="9100")
    p.add_argument("--sync-period", "-sync-period", default="5s")
    p.add_argument("--isLoadSchedule", "-isLoadSchedule", default="false")
    p.add_argument("-v", "--v", type=int, default=0, help="log verbosity (klog-style)")
    # MI355X-native
    p.add_argument("--compat", action="store_true", help="reproduce reference placements bit for bit (Go 1.16)")
    p.add_argument("--score-normalize", action="store_true", help="map scores to kube-scheduler's [0,10]")
    p.add_argument("--topology-weight", type=float, default=1.0, help="xGMI/partition term weight")
    p.add_argument("--no-hbm", action="store_true", help="ignore the nano-gpu/gpu-memory dimension")
    p.add_argument("--request-sizes", default="",
                   help="comma-separated share sizes (percent) binpack keeps holes fillable for, e.g. 10,25,50")
    p.add_argument("--no-learn-sizes", action="store_true",
                   help="binpack uses only --request-sizes, not the sizes it sees requested")
    p.add_argument("--workers", type=int, default=1, help="SO_REUSEPORT worker processes sharing one ledger")
    p.add_argument("--ledger-path", default="", help="/dev/shm path of the shared ledger")
    p.add_argument("--max-nodes", type=int, default=4096)
    p.add_argument("--max-pods", type=int, default=131072)
    p.add_argument("--kube-api", default=None, help="API server URL (default: KUBECONFIG or in-cluster)")
    p.add_argument("--host", default="0.0.0.0")
    p.add_argument("--bind-verify-pod", action="store_true", help="GET the pod on every bind (reference behaviour)")
    p.add_argument("--native-bind-writes", action=argparse.BooleanOptionalAction, default=True,
                   help="the native front door's C++ threads do each bind's PATCH + binding POST + commit "
                        "(native/src/kubewriter.cpp); --no-native-bind-writes keeps them in Python")
    p.add_argument("--bind-writer-threads", type=int, default=16,
                   help="--bind-writer-mode threads: the number of blocking writer threads (8 binds in flight "
                        "each); evented / inline: the binds in flight when --api-max-inflight is 0 (x 8)")
    p.add_argument("--api-max-inflight", type=int, default=T.API_MAX_MUTATING_INFLIGHT,
                   help="kube-apiserver's --max-mutating-requests-inflight (its default 200). The native writer "
                        "starts each worker at 3/4 of it over --workers (a bind is its binding + label PATCH), "
                        "and on a 429 halves its window and re-sends after Retry-After (+1 per clean window); "
                        "0: --bind-writer-threads x 8 binds, no sizing")
    p.add_argument("--bind-writer-mode", choices=["inline", "evented", "frontdoor", "threads"], default="evented",
                   help="native bind writes: from each front-door worker's own epoll loop (inline), on one "
                        "epoll thread (evented), sent by the front-door worker with the answers read on one "
                        "epoll thread (frontdoor), or on blocking threads")
    p.add_argument("--bind-first", action="store_true",
                   help="front door: reserve the binds of an event batch before answering its filter / "
                        "priorities requests (the next pod's filter sees the pod just bound)")
    p.add_argument("--batch-labels", action="store_true",
                   help="native writer: send the label PATCHes of bound pods in batches instead of pipelining "
                        "each behind its binding (measured slower on MI355X hosts: profiles/ab_results_r04.md)")
    p.add_argument("--spin-nap", action="store_true",
                   help="front door: sleep the busy-poll window in the kernel (microsecond epoll timeout) "
                        "instead of polling it")
    p.add_argument("--spin-recv", action=argparse.BooleanOptionalAction, default=True,
                   help="front door: each busy-poll pass first tries a non-blocking recv on the connection the "
                        "last filter / priorities answer went out on, then epoll_wait(0) (--no-spin-recv: "
                        "epoll_wait(0) alone)")
    p.add_argument("--api-write-timeout", default="30s",
                   help="native bind writer: an API request unanswered this long fails over to the slow "
                        "path (a half-open connection never answers)")
    p.add_argument("--no-assume-label", action="store_true",
                   help="bind with the binding alone (it carries the placement annotations) instead of also "
                        "PATCHing the reference's nano-gpu/assume label: one API write per bind; for clusters "
                        "where nothing selects pods by that label (this project's agent selects by node)")
    p.add_argument("--no-native-pod-watch", action="store_true",
                   help="read the pod watch with aiohttp on the event loop instead of a native thread "
                        "(native/src/podwatch.cpp)")
    p.add_argument("--reservation-ttl", default="60s")
    p.add_argument("--no-nominate", action="store_true",
                   help="priorities do not tentatively reserve the top-scored node")
    p.add_argument("--nomination-ttl", default="5s", help="release a nomination no bind adopted after this")
    p.add_argument("--decisive-filter", action="store_true",
                   help="filter answers only the node priorities would rank first (and nominates it): "
                        "kube-scheduler then skips scoring and the priorities call, one round trip a pod; "
                        "its own score plugins have no say (off: every fitting node, as the reference)")
    p.add_argument("--priority-lead", type=int, default=T.PRIORITY_LEAD,
                   help="priorities answer the nominated node this many points above every other fitting node "
                        "(normalised scores: 10 and 0), so kube-scheduler's own score plugins (about 800 points "
                        "between nodes at most, against 10 x the extender's score) bind the pod where the ledger "
                        "holds it; 0: raw scores, as the reference")
    p.add_argument("--fake-cluster", type=int, default=0, help="serve against N in-process fake MI355X nodes")
    p.add_argument("--fake-gpus-per-node", type=int, default=8)
    p.add_argument("--fake-partition", default="SPX", choices=["SPX", "DPX", "QPX", "CPX"])
    p.add_argument("--seed", type=int, default=0)
    p.add_argument("--frontend", default="native", choices=["native", "aiohttp"],
                   help="native: C++ epoll server answers filter/priorities without Python")
    p.add_argument("--frontend-threads", type=int, default=4)
    p.add_argument("--busy-poll-us", type=int, default=0,
                   help="native workers keep polling this long after an event (lower latency, more CPU)")
    p.add_argument("--lazy-label-answers", action="store_true",
                   help="native writer: a label PATCH's answer is read by a later pass of the writer's loop "
                        "instead of waking it (the connection's SO_RCVLOWAT raised once its binding answered)")
    p.add_argument("--busy-poll-prio-us", type=int, default=-1,
                   help="the polling window after a priorities answer (kube-scheduler then picks the host, "
                        "sends the bind and builds the next pod's filter); -1: --busy-poll-us, 0: sleep")
    p.add_argument("--leader-elect", action="store_true", help="active/standby replicas on a Lease")
    p.add_argument("--lease-name", default="nano-gpu-scheduler")
    p.add_argument("--lease-namespace", default=os.environ.get("POD_NAMESPACE", "kube-system"))
    p.add_argument("--identity", default=os.environ.get("POD_NAME", ""))
    p.add_argument("--cpu-affinity", default="none",
                   help="none | auto (each worker on its own L3 domain, nanogpu.affinity) | CPU list, e.g. 8-15")
    return p


def _sizes(text: str) -> list[int]:
    out = []
    for part in filter(None, (x.strip() for x in text.split(","))):
        v = int(part)
        if not 1 <= v <= 100:
            raise SystemExit(f"--request-sizes: {v} is not a percent of one device (1..100)")
        out.append(v)
    return out


def parse(argv: list[str] | None = None) -> Config:
    a = build_parser().parse_args(argv)
    if a.priority not in T.POLICIES:
        raise SystemExit(f"Priority algorithm {a.priority} is not supported")
    logging.basicConfig(level=logging.DEBUG if a.v >= 4 else logging.INFO if a.v >= 1 else logging.WARNING,
                        format="%(asctime)s %(levelname)s %(name)s: %(message)s")
    port = _int_env("PORT", T.DEFAULT_PORT)
    return Config(
        priority=a.priority, policy_config_path=a.policyConfigPath, prometheus_url=a.prometheusUrl,
        instance_port=a.instancePort, sync_period_s=parse_duration(a.sync_period),
        is_load_schedule=_bool(a.isLoadSchedule), port=port, host=a.host,
        threadness=_int_env("THREADNESS", 1, minimum=1), kubeconfig=os.environ.get("KUBECONFIG"),
        kube_api=a.kube_api, compat=a.compat, score_normalize=a.score_normalize,
        topology_weight=a.topology_weight, track_hbm=not a.no_hbm, workers=max(1, a.workers),
        ledger_path=a.ledger_path, max_nodes=a.max_nodes, max_pods=a.max_pods,
        verify_pod_on_bind=a.bind_verify_pod, native_bind_writes=a.native_bind_writes,
        bind_writer_threads=max(1, a.bind_writer_threads), api_max_inflight=max(0, a.api_max_inflight), bind_writer_mode=a.bind_writer_mode,
        native_pod_watch=not a.no_native_pod_watch, assume_label=not a.no_assume_label,
        api_write_timeout_s=parse_duration(a.api_write_timeout), bind_first=a.bind_first, spin_nap=a.spin_nap, spin_recv=a.spin_recv, batch_labels=a.batch_labels, reservation_ttl_s=parse_duration(a.reservation_ttl),
        nominate=not a.no_nominate, nomination_ttl_s=parse_duration(a.nomination_ttl),
        decisive_filter=a.decisive_filter, priority_lead=a.priority_lead,
        fake_cluster=a.fake_cluster, fake_gpus_per_node=a.fake_gpus_per_node, fake_partition=a.fake_partition,
        seed=a.seed, frontend=a.frontend, frontend_threads=max(1, a.frontend_threads), busy_poll_us=a.busy_poll_us,
        busy_poll_prio_us=a.busy_poll_prio_us, lazy_label_answers=a.lazy_label_answers,
        leader_elect=a.leader_elect, lease_name=a.lease_name, lease_namespace=a.lease_namespace, identity=a.identity,
        cpu_affinity=a.cpu_affinity, request_sizes=_sizes(a.request_sizes), learn_sizes=not a.no_learn_sizes)
