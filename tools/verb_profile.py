"""Native filter / priorities cost per request, as in the bench's bursts (64 SPX nodes, a
1000-pod stream of {10,25,50} % x {8..64} GiB, every bind changing one node's generation so the
next verb recomputes that node's plan). Runs the verbs in-process (Frontend.time_verb, no
socket), so the numbers are the verbs' own work.

    python tools/verb_profile.py [--nodes 64] [--pods 1000] [--nominate]
"""
from __future__ import annotations

import argparse
import json
import statistics
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))


def main(argv=None) -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--nodes", type=int, default=64)
    ap.add_argument("--pods", type=int, default=1000)
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--nominate", action="store_true")
    ap.add_argument("--sample", action="store_true",
                    help="send kube-scheduler's node sample (numFeasibleNodesToFind from a rotating start) "
                         "instead of every node")
    a = ap.parse_args(argv)

    from nanogpu import _native as N
    from nanogpu.k8s import podutil as pu
    from nanogpu.sim import workload as W
    from nanogpu.topology.model import synthetic_mi355x

    t = synthetic_mi355x(8)
    names = [f"mi355x-{i:03d}" for i in range(a.nodes)]
    out = {"filter_us": [], "priorities_us": []}
    for rnd in range(a.rounds):
        L = N.Ledger("", max(1024, a.nodes), 65536, True)
        ids = [L.upsert_node(n, t.ledger_devices(True), t.ledger_topo()) for n in names]
        fe = N.Frontend(L, "127.0.0.1", 0, 1)
        opts = N.Options(N.Policy.BINPACK)
        fe.set_options(opts, False, a.nominate)
        fl, pr = [], []
        from nanogpu.sim.kubescore import KubeScoring

        ks = KubeScoring()
        for spec in W.burst_specs(rnd, a.pods):
            pod = W.make_pod(spec, f"p{spec.key}", "bench", f"uid-{rnd}-{spec.key}")
            sent = [names[i] for i in ks.feasible(len(names), lambda i: True)] if a.sample else names
            body = json.dumps({"Pod": pod, "Nodes": None, "NodeNames": sent}, separators=(",", ":")).encode()
            ok, dt, resp = fe.time_verb(body, False, 1)
            assert ok
            fl.append(dt)
            fit = json.loads(resp)["NodeNames"]
            ok, dt, resp = fe.time_verb(body, True, 1)
            pr.append(dt)
            if fit:
                scores = json.loads(resp)
                best = max(scores, key=lambda h: h["Score"])["Host"]
                rc, _ = L.reserve(ids[names.index(best)], pod["metadata"]["uid"], pu.pod_demand(pod), opts)
                L.commit(pod["metadata"]["uid"])
        fe.stop()
        out["filter_us"].append(1e6 * statistics.mean(fl))
        out["priorities_us"].append(1e6 * statistics.mean(pr))
    print(json.dumps({k: [round(x, 2) for x in v] for k, v in out.items()}))
    return 0


if __name__ == "__main__":
    sys.exit(main())
