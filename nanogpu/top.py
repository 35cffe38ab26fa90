"""`python -m nanogpu.top [--url URL] [--watch S]`: per-node, per-device allocation table.

The reference exposes its cache only as a JSON dump (`POST /status`, routes.go:212-240) and
`PrintStatus` log lines (dealer.go:303-309). This reads the same `/status` body from a
running extender and prints what an operator asks first: which devices are in use, how
much compute and HBM is left, and where the free capacity is fragmented.
"""
from __future__ import annotations

import argparse
import json
import sys
import time
import urllib.request


def fetch(url: str, timeout: float = 5.0) -> dict:
    with urllib.request.urlopen(url.rstrip("/") + "/status", timeout=timeout) as r:
        return json.loads(r.read())


def _bar(used: int, total: int, width: int = 10) -> str:
    if total <= 0:
        return " " * width
    k = round(width * used / total)
    return "#" * k + "." * (width - k)


def render(status: dict, node_filter: str = "") -> str:
    rows = ["NODE                 DEV  GPU PART  USED%  COMPUTE     HBM-FREE-GiB  HEALTH"]
    tot_pct = free_pct = partial = 0
    for name in sorted(status):
        if node_filter and node_filter not in name:
            continue
        gpus = status[name].get("GPUs") or []
        seen_pools = set()
        for i, g in enumerate(gpus):
            total, free = int(g.get("PercentTotal", 100)), int(g.get("Percent", 0))
            used = total - free
            tot_pct += total
            free_pct += free
            if 0 < used < total:
                partial += free
            pool = g.get("MemoryPool", -1)
            mib_total = int(g.get("MemoryMiBTotal", 0))
            shared = pool >= 0 and pool in seen_pools
            seen_pools.add(pool)
            hbm = "-" if mib_total <= 0 else f"{g.get('MemoryMiB', 0) / 1024:7.1f}/{mib_total / 1024:.0f}" + (
                " (pool)" if shared else "")
            rows.append(f"{name[:20]:<20} {i:>3}  {g.get('GPU', i):>3} {g.get('Partition', 0):>4}  "
                        f"{100 * used // max(1, total):>4}%  [{_bar(used, total)}]  {hbm:<13} "
                        f"{'ok' if g.get('Healthy', True) else 'UNHEALTHY'}"
                        + (f"  streaming x{g.get('MemoryBoundTenants', 0)}" if g.get("MemoryBoundTenants") else "")
                        + ("  HBM-hot" if g.get("HBMHot") else ""))
    frag = 100.0 * partial / free_pct if free_pct else 0.0
    rows.append(f"\n{len(status)} nodes, {tot_pct // 100} devices, {free_pct / 100:.1f} device-equivalents free, "
                f"{frag:.1f}% of the free compute is on partly used devices")
    return "\n".join(rows)


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(prog="nanogpu.top", description=__doc__.splitlines()[0])
    ap.add_argument("--url", default="http://127.0.0.1:39999", help="extender base URL")
    ap.add_argument("--node", default="", help="only nodes whose name contains this")
    ap.add_argument("--watch", type=float, default=0.0, help="refresh every S seconds")
    ap.add_argument("--json", action="store_true", help="print the raw /status body")
    a = ap.parse_args(argv)
    while True:
        try:
            st = fetch(a.url)
        except OSError as e:
            print(f"nanogpu.top: {a.url}: {e}", file=sys.stderr)
            return 1
        out = json.dumps(st, indent=1) if a.json else render(st, a.node)
        if a.watch > 0:
            print("\033[H\033[J" + out, flush=True)
            time.sleep(a.watch)
        else:
            print(out)
            return 0


if __name__ == "__main__":
    sys.exit(main())
