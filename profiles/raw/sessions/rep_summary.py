"""Summarise gpurun_out/rep/*.json (tools/gpu_bench_repeat.sh): value, phases per run."""
import glob
import json
import sys

root = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/rep"
for n in (1, 2, 4):
    rows = []
    for f in sorted(glob.glob(f"{root}/r{n}_*.json")):
        try:
            d = json.loads(open(f).read().strip().splitlines()[-1])
        except (ValueError, IndexError):
            continue
        ph = d.get("phase_ms_per_step_rank0") or {}
        rows.append((d["value"], d["ms_per_step"], d["p50_bind_ms"], d.get("value_rtt2ms"), d.get("value_inproc_api"),
                     {k: ph.get(k) for k in ("create_ms", "schedule_ms", "release_ms")}))
    for r in rows:
        print(n, *r)
