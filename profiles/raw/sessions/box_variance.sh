#!/bin/bash
# Back-to-back headline runs on one box (README "Run-to-run variance"): the host's CPU layout,
# then N runs of the driver's command, each with its full record in --json-out.
# usage: tools/box_variance.sh OUTDIR N [extra bench flags]
out=${1:-gpurun_out/var}; n=${2:-6}; shift 2
mkdir -p "$out"
lscpu > "$out/lscpu.txt" 2>&1
python - > "$out/host.json" <<'EOF'
import json, os, time
from nanogpu import affinity
a = affinity.cpu_snapshot(); time.sleep(1.0); b = affinity.cpu_snapshot()
busy = affinity.busy_between(a, b, list(b))
print(json.dumps({"cpu_count": os.cpu_count(), "allowed": len(os.sched_getaffinity(0)),
                  "l3_domains": affinity.l3_domains(), "busy_pct_1s": {c: round(100 * v, 1) for c, v in busy.items()}}))
EOF
for i in $(seq 1 "$n"); do
  timeout -k 10 240 python bench.py --gpus 1 --steps 20 --warmup 5 "$@" --json-out "$out/b$i.json" \
    > "$out/b$i.log" 2>&1 || exit $?
  tail -c 400 "$out/b$i.log"; echo
done
