#!/bin/bash
# Round-5 box session M: headline runs after the harness's per-step bookkeeping left the clock,
# with the gaps between steps. usage: tools/box_r05m.sh OUT
set -o pipefail
OUT="$1" REPS=4 tools/bench_arms.sh "" || exit $?
python - "$1" <<'PY'
import glob, json, sys
for f in sorted(glob.glob(sys.argv[1] + "/arm*.json")):
    d = json.load(open(f)); st = d["diagnostics"]["step_diag_rank0"]
    gaps = [round(1e3 * (st[k + 1]["t0"] - st[k]["t2"]), 2) for k in range(len(st) - 1)]
    print(f.split("/")[-1], d["value"], d["ms_per_step"], d["p50_bind_ms"], d["p99_bind_ms"], "gaps", max(gaps), "foreign", d.get("foreign_cpus_rank0"), d.get("foreign_cpus_apiserver"))
PY
