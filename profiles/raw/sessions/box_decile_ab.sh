#!/bin/bash
# Interleaved headline arms with the bind-hop deciles printed (where in a burst the API tail sits).
# usage: OUT=dir REPS=n tools/box_decile_ab.sh "flags A" "flags B" ...
set -o pipefail
out=${OUT:-gpurun_out/decile}
OUT="$out" REPS=${REPS:-3} tools/bench_arms.sh "$@" || exit $?
python - "$out" <<'PY'
import glob, json, sys
for f in sorted(glob.glob(sys.argv[1] + "/arm*.json")):
    d = json.load(open(f))
    g = d["diagnostics"]["bind_hops_us_by_decile_rank0"]
    print(f.split("/")[-1], d["value"], "p99", d["p99_bind_ms"], "api deciles", g["api"][:4], "...", g["api"][-2:],
          "foreign_api", d.get("foreign_cpus_apiserver"))
PY
