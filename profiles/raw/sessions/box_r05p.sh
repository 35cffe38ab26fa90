#!/bin/bash
# Round-5 box session P: the API server's watch cache size (64k events per kind, the default,
# vs 16k: the timed steps then all evict) on the headline, interleaved. usage: tools/box_r05p.sh OUT
set -o pipefail
OUT="$1" REPS=3 tools/bench_arms.sh "" "--apiserver-history 16384" || exit $?
python - "$1" <<'PY'
import glob, json, sys
for f in sorted(glob.glob(sys.argv[1] + "/arm*.json")):
    d = json.load(open(f)); st = d["diagnostics"]["step_diag_rank0"]
    print(f.split("/")[-1], d["value"], d["p50_bind_ms"], d["p99_bind_ms"], d["diagnostics"]["phase_ms_per_step_rank0"],
          "foreign", d.get("foreign_cpus_apiserver"))
PY
