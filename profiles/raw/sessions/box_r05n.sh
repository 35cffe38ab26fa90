#!/bin/bash
# Round-5 box session N: a soak of the headline (300 timed 1,000-pod steps), steady churn over
# 60 steps and the decisive filter over 100: rate over time, memory before / after.
# usage: tools/box_r05n.sh OUT
set -o pipefail
out=$1
mkdir -p "$out"
timeout -k 10 900 python bench.py --gpus 1 --steps 300 --warmup 5 --rtt-variant-ms 0 --steady-variant-steps 60 \
  --nodes-variant 0 --inproc-variant-steps 0 --decisive-variant-steps 100 --json-out "$out/soak.json" \
  > "$out/soak.out" 2> "$out/soak.err" || exit $?
python - "$out/soak.json" <<'PY'
import json, sys
d = json.load(open(sys.argv[1])); st = d["diagnostics"]["step_diag_rank0"]
dur = [1e3 * (s["t1"] - s["t0"]) for s in st]
chunks = [dur[i:i + 50] for i in range(0, len(dur), 50)]
print({k: d.get(k) for k in ("value", "p50_bind_ms", "p99_bind_ms", "frag_pct", "value_steady", "frag_pct_steady",
                             "value_decisive_filter", "extender_cpu_us_per_pod_rank0", "extender_rss_mib_before_after_rank0")})
print("step ms by 50-step block:", [round(sum(c) / len(c), 2) for c in chunks])
PY
# the decisive filter with one front-door thread (filters queue behind binds on it) vs two
OUT="$out/arms" REPS=2 tools/bench_arms.sh "--decisive-filter" "--decisive-filter --frontend-threads 2" || exit $?
echo done
