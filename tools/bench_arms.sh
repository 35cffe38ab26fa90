#!/bin/bash
# Interleaved A/B/C... of bench.py flag sets on one GPU box: OUT=dir REPS=n tools/bench_arms.sh "flags A" "flags B" ...
# Each arm's runs alternate with the others' (so host noise falls on every arm alike); headline
# pass only (no variant passes) unless an arm's flags ask for them.
set -o pipefail
out=${OUT:-gpurun_out/arms}; reps=${REPS:-3}
mkdir -p "$out"
base="--gpus 1 --steps 20 --warmup 5 --rtt-variant-ms 0 --steady-variant-steps 0 --nodes-variant 0 --inproc-variant-steps 0 --decisive-variant-steps 0"
for i in $(seq 1 "$reps"); do
  k=0
  for flags in "$@"; do
    k=$((k + 1))
    timeout -k 10 240 python bench.py $base $flags --json-out "$out/arm${k}_$i.json" > "$out/arm${k}_$i.log" 2>&1 || exit $?
    python -c "import json; d=json.load(open('$out/arm${k}_$i.json')); print('arm$k', '$flags', d['value'], d['p50_bind_ms'], d['extender_cpu_us_per_pod_rank0'], d['diagnostics']['extender_cpu_us_per_pod_by_thread_rank0'])"
  done
done
