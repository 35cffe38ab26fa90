#!/bin/bash
# Interleaved headline runs with and without an environment setting (A/B of a build switch).
# usage: OUT=dir REPS=n tools/box_env_ab.sh "VAR=value"
set -o pipefail
out=${OUT:-gpurun_out/envab}; reps=${REPS:-3}
mkdir -p "$out"
base="--gpus 1 --steps 20 --warmup 5 --rtt-variant-ms 0 --steady-variant-steps 0 --nodes-variant 0 --inproc-variant-steps 0"
for i in $(seq 1 "$reps"); do
  for arm in A B; do
    if [ "$arm" = B ]; then envset="$1"; else envset=""; fi
    env $envset timeout -k 10 240 python bench.py $base --json-out "$out/$arm$i.json" > "$out/$arm$i.log" 2>&1 || exit $?
    python -c "
import json; d=json.load(open('$out/$arm$i.json')); g=d['diagnostics']
print('$arm', '$envset', d['value'], d['p50_bind_ms'], d['p99_bind_ms'], d['extender_cpu_us_per_pod_rank0'], d['extender_share_of_cycle'], g['native_verb_mean_us'], d['phase_ms_per_step_rank0'] if 'phase_ms_per_step_rank0' in d else g.get('phase_ms_per_step_rank0'))"
  done
done
