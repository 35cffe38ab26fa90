#!/bin/bash
# One GPU-box session: headline runs with the system-call tally (bench.py --io-tally) and one
# native CPU profile of the extender (60 steps). usage: tools/box_prof.sh OUT [reps]
set -o pipefail
out=$1; reps=${2:-2}
mkdir -p "$out"
OUT="$out/arms" REPS=$reps tools/bench_arms.sh "--io-tally" || exit $?
timeout -k 10 300 python bench.py --gpus 1 --steps 60 --warmup 5 --rtt-variant-ms 0 --steady-variant-steps 0 --nodes-variant 0 \
  --inproc-variant-steps 0 --cpu-profile-out "$out/cpuprof.json" --json-out "$out/cpuprof_bench.json" > "$out/cpuprof.log" 2>&1 || exit $?
echo done
