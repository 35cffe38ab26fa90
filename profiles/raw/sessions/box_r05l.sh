#!/bin/bash
# Round-5 box session L: the decisive filter as the headline pass (which thread bounds it),
# twice plain and once with the call-site tally. usage: tools/box_r05l.sh OUT
set -o pipefail
OUT="$1" REPS=2 tools/bench_arms.sh "--decisive-filter" || exit $?
timeout -k 10 240 python bench.py --gpus 1 --steps 20 --warmup 5 --rtt-variant-ms 0 --steady-variant-steps 0 \
  --nodes-variant 0 --inproc-variant-steps 0 --decisive-variant-steps 0 --decisive-filter --io-tally \
  --json-out "$1/tally.json" > "$1/tally.log" 2>&1 || exit $?
echo done
