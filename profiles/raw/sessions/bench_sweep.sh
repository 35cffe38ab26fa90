#!/bin/bash
# Front-door knob sweep of bench.py on one GPU box (each run bounded; stops at the first failure).
set -o pipefail
mkdir -p gpurun_out/sweep
for cfg in "0 2" "20 2" "0 4" "20 4" "100 2"; do
  set -- $cfg
  out=gpurun_out/sweep/bp$1_ft$2.json
  timeout -k 10 240 python bench.py --steps 10 --warmup 2 --busy-poll-us $1 --frontend-threads $2 \
    --json-out $out > gpurun_out/sweep/bp$1_ft$2.log 2>&1 || exit $?
done
