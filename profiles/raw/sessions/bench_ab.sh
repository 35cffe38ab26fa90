#!/bin/bash
# A/B of bench.py flags on one GPU box: alternates "$A" and "$B" runs, 3 each.
set -o pipefail
mkdir -p gpurun_out/ab
for i in 1 2 3; do
  timeout -k 10 240 python bench.py $A --json-out gpurun_out/ab/a$i.json > gpurun_out/ab/a$i.log 2>&1 || exit $?
  timeout -k 10 240 python bench.py $B --json-out gpurun_out/ab/b$i.json > gpurun_out/ab/b$i.log 2>&1 || exit $?
done
