#!/bin/bash
# Quick bench on the box: 1 rank on the GPU (20 steps) then the gloo/--no-gpu rank rehearsal.
set -o pipefail
mkdir -p gpurun_out/quick
timeout -k 10 600 python -u bench.py --steps ${BENCH_STEPS:-20} --warmup 3 $FLAGS > gpurun_out/quick/r1.json 2> gpurun_out/quick/r1.err || { echo "bench failed"; tail -30 gpurun_out/quick/r1.err; exit 1; }
tail -1 gpurun_out/quick/r1.json | cut -c1-400
bash tools/gpu_ranks_rehearsal.sh
