#!/bin/bash
# Multi-rank rehearsal on the 1-GPU box: torchrun with gloo and --no-gpu (no rank touches the
# card), N = 2 and 4, one run each, JSON lines to gpurun_out/ranks/.
set -o pipefail
mkdir -p gpurun_out/ranks
for N in ${RANKS:-2 4}; do
  timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node $N \
    --master-addr 127.0.0.1 --master-port $((29400 + N)) bench.py --gpus $N --no-gpu \
    --steps ${STEPS:-10} --warmup 2 $FLAGS > gpurun_out/ranks/r$N.json 2> gpurun_out/ranks/r$N.err || { echo "ranks $N failed"; tail -20 gpurun_out/ranks/r$N.err; exit 1; }
  tail -1 gpurun_out/ranks/r$N.json | cut -c1-600
done
