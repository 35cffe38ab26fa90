#!/bin/bash
# Repeated bench runs on the box (the box is shared: single runs are noisy): 1 rank on the
# GPU x REPS, then the gloo/--no-gpu rank rehearsal (2 and 4 ranks) x REPS.
set -o pipefail
mkdir -p gpurun_out/rep
for i in $(seq 1 ${REPS:-3}); do
  timeout -k 10 600 python -u bench.py --steps 20 --warmup 3 $FLAGS > gpurun_out/rep/r1_$i.json 2> gpurun_out/rep/r1_$i.err || { echo "bench failed"; tail -30 gpurun_out/rep/r1_$i.err; exit 1; }
  tail -1 gpurun_out/rep/r1_$i.json | cut -c1-200
  for N in 2 4; do
    timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node $N \
      --master-addr 127.0.0.1 --master-port $((29400 + N + 10 * i)) bench.py --gpus $N --no-gpu \
      --steps 10 --warmup 2 $FLAGS > gpurun_out/rep/r${N}_$i.json 2> gpurun_out/rep/r${N}_$i.err || { echo "ranks $N failed"; tail -20 gpurun_out/rep/r${N}_$i.err; exit 1; }
    tail -1 gpurun_out/rep/r${N}_$i.json | cut -c1-200
  done
done
