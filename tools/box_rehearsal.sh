#!/bin/bash
# One box session: the headline bench on the GPU (REPS runs), then the multi-rank rehearsal
# (gloo, --no-gpu: no rank touches the GPU) at each N given, every variant pass.
# usage: tools/box_rehearsal.sh OUT [N ...]        e.g. tools/box_rehearsal.sh gpurun_out/r06c 2 4 8
set -o pipefail
out=$1; shift
mkdir -p "$out"
for k in $(seq 1 "${REPS:-2}"); do
  timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 3 --json-out "$out/bench_$k.json" \
    > "$out/bench_$k.line" 2> "$out/bench_$k.err" || { tail -30 "$out/bench_$k.err"; exit 1; }
  echo "bench $k: $(head -c 300 "$out/bench_$k.line" | tail -c 120)"
done
for n in "$@"; do
  timeout -k 10 420 python bench.py --gpus "$n" --no-gpu --steps 10 --warmup 2 --json-out "$out/ranks$n.json" \
    > "$out/ranks$n.line" 2> "$out/ranks$n.err" || { tail -30 "$out/ranks$n.err"; exit 1; }
  echo "ranks $n done"
done
echo done
