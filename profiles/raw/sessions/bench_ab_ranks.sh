#!/bin/bash
# A/B of two source trees with N ranks (torchrun; gloo with --no-gpu in $FLAGS, so no rank
# touches the card): this tree (A) and a worktree of another commit at $B_TREE, built in
# place beforehand; 3 alternating runs each.
set -o pipefail
mkdir -p gpurun_out/abr
N=${NPROC:-2}
run() {   # $1 = tree, $2 = output json, $3 = port
  (cd "$1" && timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node $N \
     --master-addr 127.0.0.1 --master-port $3 bench.py --gpus $N $FLAGS) > "$2" 2> "$2.err"
}
for i in 1 2 3; do
  run . gpurun_out/abr/a${N}_$i.json $((29500 + i)) || exit $?
  run "$B_TREE" "$PWD/gpurun_out/abr/b${N}_$i.json" $((29600 + i)) || exit $?
done
