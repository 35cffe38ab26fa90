#!/bin/bash
# A/B of two source trees on one GPU box: this tree (A) and a git worktree of another commit
# at $B_TREE (built in place beforehand), 3 alternating runs each, same flags ($FLAGS).
set -o pipefail
mkdir -p gpurun_out/abt
for i in 1 2 3; do
  timeout -k 10 240 python bench.py $FLAGS --json-out gpurun_out/abt/a$i.json > gpurun_out/abt/a$i.log 2>&1 || exit $?
  (cd "$B_TREE" && timeout -k 10 240 python bench.py $FLAGS --json-out "$OLDPWD/gpurun_out/abt/b$i.json") \
    > gpurun_out/abt/b$i.log 2>&1 || exit $?
done
