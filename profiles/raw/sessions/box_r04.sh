#!/bin/bash
# Round-4 box session: the GPU tests, interleaved headline arms (with the system-call tally),
# and a kernel trace of one plain headline run. usage: tools/box_r04.sh OUT "arm flags" ...
set -o pipefail
out=$1; shift
mkdir -p "$out"
timeout -k 10 420 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > "$out/gputest.log" 2>&1 || exit $?
tail -2 "$out/gputest.log"
OUT="$out/arms" REPS=${REPS:-3} tools/bench_arms.sh "$@" || exit $?
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$out/rocprof" -o run -- python3 bench.py --gpus 1 --steps 20 --warmup 5 \
  --json-out "$out/rocprof_bench.json" > "$out/rocprof.log" 2>&1 || exit $?
echo done
