#!/bin/bash
# End-of-round box session: the GPU tests, interleaved headline arms (default first), one full
# default bench.py as the driver runs it (every variant pass), and a kernel trace.
# usage: tools/box_final.sh OUT "arm flags" ["arm flags" ...]   (REPS: runs per arm, default 3)
set -o pipefail
out=$1; shift
mkdir -p "$out"
timeout -k 10 420 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > "$out/gputest.log" 2>&1 || exit $?
tail -2 "$out/gputest.log"
OUT="$out/arms" REPS=${REPS:-3} tools/bench_arms.sh "$@" || exit $?
timeout -k 10 600 python bench.py --json-out "$out/full.json" > "$out/full.log" 2>&1 || exit $?
tail -c 1200 "$out/full.log"
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$out/rocprof" -o run -- python3 bench.py --gpus 1 --steps 20 --warmup 5 \
  --rtt-variant-ms 0 --steady-variant-steps 0 --nodes-variant 0 --inproc-variant-steps 0 \
  --json-out "$out/rocprof_bench.json" > "$out/rocprof.log" 2>&1 || exit $?
echo done
