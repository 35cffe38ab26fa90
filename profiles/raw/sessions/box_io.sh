#!/bin/bash
# One GPU-box session: the GPU tests, then interleaved headline arms with the system-call
# tally on (bench.py --io-tally). usage: tools/box_io.sh OUT "arm flags" ["arm flags" ...]
set -o pipefail
out=$1; shift
mkdir -p "$out"
timeout -k 10 420 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > "$out/gputest.log" 2>&1 || exit $?
tail -2 "$out/gputest.log"
OUT="$out/arms" REPS=${REPS:-3} tools/bench_arms.sh "$@" || exit $?
echo done
