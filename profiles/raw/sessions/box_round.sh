#!/bin/bash
# One GPU-box session of round-4 measurements: interleaved A/B arms, back-to-back headline runs,
# a kernel trace of one headline run and a native CPU profile of another.
# usage: tools/box_round.sh OUT "arm flags" ["arm flags" ...]
set -o pipefail
out=$1; shift
mkdir -p "$out"
timeout -k 10 420 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > "$out/gputest.log" 2>&1 || exit $?
tail -2 "$out/gputest.log"
OUT="$out/arms" REPS=${REPS:-3} tools/bench_arms.sh "$@" || exit $?
tools/box_variance.sh "$out/var" ${VAR_RUNS:-4} || exit $?
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$out/rocprof" -o run -- python3 bench.py --gpus 1 --steps 20 --warmup 5 \
  --json-out "$out/rocprof_bench.json" > "$out/rocprof.log" 2>&1 || exit $?
timeout -k 10 300 python bench.py --gpus 1 --steps 60 --warmup 5 --rtt-variant-ms 0 --steady-variant-steps 0 --nodes-variant 0 \
  --inproc-variant-steps 0 --cpu-profile-out "$out/cpuprof.json" --json-out "$out/cpuprof_bench.json" > "$out/cpuprof.log" 2>&1 || exit $?
echo done
