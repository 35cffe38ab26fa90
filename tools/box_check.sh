#!/bin/bash
# A check of the tree on a GPU box: the GPU tests, smoke(), one default `python bench.py`
# (what the driver runs at round end; REPS of them). usage: [REPS=n] [PROF=1] [RANKS="2 4 8"] bash tools/box_check.sh [OUT]
set -o pipefail
out=${1:-gpurun_out/check}
mkdir -p "$out"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > "$out/gputest.log" 2>&1 || exit $?
tail -2 "$out/gputest.log"
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$out/smoke.log" 2>&1 || exit $?
tail -2 "$out/smoke.log"
for k in $(seq 1 "${REPS:-1}"); do
  timeout -k 10 400 python bench.py --gpus 1 --steps 20 --warmup 5 --json-out "$out/bench_$k.json" > "$out/bench_$k.log" 2>&1 || exit $?
  tail -c 400 "$out/bench_$k.log"; echo
done
# PROF=1: a kernel trace of a headline run as well (rocprofv3 --kernel-trace --stats)
if [ -n "$PROF" ]; then
  root=$(pwd); cd /tmp && export TMPDIR=/tmp
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$root/$out/rocprof" -o run -- python3 "$root/bench.py" --gpus 1 \
    --steps 20 --warmup 5 --rtt-variant-ms 0 --steady-variant-steps 0 --nodes-variant 0 --inproc-variant-steps 0 \
    --decisive-variant-steps 0 --json-out "$root/$out/rocprof_bench.json" > "$root/$out/rocprof.log" 2>&1 || exit $?
  echo "rocprof done"; cd "$root"
fi
# RANKS="2 4 8": the gloo rehearsal at those N (no rank touches the GPU)
for n in $RANKS; do
  timeout -k 10 420 python bench.py --gpus "$n" --no-gpu --steps 10 --warmup 2 --json-out "$out/ranks$n.json" \
    > "$out/ranks$n.line" 2> "$out/ranks$n.err" || { tail -30 "$out/ranks$n.err"; exit 1; }
  echo "ranks $n done"
done
