#!/bin/bash
# Round-5 box session B: interleaved headline arms (default vs more API-server threads), one
# headline run with the call-site tally, then the multi-rank rehearsal through bench.py's own
# launcher (`--gpus N --no-gpu`: N gloo ranks on the box's CPUs, no rank touches the GPU).
# usage: tools/box_r05b.sh OUT
set -o pipefail
out=$1
mkdir -p "$out"
OUT="$out/arms" REPS=${REPS:-3} tools/bench_arms.sh "" "--apiserver-threads 8" || exit $?
timeout -k 10 240 python bench.py --gpus 1 --steps 20 --warmup 5 --rtt-variant-ms 0 --steady-variant-steps 0 \
  --nodes-variant 0 --inproc-variant-steps 0 --io-tally --json-out "$out/tally.json" > "$out/tally.log" 2>&1 || exit $?
for N in ${RANKS:-1 2 4 8}; do
  timeout -k 10 400 python bench.py --gpus "$N" --no-gpu --steps 10 --warmup 2 --json-out "$out/ranks$N.json" \
    > "$out/ranks$N.log" 2>&1 || { echo "ranks $N failed"; tail -20 "$out/ranks$N.log"; exit 1; }
  python -c "
import json; d=json.load(open('$out/ranks$N.json'))
print($N, {k: d.get(k) for k in ('n_gpus','value','value_independent_schedulers','frag_pct_steady','value_steady','bind_handoffs','p99_bind_ms','schedule_ms_by_rank')})"
done
echo done
