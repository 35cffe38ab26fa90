#!/bin/bash
# Round-5 box session J: one headline run with the call-site tally, then the multi-rank
# rehearsal through bench.py's own launcher (`--gpus N --no-gpu`: N gloo ranks on the box's
# CPUs, no rank touches the GPU), every variant pass (the decisive filter's included).
# usage: tools/box_r05j.sh OUT
set -o pipefail
out=$1
mkdir -p "$out"
timeout -k 10 240 python bench.py --gpus 1 --steps 20 --warmup 5 --rtt-variant-ms 0 --steady-variant-steps 0 \
  --nodes-variant 0 --inproc-variant-steps 0 --io-tally --json-out "$out/tally.json" > "$out/tally.log" 2>&1 || exit $?
echo tally done
for N in ${RANKS:-1 2 4 8}; do
  timeout -k 10 400 python bench.py --gpus "$N" --no-gpu --steps 10 --warmup 2 --json-out "$out/ranks$N.json" \
    > "$out/ranks$N.log" 2>&1 || { echo "ranks $N failed"; tail -20 "$out/ranks$N.log"; exit 1; }
  python -c "
import json; d=json.load(open('$out/ranks$N.json'))
print($N, {k: d.get(k) for k in ('n_gpus','value','value_decisive_filter','value_independent_schedulers','frag_pct_steady','value_steady','value_nodes1000','bind_handoffs','p99_bind_ms')})"
done
echo done
