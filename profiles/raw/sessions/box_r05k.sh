#!/bin/bash
# Round-5 box session K: steady-churn frag at 8 gloo ranks (one kube-scheduler, binds over every
# rank's worker), the verbs' deferred bookkeeping on (default) vs off (NANOGPU_FE_NO_DEFER=1),
# interleaved. usage: tools/box_r05k.sh OUT
set -o pipefail
out=$1
mkdir -p "$out"
base="--gpus 8 --no-gpu --steps 4 --warmup 1 --rtt-variant-ms 0 --nodes-variant 0 --inproc-variant-steps 0 --decisive-variant-steps 0 --independent-variant-steps 0 --steady-variant-steps 6"
for i in 1 2 3; do
  for arm in defer nodefer; do
    if [ $arm = nodefer ]; then export NANOGPU_FE_NO_DEFER=1; else unset NANOGPU_FE_NO_DEFER; fi
    timeout -k 10 300 python bench.py $base --json-out "$out/${arm}_$i.json" > "$out/${arm}_$i.log" 2>&1 || { echo "$arm $i failed"; tail -20 "$out/${arm}_$i.log"; exit 1; }
    python -c "
import json; d=json.load(open('$out/${arm}_$i.json')); g=d['diagnostics']
print('$arm', $i, d.get('value'), d.get('value_steady'), d.get('frag_pct_steady'), g.get('frag_pct_steady_each_step'), g.get('nominations_steady'))"
  done
done
echo done
