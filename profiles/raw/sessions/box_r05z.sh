#!/bin/bash
# Round-5 final box session (the round's last tree): GPU tests, smoke, two driver-style bench runs with
# every variant pass, and a kernel trace of a headline run. usage: tools/box_r05z.sh OUT
set -o pipefail
out=$1
mkdir -p "$out"
timeout -k 10 420 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > "$out/gputest.log" 2>&1 || exit $?
tail -2 "$out/gputest.log"
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$out/smoke.log" 2>&1 || exit $?
echo smoke ok
for i in 1 2; do
  timeout -k 10 600 python bench.py --gpus 1 --steps 20 --warmup 5 --json-out "$out/full$i.json" > "$out/full$i.log" 2>&1 || exit $?
  python -c "
import json; d=json.load(open('$out/full$i.json'))
print({k: d.get(k) for k in ('value','p50_bind_ms','p99_bind_ms','bind_tail_hop','extender_cpu_us_per_pod_rank0','extender_share_of_cycle','value_nodes1000','extender_share_of_cycle_nodes1000','extender_verb_share_of_cycle_nodes1000','cycle_us_nodes1000','frag_pct','frag_pct_steady','value_rtt2ms','value_decisive_filter','extender_held_share_of_cycle_nodes1000')})"
done
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$out/rocprof" -o run -- python3 bench.py --gpus 1 --steps 20 --warmup 5 \
  --rtt-variant-ms 0 --steady-variant-steps 0 --nodes-variant 0 --inproc-variant-steps 0 --decisive-variant-steps 0 \
  --json-out "$out/rocprof_bench.json" > "$out/rocprof.log" 2>&1 || exit $?
echo done
