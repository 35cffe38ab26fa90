#!/bin/bash
# Round-5 box session H: GPU tests, smoke, three driver-style bench runs (the extender's loop on
# its own thread; the front door's residence share of the 1,000-node cycle). usage: tools/box_r05h.sh OUT
set -o pipefail
out=$1
mkdir -p "$out"
timeout -k 10 420 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > "$out/gputest.log" 2>&1 || exit $?
tail -2 "$out/gputest.log"
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$out/smoke.log" 2>&1 || exit $?
echo smoke ok
for i in 1 2 3; do
  timeout -k 10 600 python bench.py --gpus 1 --steps 20 --warmup 5 --json-out "$out/full$i.json" > "$out/full$i.out" 2> "$out/full$i.err" || exit $?
  python -c "
import json; d=json.load(open('$out/full$i.json')); g=d.get('diagnostics', {})
print({k: d.get(k) for k in ('value','p50_bind_ms','p99_bind_ms','bind_tail_hop','extender_cpu_us_per_pod_rank0','bench_harness_cpu_us_per_pod_rank0','extender_share_of_cycle','value_nodes1000','extender_share_of_cycle_nodes1000','extender_held_share_of_cycle_nodes1000','extender_verb_share_of_cycle_nodes1000','cycle_us_nodes1000','frag_pct','value_rtt2ms')})
print(g.get('extender_cpu_us_per_pod_by_thread_rank0'))"
done
echo done
