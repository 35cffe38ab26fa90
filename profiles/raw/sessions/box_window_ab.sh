set -o pipefail
out=gpurun_out/r04z; mkdir -p $out
for i in 1 2; do
  for w in 20 8; do
    timeout -k 10 300 python bench.py --gpus 1 --steps 3 --warmup 1 --nodes 1000 --pods 15625 --rtt-variant-ms 0 --steady-variant-steps 0 --nodes-variant 0 --inproc-variant-steps 0 --busy-poll-us $w --json-out $out/n1000_w${w}_$i.json > $out/n1000_w${w}_$i.log 2>&1 || exit $?
    python -c "import json; d=json.load(open('$out/n1000_w${w}_$i.json')); print('n1000 w$w', d['value'], d['p50_bind_ms'], d['extender_cpu_us_per_pod_rank0'])"
    timeout -k 10 240 python bench.py --gpus 1 --steps 20 --warmup 5 --rtt-variant-ms 0 --steady-variant-steps 0 --nodes-variant 0 --inproc-variant-steps 0 --busy-poll-us $w --json-out $out/h_w${w}_$i.json > $out/h_w${w}_$i.log 2>&1 || exit $?
    python -c "import json; d=json.load(open('$out/h_w${w}_$i.json')); print('head w$w', d['value'], d['p50_bind_ms'], d['extender_cpu_us_per_pod_rank0'])"
  done
done
