# Headline only (no variant passes), twice: quick A/B of an extender change on the box.
set -o pipefail
mkdir -p gpurun_out/quick
for i in 1 2; do
  timeout -k 10 200 python bench.py --steps 20 --warmup 5 --rtt-variant-steps 0 --inproc-variant-steps 0 \
    --steady-variant-steps 0 --nodes-variant 0 "$@" 2>/dev/null | tail -1 > gpurun_out/quick/run$i.json || exit 1
done
echo done
