# Headline-only bench over a list of flag sets (one run each), for A/B on the box:
#   bash tools/bench_matrix.sh "--busy-poll-us 0" "--busy-poll-us 20 --frontend-threads 1" ...
set -o pipefail
mkdir -p gpurun_out/matrix
i=0
for flags in "$@"; do
  i=$((i + 1))
  timeout -k 10 200 python bench.py --steps 20 --warmup 5 --rtt-variant-steps 0 --inproc-variant-steps 0 \
    --steady-variant-steps 0 --nodes-variant 0 $flags 2>/dev/null | tail -1 > gpurun_out/matrix/m$i.json || exit 1
  echo "$flags" > gpurun_out/matrix/m$i.flags
done
echo done
