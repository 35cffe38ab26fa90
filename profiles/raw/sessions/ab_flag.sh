# A/B of one bench flag on the same box: headline only, alternating runs with and without
# FLAG (e.g. FLAG=--no-native-pod-watch), JSON lines to gpurun_out/abflag/.
set -o pipefail
mkdir -p gpurun_out/abflag
for i in ${RUNS:-1 2 3}; do
  for v in a b; do
    f=""; [ $v = b ] && f="$FLAG"
    timeout -k 10 200 python bench.py --steps 20 --warmup 5 --rtt-variant-steps 0 --inproc-variant-steps 0 \
      --steady-variant-steps 0 --nodes-variant 0 --independent-variant-steps 0 $f 2>/dev/null \
      | tail -1 > gpurun_out/abflag/$v$i.json || exit 1
    echo "$v$i $(cut -c1-120 gpurun_out/abflag/$v$i.json)"
  done
done
