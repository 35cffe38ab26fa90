set -o pipefail
mkdir -p gpurun_out/ab
for i in 1 2; do
  (cd ab_old && timeout -k 10 200 python bench.py --steps 20 --warmup 5 2>/dev/null | tail -1 > ../gpurun_out/ab/old$i.json) || exit 1
  timeout -k 10 200 python bench.py --steps 20 --warmup 5 2>/dev/null | tail -1 > gpurun_out/ab/new$i.json || exit 1
done
echo done
