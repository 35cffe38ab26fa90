set -o pipefail
out=gpurun_out/r06b; mkdir -p $out
timeout -k 10 480 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $out/gputest.log 2>&1 || { tail -40 $out/gputest.log; exit 1; }
tail -2 $out/gputest.log
for arm in a b; do
  timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 3 --json-out $out/bench_$arm.json > $out/bench_$arm.line 2> $out/bench_$arm.err || { tail -30 $out/bench_$arm.err; exit 1; }
done
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 3 --apiserver-spin-us 0 --json-out $out/bench_nospin.json > $out/bench_nospin.line 2> $out/bench_nospin.err || { tail -30 $out/bench_nospin.err; exit 1; }
echo done
