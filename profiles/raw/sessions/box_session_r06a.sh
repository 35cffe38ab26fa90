set -o pipefail
out=gpurun_out/r06a; mkdir -p $out
timeout -k 10 420 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $out/gputest.log 2>&1 || { tail -30 $out/gputest.log; exit 1; }
tail -2 $out/gputest.log
timeout -k 10 600 python bench.py --gpus 1 --steps 20 --warmup 3 --json-out $out/bench.json > $out/bench.line 2> $out/bench.err || { tail -30 $out/bench.err; exit 1; }
cat $out/bench.line | head -c 600
