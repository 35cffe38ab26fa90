#!/bin/bash
# Round-end check on one MI355X box (run through gpurun): GPU tests, smoke(), default bench.
# Each GPU step has its own time limit; the first failure ends the script.
set -o pipefail
tag=${1:-v}
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread \
  > gpurun_out/gpu_tests_$tag.log 2>&1 || exit $?
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke(); print('SMOKE OK')" \
  > gpurun_out/smoke_$tag.log 2>&1 || exit $?
timeout -k 10 250 python bench.py > gpurun_out/bench_$tag.json 2> gpurun_out/bench_$tag.err || exit $?
tail -1 gpurun_out/gpu_tests_$tag.log
tail -1 gpurun_out/smoke_$tag.log
tail -1 gpurun_out/bench_$tag.json | cut -c1-200
