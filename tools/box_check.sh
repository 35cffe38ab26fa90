#!/bin/bash
# A check of the tree on a GPU box: the GPU tests, smoke(), one default `python bench.py`
# (what the driver runs at round end). usage: bash tools/box_check.sh [OUT]
set -o pipefail
out=${1:-gpurun_out/check}
mkdir -p "$out"
timeout -k 10 420 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > "$out/gputest.log" 2>&1 || exit $?
tail -2 "$out/gputest.log"
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$out/smoke.log" 2>&1 || exit $?
tail -2 "$out/smoke.log"
timeout -k 10 400 python bench.py > "$out/bench.log" 2>&1 || exit $?
tail -c 700 "$out/bench.log"
