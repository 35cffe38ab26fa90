#!/bin/bash
# GPU tests and smoke only. usage: tools/box_gputest.sh OUT
set -o pipefail
mkdir -p "$1"
timeout -k 10 420 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > "$1/gputest.log" 2>&1 || { tail -30 "$1/gputest.log"; exit 1; }
tail -2 "$1/gputest.log"
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$1/smoke.log" 2>&1 || exit $?
echo smoke ok
