#!/bin/bash
# Round-5 box session: GPU tests, smoke, the launcher's refusal on a 1-GPU box, then the driver's
# bench command (every variant pass) REPS times. usage: tools/box_r05.sh OUT
set -o pipefail
out=$1
mkdir -p "$out"
timeout -k 10 420 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > "$out/gputest.log" 2>&1 || exit $?
tail -2 "$out/gputest.log"
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$out/smoke.log" 2>&1 || exit $?
timeout -k 10 120 python bench.py --gpus 2 --steps 1 > "$out/refuse.log" 2>&1
rc=$?
echo "launcher on a 1-GPU box, --gpus 2: rc=$rc"
[ "$rc" -eq 2 ] || exit 1
for i in $(seq 1 "${REPS:-2}"); do
  timeout -k 10 600 python bench.py --gpus 1 --steps 20 --warmup 5 --json-out "$out/full$i.json" > "$out/full$i.log" 2>&1 || exit $?
  tail -c 700 "$out/full$i.log"
done
echo done
