set -o pipefail
mkdir -p gpurun_out/r04w
timeout -k 10 420 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/r04w/gputest.log 2>&1 || exit $?
tail -2 gpurun_out/r04w/gputest.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r04w/smoke.log 2>&1 || exit $?
tail -2 gpurun_out/r04w/smoke.log
timeout -k 10 400 python bench.py > gpurun_out/r04w/bench.log 2>&1 || exit $?
tail -c 700 gpurun_out/r04w/bench.log
