# GPU validation on the gpurun box: GPU tests, smoke(), a 20-step bench, a kernel-trace profile.
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd $R
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/gputest.log 2>&1 || { echo "gpu tests failed rc=$?"; tail -30 gpurun_out/gputest.log; exit 1; }
tail -5 gpurun_out/gputest.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { echo "smoke failed"; tail -30 gpurun_out/smoke.log; exit 1; }
tail -2 gpurun_out/smoke.log
timeout -k 10 600 python -u bench.py --steps ${BENCH_STEPS:-20} --warmup 3 > gpurun_out/bench.log 2>&1 || { echo "bench failed"; tail -30 gpurun_out/bench.log; exit 1; }
tail -1 gpurun_out/bench.log | cut -c1-1500
if [ "${PROFILE:-1}" = "1" ]; then
  cd /tmp && export TMPDIR=/tmp
  timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof -o run -- python3 $R/bench.py --steps 5 --warmup 1 > $R/gpurun_out/prof.log 2>&1 || { echo "prof failed"; tail -20 $R/gpurun_out/prof.log; exit 1; }
fi
if [ "${CONFIGS:-0}" = "1" ]; then
  cd $R && timeout -k 10 600 python -u -m nanogpu.sim.configs --out gpurun_out/configs.json > gpurun_out/configs.log 2>&1 || { echo "configs failed"; tail -20 gpurun_out/configs.log; exit 1; }
  tail -3 gpurun_out/configs.log
fi
echo done
