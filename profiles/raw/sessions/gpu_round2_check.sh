# Round-2 check on the gpurun box: GPU tests, smoke, default bench, a rank-0 profile of the
# shared-API path, and 2/4-rank CPU (gloo, --no-gpu) rehearsals of the multi-rank path.
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/r2
cd $R
if [ "${SKIP_TESTS:-0}" != "1" ]; then
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/r2/gputest.log 2>&1 || { echo "gpu tests failed"; tail -30 gpurun_out/r2/gputest.log; exit 1; }
tail -2 gpurun_out/r2/gputest.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r2/smoke.log 2>&1 || { echo "smoke failed"; tail -30 gpurun_out/r2/smoke.log; exit 1; }
tail -1 gpurun_out/r2/smoke.log
fi
timeout -k 10 300 python -u bench.py --steps 20 --warmup 3 > gpurun_out/r2/bench.log 2>&1 || { echo "bench failed"; tail -30 gpurun_out/r2/bench.log; exit 1; }
tail -1 gpurun_out/r2/bench.log | cut -c1-600
timeout -k 10 300 python -u bench.py --steps 10 --warmup 2 --rtt-variant-ms 0 --inproc-variant-steps 0 --profile-out gpurun_out/r2/prof_rank0.txt > gpurun_out/r2/bench_prof.log 2>&1 || { echo "prof bench failed"; tail -30 gpurun_out/r2/bench_prof.log; exit 1; }
for n in 2 4; do
  timeout -k 10 300 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node $n --master-addr 127.0.0.1 --master-port $((29600+n)) bench.py --gpus $n --no-gpu --steps 10 --warmup 2 --rtt-variant-ms 0 > gpurun_out/r2/gloo_$n.log 2>&1 || { echo "gloo $n failed"; tail -30 gpurun_out/r2/gloo_$n.log; exit 1; }
  tail -1 gpurun_out/r2/gloo_$n.log | cut -c1-400
done
echo done
