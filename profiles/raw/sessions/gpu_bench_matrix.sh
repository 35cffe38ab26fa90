# Bench variants on the gpurun box, one JSON line each into gpurun_out/matrix/.
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/matrix
cd $R
run() {  # name, args...
  local n=$1; shift
  timeout -k 10 300 python -u bench.py "$@" > gpurun_out/matrix/$n.log 2>&1 || { echo "$n failed"; tail -20 gpurun_out/matrix/$n.log; return 1; }
  tail -1 gpurun_out/matrix/$n.log > gpurun_out/matrix/$n.json
  python - "$n" <<'PY'
import json, sys
d = json.loads(open(f"gpurun_out/matrix/{sys.argv[1]}.json").read())
print(sys.argv[1], {k: d[k] for k in d if k.startswith(("value", "p50_bind", "p99_bind", "frag_pct", "extender_cpu", "error"))})
PY
}
for spec in ${MATRIX:-default shared}; do
  case $spec in
    default) run default --steps 20 --warmup 3 || exit 1 ;;
    nokube) run nokube --no-kube-combine --steps 20 --warmup 3 --rtt-variant-ms 0 --inproc-variant-steps 0 || exit 1 ;;
    w8) run w8 --bind-writer-threads 8 --steps 20 --warmup 3 --rtt-variant-ms 0 --inproc-variant-steps 0 || exit 1 ;;
    w32) run w32 --bind-writer-threads 32 --steps 20 --warmup 3 --rtt-variant-ms 0 --inproc-variant-steps 0 || exit 1 ;;
    w128) run w128 --steps 20 --warmup 3 --rtt-variant-ms 0 --inproc-variant-steps 0 || exit 1 ;;
    fe4) run fe4 --frontend-threads 4 --steps 20 --warmup 3 --rtt-variant-ms 0 --inproc-variant-steps 0 || exit 1 ;;
    t8) run t8 --apiserver-threads 8 --steps 20 --warmup 3 --rtt-variant-ms 0 --inproc-variant-steps 0 || exit 1 ;;
  esac
done
echo done
