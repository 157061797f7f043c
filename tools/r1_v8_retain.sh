# Retained walk experiments (round 1, v8): GPU retain tests, then the R bench over filters per
# wave tile (EMQX_RETAIN_TILE) and step budgets (EMQX_RETAIN_STEP_BUDGET, 0 = none).
set -o pipefail
mkdir -p gpurun_out/${TAG:-r1_v8}
timeout -k 10 400 python -u -m pytest tests/test_gpu_retain.py -x -v --timeout 120 --timeout-method thread > gpurun_out/${TAG:-r1_v8}/pytest_retain.log 2>&1 || { tail -30 gpurun_out/${TAG:-r1_v8}/pytest_retain.log; exit 1; }
tail -3 gpurun_out/${TAG:-r1_v8}/pytest_retain.log
for cfg in ${CFGS:-"64 0" "16 0" "8 0" "4 0" "2 0" "8 512" "4 256"}; do
  set -- $cfg
  EMQX_RETAIN_TILE=$1 EMQX_RETAIN_STEP_BUDGET=$2 timeout -k 10 300 python -u bench.py --workload R --no-cpu-baseline > gpurun_out/${TAG:-r1_v8}/benchR_t$1_b$2.json 2> gpurun_out/${TAG:-r1_v8}/benchR_t$1_b$2.err || { echo "bench $cfg failed"; tail -20 gpurun_out/${TAG:-r1_v8}/benchR_t$1_b$2.err; exit 1; }
  python -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], d['value'], d['walk_ms_median'], d['call_ms_median'], d['walk_spill_rounds'])" gpurun_out/${TAG:-r1_v8}/benchR_t$1_b$2.json "tile=$1 budget=$2"
done
