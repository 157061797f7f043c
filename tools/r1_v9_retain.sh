# Retained walk/out experiments (round 1, v9): GPU retain tests, step budgets with 64-node
# spill pieces at 8 filters per tile, the default R bench line, and a rocprofv3 kernel-stats pass.
set -o pipefail
O=gpurun_out/r1_v9
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_retain.py -x -v --timeout 120 --timeout-method thread > $O/pytest_retain.log 2>&1 || { tail -30 $O/pytest_retain.log; exit 1; }
tail -1 $O/pytest_retain.log
for cfg in "8 32" "8 64" "8 128" "8 0"; do
  set -- $cfg
  EMQX_RETAIN_TILE=$1 EMQX_RETAIN_STEP_BUDGET=$2 timeout -k 10 300 python -u bench.py --workload R --no-cpu-baseline > $O/benchR_t$1_b$2.json 2> $O/benchR_t$1_b$2.err || { echo "bench $cfg failed"; tail -20 $O/benchR_t$1_b$2.err; exit 1; }
  python -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], d['value'], d['walk_ms_median'], d['call_ms_median'], d['walk_spill_rounds'], d['walk_spilled_items'])" $O/benchR_t$1_b$2.json "tile=$1 budget=$2"
done
timeout -k 10 400 python -u bench.py --workload R > $O/benchR.json 2> $O/benchR.err || { tail -20 $O/benchR.err; exit 1; }
cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$O/profR -o run -- python3 $GRAFT_REPO_ROOT/bench.py --workload R --no-cpu-baseline > $GRAFT_REPO_ROOT/$O/profR.json 2> $GRAFT_REPO_ROOT/$O/profR.err || { tail -20 $GRAFT_REPO_ROOT/$O/profR.err; exit 1; }
head -6 $GRAFT_REPO_ROOT/$O/profR/run_kernel_stats.csv | cut -c1-160
