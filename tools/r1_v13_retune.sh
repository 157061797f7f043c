# Retained walk retune after the paired lower bounds (round 1, v13): tile x budget.
set -o pipefail
O=gpurun_out/r1_v13
mkdir -p $O
for cfg in "8 128" "8 96" "8 192" "8 256" "16 128" "4 128"; do
  set -- $cfg
  EMQX_RETAIN_TILE=$1 EMQX_RETAIN_STEP_BUDGET=$2 timeout -k 10 300 python -u bench.py --workload R --no-cpu-baseline > $O/benchR_t$1_b$2.json 2> $O/benchR_t$1_b$2.err || { echo "bench $cfg failed"; tail -20 $O/benchR_t$1_b$2.err; exit 1; }
  python -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], round(d['value']), d['walk_ms_median'], d['call_ms_median'], d['walk_spill_rounds'], d['walk_spilled_items'])" $O/benchR_t$1_b$2.json "t$1_b$2"
done
