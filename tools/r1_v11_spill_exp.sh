# Spill-round dealing experiment (round 1, v11): pieces per spill wave (EMQX_RETAIN_SPILL_PER_WAVE).
set -o pipefail
O=gpurun_out/r1_v11s
mkdir -p $O
for per in 1 2 4 8 16; do
  EMQX_RETAIN_SPILL_PER_WAVE=$per timeout -k 10 300 python -u bench.py --workload R --no-cpu-baseline > $O/benchR_p$per.json 2> $O/benchR_p$per.err || { echo "bench per=$per failed"; tail -20 $O/benchR_p$per.err; exit 1; }
  python -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], round(d['value']), d['walk_ms_median'], d['call_ms_median'], d['walk_spill_rounds'], d['walk_spilled_items'])" $O/benchR_p$per.json "per=$per"
done
