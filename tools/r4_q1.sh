#!/bin/bash
# Work-sharing retained walk: GPU parity (all retained tests), R bench in queue and spill mode,
# kernel stats of the queue mode.
set -u
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r4_q1}
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_retain.py > $OUT/pytest.log 2>&1 || { tail -40 $OUT/pytest.log; exit 1; }
tail -3 $OUT/pytest.log
timeout -k 10 300 python -u bench.py --workload R --no-cpu-baseline > $OUT/bench_R_queue.json 2> $OUT/bench_R_queue.err || { tail -20 $OUT/bench_R_queue.err; exit 1; }
EMQX_RETAIN_BALANCE=0 timeout -k 10 300 python -u bench.py --workload R --no-cpu-baseline > $OUT/bench_R_spill.json 2> $OUT/bench_R_spill.err || { tail -20 $OUT/bench_R_spill.err; exit 1; }
for m in queue spill; do python3 -c "import json;d=json.load(open('$OUT/bench_R_$m.json'));print('$m',d['value'],d['ms_per_step'],d['call_ms_median'],d['walk_ms_median'],d['walk_spilled_items'],d['walk_shares'],d['walk_queue_aborts'],d['node_visits_per_filter'])"; done
ROOT=$(pwd)
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$ROOT/$OUT/profR" -o run -- python3 "$ROOT/bench.py" --workload R --steps 10 --no-cpu-baseline > "$ROOT/$OUT/profR.json" 2> "$ROOT/$OUT/profR.err" || { tail -20 "$ROOT/$OUT/profR.err"; exit 1; }
cd "$ROOT"
f=$(find $OUT/profR -name "*kernel_stats.csv" | head -1)
cp "$f" $OUT/kernel_stats_R.csv
python3 - "$f" <<'PY'
import csv,sys
for r in csv.DictReader(open(sys.argv[1])):
    n=r['Name']
    if 'retain' not in n: continue
    print("%-60s %5s %10.1f us avg %10.1f min %10.1f max" % (n[:60], r['Calls'], float(r['AverageNs'])/1e3, float(r['MinNs'])/1e3, float(r['MaxNs'])/1e3))
PY
