#!/bin/bash
# Work-sharing retained walk at its defaults: all retained GPU tests, the R line, kernel stats and
# the FETCH/WRITE passes (tools/bench_r.sh), then the spill-round line for comparison.
set -u
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r4_q20}
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_retain.py > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
bash tools/bench_r.sh $OUT/queue || exit 1
EMQX_RETAIN_BALANCE=0 timeout -k 10 300 python -u bench.py --workload R --no-cpu-baseline > $OUT/bench_R_spill.json 2> $OUT/bench_R_spill.err || { tail -20 $OUT/bench_R_spill.err; exit 1; }
python3 -c "
import json
for f in ('$OUT/queue/benchR.json','$OUT/bench_R_spill.json'):
    d=json.load(open(f)); print(f, d['value'], d['ms_per_step'], d['call_ms_median'], d['walk_ms_median'], d['walk_shares'], d['walk_queue_aborts'], d.get('cpu_baseline',{}).get('value'))"
f=$(find $OUT/queue/prof -name "*kernel_stats.csv" | head -1)
python3 - "$f" <<'PY'
import csv,sys
for r in csv.DictReader(open(sys.argv[1])):
    n=r['Name']
    if 'retain' not in n and 'scan' not in n: continue
    print("%-60s %5s %10.1f us avg %10.1f min %10.1f max" % (n[:60], r['Calls'], float(r['AverageNs'])/1e3, float(r['MinNs'])/1e3, float(r['MaxNs'])/1e3))
PY
