#!/bin/bash
# Fan-out chunk offsets A/B: one pass (look-back) vs count + partials; tests, E benches, kernel stats.
set -u
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r4_v16}
mkdir -p $OUT
timeout -k 10 500 python -u -m pytest -x -v --timeout 240 --timeout-method thread tests/test_gpu_fanout.py \
  tests/test_gpu_fanout_state.py tests/test_gpu_share_parity.py > $OUT/pytest.log 2>&1 || { tail -40 $OUT/pytest.log; exit 1; }
tail -2 $OUT/pytest.log
EMQX_FANOUT_ONEPASS=0 timeout -k 10 300 python -u -m pytest -x -q --timeout 240 --timeout-method thread tests/test_gpu_fanout.py \
  tests/test_gpu_share_parity.py > $OUT/pytest_twopass.log 2>&1 || { tail -40 $OUT/pytest_twopass.log; exit 1; }
tail -2 $OUT/pytest_twopass.log
for op in 1 0; do for st in hash_clientid round_robin; do
EMQX_FANOUT_ONEPASS=$op timeout -k 10 300 python -u bench.py --workload E --strategy $st --steps 20 > $OUT/bench_E_${st}_op$op.json 2> $OUT/bench_E_${st}_op$op.err || { tail -20 $OUT/bench_E_${st}_op$op.err; exit 1; }
python3 -c "import json;d=json.load(open('$OUT/bench_E_${st}_op$op.json'));print('E $st onepass=$op',d['value'],d['ms_per_step'],d['fanout_call_ms'],d['match_call_ms'],d.get('parity',{}).get('mismatches'))"
done; done
ROOT=$(pwd)
for op in 1 0; do
cd /tmp
EMQX_FANOUT_ONEPASS=$op timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$ROOT/$OUT/prof_op$op" -o run -- python3 "$ROOT/bench.py" --workload E --no-cpu-baseline --streams 1 --steps 10 > "$ROOT/$OUT/prof_op$op.json" 2> "$ROOT/$OUT/prof_op$op.err" || { tail -20 "$ROOT/$OUT/prof_op$op.err"; exit 1; }
cd "$ROOT"
f=$(find $OUT/prof_op$op -name "*kernel_stats.csv" | head -1)
echo "== onepass=$op"
python3 - "$f" <<'PY'
import csv,sys
for r in csv.DictReader(open(sys.argv[1])):
    n=r['Name']
    if 'fanout' not in n and 'match_fast' not in n and 'scatter_fast' not in n: continue
    print("%-60s %5s %10.1f us avg %10.1f min %10.1f max" % (n[:60], r['Calls'], float(r['AverageNs'])/1e3, float(r['MinNs'])/1e3, float(r['MaxNs'])/1e3))
PY
done
