#!/bin/bash
# E hash_clientid vs round_robin on one box (interleaved), and round_robin kernel stats.
set -u
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r4_q37}
mkdir -p $OUT
for s in hash_clientid round_robin hash_clientid round_robin; do
  timeout -k 10 300 python -u bench.py --workload E --steps 30 --no-cpu-baseline --strategy $s > $OUT/bench_E_$s.json 2> $OUT/bench_E_$s.err || { tail -20 $OUT/bench_E_$s.err; exit 1; }
  python3 -c "import json;d=json.load(open('$OUT/bench_E_$s.json'));print('$s', d['value'], d['ms_per_step'], d.get('fanout_call_ms'))"
done
ROOT=$(pwd)
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$ROOT/$OUT/prof" -o run -- python3 "$ROOT/bench.py" --workload E --steps 20 --no-cpu-baseline --strategy round_robin --streams 1 > "$ROOT/$OUT/prof.json" 2> "$ROOT/$OUT/prof.err" || { tail -20 "$ROOT/$OUT/prof.err"; exit 1; }
cd "$ROOT"
f=$(find $OUT/prof -name "*kernel_stats.csv" | head -1)
python3 - "$f" <<'PY'
import csv,sys
for r in csv.DictReader(open(sys.argv[1])):
    print("%-70s %5s %8.1f us avg" % (r['Name'][:70], r['Calls'], float(r['AverageNs'])/1e3))
PY
