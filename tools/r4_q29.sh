#!/bin/bash
# Config E kernel stats (3 streams).
set -u
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r4_q29}
mkdir -p $OUT
ROOT=$(pwd)
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$ROOT/$OUT/prof" -o run -- python3 "$ROOT/bench.py" --workload E --steps 20 --no-cpu-baseline > "$ROOT/$OUT/benchE.json" 2> "$ROOT/$OUT/benchE.err" || { tail -20 "$ROOT/$OUT/benchE.err"; exit 1; }
cd "$ROOT"
f=$(find $OUT/prof -name "*kernel_stats.csv" | head -1)
cp $f $OUT/kernel_stats_E.csv
python3 - "$f" <<'PY'
import csv,sys
for r in csv.DictReader(open(sys.argv[1])):
    print("%-70s %5s %8.1f us avg %8.1f total ms" % (r['Name'][:70], r['Calls'], float(r['AverageNs'])/1e3, float(r['TotalDurationNs'])/1e6))
PY
