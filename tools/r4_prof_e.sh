# rocprofv3 kernel stats of config E with a given $share strategy (one stream, 10 steps)
set -u
OUT=gpurun_out/${1:-r4_profE}; ST=${2:-round_robin}; shift 2; EXTRA="$@"
mkdir -p $OUT
ROOT=$(pwd)
cd /tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$ROOT/$OUT/prof_$ST" -o run -- python3 "$ROOT/bench.py" --workload E --strategy $ST --no-cpu-baseline --streams 1 --steps 10 $EXTRA > "$ROOT/$OUT/prof_$ST.json" 2> "$ROOT/$OUT/prof_$ST.err" || { echo rocprof failed; tail "$ROOT/$OUT/prof_$ST.err"; exit 1; }
cd "$ROOT"
f=$(find $OUT/prof_$ST -name "*kernel_stats.csv" | head -1)
python3 - "$f" <<'PY'
import csv,sys
for r in csv.DictReader(open(sys.argv[1])):
    n=r['Name']
    if 'rocprim' in n: n='rocprim '+('onesweep_iter' if 'onesweep_iteration' in n else 'histo' if 'histogram' in n else 'other')
    print("%-60s %5s %10.1f us avg %10.1f min %10.1f max" % (n[:60], r['Calls'], float(r['AverageNs'])/1e3, float(r['MinNs'])/1e3, float(r['MaxNs'])/1e3))
PY
