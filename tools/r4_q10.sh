#!/bin/bash
# Per-mode kernel traces of config R (spill rounds vs sharded queue) + reserved record counts.
set -u
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r4_q10}
mkdir -p $OUT
B="balance=1,queue_check=4,queue_wait=65536,queue_piece=512,queue_sleep=1,queue_shards=64"
ROOT=$(pwd)
for m in spill queue; do
  if [ $m = spill ]; then S='balance=0'; else S="$B"; fi
  cd /tmp
  EMQX_RETAIN_PROF=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$ROOT/$OUT/prof_$m" -o run -- python3 "$ROOT/tools/retain_sweep.py" --calls=8 "$S" > "$ROOT/$OUT/$m.json" 2> "$ROOT/$OUT/$m.err" || { tail -20 "$ROOT/$OUT/$m.err"; exit 1; }
  cd "$ROOT"
  cat $OUT/$m.json
  grep RETAIN_CTRL $OUT/$m.err | tail -1
  f=$(find $OUT/prof_$m -name "*kernel_stats.csv" | head -1)
  python3 - "$f" <<'PY'
import csv,sys
for r in csv.DictReader(open(sys.argv[1])):
    n=r['Name']
    if 'retain' not in n and 'scan' not in n and 'fill' not in n: continue
    print("%-60s %5s %10.1f us avg %10.1f min %10.1f max" % (n[:60], r['Calls'], float(r['AverageNs'])/1e3, float(r['MinNs'])/1e3, float(r['MaxNs'])/1e3))
PY
done
