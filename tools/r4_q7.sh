#!/bin/bash
# Sharded work-sharing walk: tuning sweep (uncapped waiters) + kernel stats of both modes.
set -u
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r4_q7}
mkdir -p $OUT
B="balance=1,queue_check=4,queue_wait=65536,queue_piece=512,queue_sleep=1,queue_shards=64,queue_roam=8"
timeout -k 10 400 python -u tools/retain_sweep.py 'balance=0' "$B" "${B/roam=8/roam=0}" "${B/roam=8/roam=2}" "${B/roam=8/roam=24}" "${B/roam=8/roam=63}" \
  "${B/shards=64/shards=128}" "${B/shards=64/shards=32}" "${B/piece=512/piece=256}" 'balance=0' "$B" > $OUT/sweep.jsonl 2> $OUT/sweep.err || { tail -20 $OUT/sweep.err; exit 1; }
cat $OUT/sweep.jsonl
ROOT=$(pwd)
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$ROOT/$OUT/prof" -o run -- python3 "$ROOT/tools/retain_sweep.py" --calls=8 'balance=0' "$B" > "$ROOT/$OUT/prof.json" 2> "$ROOT/$OUT/prof.err" || { tail -20 "$ROOT/$OUT/prof.err"; exit 1; }
cd "$ROOT"
f=$(find $OUT/prof -name "*kernel_stats.csv" | head -1)
python3 - "$f" <<'PY'
import csv,sys
for r in csv.DictReader(open(sys.argv[1])):
    n=r['Name']
    if 'retain' not in n and 'scan' not in n and 'fill' not in n: continue
    print("%-60s %5s %10.1f us avg %10.1f min %10.1f max" % (n[:60], r['Calls'], float(r['AverageNs'])/1e3, float(r['MinNs'])/1e3, float(r['MaxNs'])/1e3))
PY
