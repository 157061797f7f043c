#!/bin/bash
# Interleaved A/B of queue shard counts / roaming against the spill rounds (config R).
set -u
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r4_q18}
mkdir -p $OUT
B="balance=1,queue_check=4,queue_wait=65536,queue_piece=512,queue_sleep=1"
S=""
for rep in 1 2; do
  S="$S balance=0 $B,queue_shards=256,queue_roam=8 $B,queue_shards=256,queue_roam=2 $B,queue_shards=256,queue_roam=4 $B,queue_shards=256,queue_roam=16 $B,queue_shards=512,queue_roam=8 $B,queue_shards=512,queue_roam=4 $B,queue_shards=1024,queue_roam=8 $B,queue_shards=1024,queue_roam=16"
done
timeout -k 10 500 python -u tools/retain_sweep.py --calls=20 $S > $OUT/sweep.jsonl 2> $OUT/sweep.err || { tail -20 $OUT/sweep.err; exit 1; }
python3 - $OUT/sweep.jsonl <<'PY'
import json,sys,collections
d=collections.defaultdict(list)
for l in open(sys.argv[1]):
    j=json.loads(l); d[j['spec'].replace('balance=1,queue_check=4,queue_wait=65536,queue_piece=512,queue_sleep=1,','')].append((j['call_ms'],j['walk_ms']))
for k,v in d.items(): print("%-50s call %s walk %s" % (k, [x[0] for x in v], [x[1] for x in v]))
PY
