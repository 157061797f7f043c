#!/bin/bash
# Queue-walk tile size and wave count A/B (config R).
set -u
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r4_q24}
mkdir -p $OUT
S=""
for rep in 1 2; do S="$S balance=1 queue_check=8 queue_check=2,queue_check=4 queue_roam=8 queue_roam=2,queue_roam=4 queue_shards=1024 queue_shards=256,queue_shards=512 queue_piece=256 queue_piece=1024,queue_piece=512 tile=18 tile=15,tile=16"; done
timeout -k 10 400 python -u tools/retain_sweep.py --calls=20 $S > $OUT/sweep.jsonl 2> $OUT/sweep.err || { tail -20 $OUT/sweep.err; exit 1; }
python3 - $OUT/sweep.jsonl <<'PY'
import json,sys,collections
d=collections.defaultdict(list)
for l in open(sys.argv[1]):
    j=json.loads(l); d[j['spec']].append((j['call_ms'],j['walk_ms']))
for k,v in d.items(): print("%-40s call %s walk %s" % (k, [x[0] for x in v], [x[1] for x in v]))
PY
