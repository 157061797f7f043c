#!/bin/bash
# Output-kernel ablations (RETAIN_PROF build) in spill and queue mode: where the queue mode's
# slower count/write passes lose time (bit 0: no small rows, 1: no big records, 2: no atomics).
set -u
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r4_q9}
mkdir -p $OUT
B="balance=1,queue_check=4,queue_wait=65536,queue_piece=512,queue_sleep=1,queue_shards=64"
for abl in 0 1 2 4; do
  EMQX_LIB=$(pwd)/emqx_amd/_build_prof/libemqxmatch.so EMQX_RETAIN_PROF=1 EMQX_RETAIN_ABLATE=$abl timeout -k 10 200 python -u tools/retain_sweep.py --calls=6 --nocheck 'balance=0' "$B" > $OUT/abl$abl.jsonl 2> $OUT/abl$abl.err || { tail -20 $OUT/abl$abl.err; exit 1; }
  echo "ablate $abl"; cat $OUT/abl$abl.jsonl | python3 -c "
import sys,json
for l in sys.stdin:
    d=json.loads(l); print(d['spec'][:9], 'call', d['call_ms'], 'walk', d['walk_ms'], 'out', round(d['call_ms']-d['walk_ms'],4))"
done
