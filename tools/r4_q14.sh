#!/bin/bash
# Queue-mode phase counters (RETAIN_PROF build) at the round-4 defaults.
set -u
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r4_q14}
mkdir -p $OUT
EMQX_LIB=$(pwd)/emqx_amd/_build_prof/libemqxmatch.so EMQX_RETAIN_PROF=1 timeout -k 10 300 python -u tools/retain_sweep.py --calls=4 \
  'balance=0' 'balance=1' 'balance=1,queue_shards=16' > $OUT/sweep.jsonl 2> $OUT/sweep.err || { tail -20 $OUT/sweep.err; exit 1; }
cat $OUT/sweep.jsonl
grep -E "RETAIN_PROF|RETAIN_QPROF|RETAIN_CTRL" $OUT/sweep.err | awk 'NR%12==0 || NR%12==11 || NR%12==10'
