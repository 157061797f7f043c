#!/bin/bash
# Sharded device step on config C's 100M table at world 1 (parity: rank 0's first 10K topics
# against the oracle restated on the filters that can match them, oracle/pruned.py).
set -u
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r4_shardC}
mkdir -p $OUT
timeout -k 10 1150 python -u bench.py --sharded --n-filters 100000000 --vocab-scale 4 --steps 20 --warmup 3 \
  > $OUT/bench_sharded_C.json 2> $OUT/bench_sharded_C.err || { tail -30 $OUT/bench_sharded_C.err; exit 1; }
head -c 1500 $OUT/bench_sharded_C.json; echo
tail -5 $OUT/bench_sharded_C.err
