#!/bin/bash
# Config C's 100M-filter table on one GPU (C1) with its parity block and CPU baseline: the C++
# DFS (oracle/trie_oracle.cpp) over the whole 100M table on a 200K-topic sample of the batch.
set -u
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r4_c1}
mkdir -p $OUT
timeout -k 10 1150 python -u bench.py --n-filters 100000000 --vocab-scale 4 --cpu-sample 200000 --no-host-api \
  > $OUT/benchC1.json 2> $OUT/benchC1.err || { tail -30 $OUT/benchC1.err; exit 1; }
head -c 1500 $OUT/benchC1.json; echo
tail -5 $OUT/benchC1.err
