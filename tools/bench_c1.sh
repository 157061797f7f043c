#!/bin/bash
# Config C's 100M-filter table (B generator, vocab x4, seed 3) held whole on ONE MI355X:
# the bench line (1M-topic batches) and the rocprofv3 kernel stats are not repeated here
# (the generation + build take ~10 min); the bench's own HIP-event kernel time is reported.
set -e
export TMPDIR=/tmp
O=gpurun_out/c1; mkdir -p $O
timeout -k 10 1100 python -u bench.py --n-filters 100000000 --vocab-scale 4 --no-cpu-baseline --steps 10 > $O/benchC1.json 2> $O/benchC1.err || { tail -30 $O/benchC1.err; exit 1; }
cat $O/benchC1.json
tail -5 $O/benchC1.err
