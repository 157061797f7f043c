#!/bin/bash
# Config R with 1..4 concurrent callers.
set -u
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r4_q27}
mkdir -p $OUT
for n in 1 2 3 4; do
  timeout -k 10 300 python -u bench.py --workload R --no-cpu-baseline --streams $n --steps 40 > $OUT/bench_R_s$n.json 2> $OUT/bench_R_s$n.err || { tail -20 $OUT/bench_R_s$n.err; exit 1; }
  python3 -c "import json;d=json.load(open('$OUT/bench_R_s$n.json'));print($n, d['value'], d['ms_per_step'], d['call_ms_median'], d['walk_ms_median'], d['walk_queue_aborts'])"
done
