#!/bin/bash
# Config E with 2 / 3 / 4 streams.
set -u
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r4_q28}
mkdir -p $OUT
for n in 3 2 4 3; do
  timeout -k 10 300 python -u bench.py --workload E --steps 30 --no-cpu-baseline --streams $n > $OUT/bench_E_s$n.json 2> $OUT/bench_E_s$n.err || { tail -20 $OUT/bench_E_s$n.err; exit 1; }
  python3 -c "import json;d=json.load(open('$OUT/bench_E_s$n.json'));print($n, d['value'], d['ms_per_step'], d.get('fanout_call_ms'))"
done
