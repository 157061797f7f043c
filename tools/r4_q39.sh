#!/bin/bash
# T (per-call changes through the coalescer) with the spinning worker pool.
set -u
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r4_q39}
mkdir -p $OUT
timeout -k 10 400 python -u bench.py --workload T > $OUT/bench_T.json 2> $OUT/bench_T.err || { tail -20 $OUT/bench_T.err; exit 1; }
python3 -c "
import json;d=json.load(open('$OUT/bench_T.json'));print('T single', d['single_op']['subscribe']['p50_us'], d['single_op']['subscribe']['p99_us'], d['single_op']['route_add_delete']['p50_us']); [print(r['callers'], r['ops_per_s'], r['p99_us']) for r in d['storm']]; print(d['publish_alone']['messages_per_s'], d['publish_during_storm']['messages_per_s'])"
