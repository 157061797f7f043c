#!/bin/bash
# S with untimed warmup rounds and per-round times.
set -u
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r4_q30}
mkdir -p $OUT
EMQX_SUBTAB_PROF=1 timeout -k 10 400 python -u bench.py --workload S > $OUT/bench_S.json 2> $OUT/bench_S.err || { tail -20 $OUT/bench_S.err; exit 1; }
python3 -c "
import json;d=json.load(open('$OUT/bench_S.json'));print('S',d['value'],d['ms_per_step'],d['host_ms_p50'],d['commit_ms'],d['cpu_baseline']['value']); print(d['round_ms'])"
grep SUBTAB_PROF $OUT/bench_S.err | tail -8
