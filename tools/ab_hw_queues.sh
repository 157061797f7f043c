#!/bin/bash
# Interleaved A/B of HIP's hardware queues per process (GPU_MAX_HW_QUEUES 4 = the default, 8) on
# the config B line and the world-1 sharded step (fixed form, three lanes).
set -u
O=gpurun_out/${1:-r6_hwq}; mkdir -p $O
for r in 1 2; do
  for q in 4 8; do
    GPU_MAX_HW_QUEUES=$q timeout -k 10 300 python bench.py --cache /tmp/wlB --no-cpu-baseline --no-host-api > $O/B_q${q}_$r.json 2> $O/B_q${q}_$r.err || { tail -20 $O/B_q${q}_$r.err; exit 1; }
    GPU_MAX_HW_QUEUES=$q timeout -k 10 300 python bench.py --sharded --steps 100 --no-cpu-baseline > $O/S_q${q}_$r.json 2> $O/S_q${q}_$r.err || { tail -20 $O/S_q${q}_$r.err; exit 1; }
    python3 -c "
import json,sys
b=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); s=json.loads(open(sys.argv[2]).read().strip().splitlines()[-1])
print(sys.argv[3], 'B', b['value'], b['ms_per_step'], 'sharded', s['value'], s['ms_per_step'], s['parity']['mismatching_topics_per_rank'])" $O/B_q${q}_$r.json $O/S_q${q}_$r.json "q=$q r=$r"
  done
done
