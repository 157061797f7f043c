#!/bin/bash
# Interleaved A/B of the sharded step's two forms (EMQX_SHARD_FIXED 0 = classic size syncs,
# 1 = fixed capacities) at several steps in flight, config B at world 1.
# Usage: bash tools/ab_shard_fixed.sh OUT [fixed:depth ...]   (default 0:3 1:3 1:2)
set -u
O=gpurun_out/${1:-r6_fixed}; shift || true
CFGS=${*:-"0:3 1:3 1:2"}
mkdir -p $O
for r in 1 2; do
  for cfg in $CFGS; do
    f=${cfg%%:*}; d=${cfg##*:}
    EMQX_SHARD_FIXED=$f EMQX_SHARD_DEPTH=$d timeout -k 10 300 python bench.py --sharded --steps 100 --no-cpu-baseline > $O/f${f}_d${d}_$r.json 2> $O/f${f}_d${d}_$r.err || { tail -20 $O/f${f}_d${d}_$r.err; exit 1; }
    python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], d['value'], d['ms_per_step'], d['parity']['mismatching_topics_per_rank'], d.get('fixed_steps_redone'))" $O/f${f}_d${d}_$r.json "fixed=$f depth=$d r=$r"
  done
done
