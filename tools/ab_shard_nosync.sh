#!/bin/bash
set -u
O=gpurun_out/r6_nosync; mkdir -p $O
for r in 1 2; do
  for cfg in "0 2" "1 2" "0 3" "1 3"; do
    set -- $cfg
    EMQX_SHARD_NOSYNC_PROBE=$1 EMQX_SHARD_DEPTH=$2 timeout -k 10 300 python bench.py --sharded --steps 100 --no-cpu-baseline > $O/p$1_d$2_$r.json 2> $O/p$1_d$2_$r.err || { tail -20 $O/p$1_d$2_$r.err; exit 1; }
    python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], d['value'], d['ms_per_step'], d['parity']['mismatching_topics_per_rank'])" $O/p$1_d$2_$r.json "probe=$1 depth=$2 r=$r"
  done
done
