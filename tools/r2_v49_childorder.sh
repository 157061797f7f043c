#!/bin/bash
# A/B of the trie's child order (layout): creation order (default) vs EMQX_CHILD_ORDER (hash | size), alternating.
set -u -o pipefail
O=gpurun_out/${1:-r2_v49}
mkdir -p $O
for k in 1 2; do
  for ord in creation size; do
    if [ $ord = creation ]; then unset EMQX_CHILD_ORDER; else export EMQX_CHILD_ORDER=$ord; fi
    timeout -k 10 400 python -u bench.py --cache /tmp/wlB --no-cpu-baseline --no-host-api > $O/B_${ord}_$k.json 2> $O/B_${ord}_$k.err || { echo failed; tail -5 $O/B_${ord}_$k.err; exit 1; }
    python -c "import json; d=json.loads(open('$O/B_${ord}_$k.json').read().strip().splitlines()[-1]); print('$ord', $k, d['value'], d['ms_per_step'], d['roofline']['kernel_ms_avg'])"
  done
done
