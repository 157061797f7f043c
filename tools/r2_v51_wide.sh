#!/bin/bash
# A/B of the wide nodes' bucket load (EMQX_WIDE_SLACK: array = next_pow2(k * edges)): 4 (default) vs 2, alternating.
set -u -o pipefail
O=gpurun_out/${1:-r2_v51}
mkdir -p $O
for k in 1 2; do
  for sl in 4 2; do
    export EMQX_WIDE_SLACK=$sl
    timeout -k 10 400 python -u bench.py --cache /tmp/wlB --no-cpu-baseline --no-host-api --diag > $O/B_s${sl}_$k.json 2> $O/B_s${sl}_$k.err || { echo failed; tail -5 $O/B_s${sl}_$k.err; exit 1; }
    python -c "import json; d=json.loads(open('$O/B_s${sl}_$k.json').read().strip().splitlines()[-1]); dg=d['diag_per_topic']; print('slack $sl', $k, d['value'], d['ms_per_step'], d['roofline']['kernel_ms_avg'], 'lit_extra', dg['lit_extra_loads'], 'table GB?')"
    grep "table:" $O/B_s${sl}_$k.err
  done
done
