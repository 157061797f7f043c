#!/bin/bash
# Locality experiment: host-side permutations of the same batch (bench.py --order) on B and D.
set -e
O=gpurun_out/order; mkdir -p $O
for w in B D; do
  for o in none sorted xcd; do
    timeout -k 10 300 python -u bench.py --workload $w --cache /tmp/wl$w --no-cpu-baseline --order $o --steps 10 > $O/$w-$o.json 2> $O/$w-$o.err
    python -c "import json;d=json.load(open('$O/$w-$o.json'));print('$w $o', d['value'], d['roofline']['kernel_ms_avg'])"
  done
done
