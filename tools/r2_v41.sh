#!/bin/bash
# D: walk-order keys of 2 bits per level sorted as u32 (32 bits) vs the 4-bit/64-bit default.
set -u -o pipefail
O=gpurun_out/${1:-r2_v41}
mkdir -p $O
for cfg in "4 64" "2 32"; do
  set -- $cfg
  timeout -k 10 600 python -u bench.py --workload D --cache /tmp/wlD --steps 10 --no-cpu-baseline --no-host-api --walk-level-bits $1 --walk-sort-bits $2 > $O/benchD_l$1_s$2.json 2> $O/benchD_l$1_s$2.err || { echo D failed; tail -5 $O/benchD_l$1_s$2.err; exit 1; }
  python -c "import json; d=json.loads(open('$O/benchD_l$1_s$2.json').read().strip().splitlines()[-1]); print('D l$1 s$2', d['value'], d['ms_per_step'], d['call_ms_avg'], d['roofline']['kernel_ms_avg'], d['order_ms_avg'])"
done
