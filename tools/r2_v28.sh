#!/bin/bash
# E (match + fan-out) bench line and kernel stats; D with three streams.
set -u -o pipefail
O=gpurun_out/${1:-r2_v28}
mkdir -p $O
export TMPDIR=/tmp
ROOT=$(pwd)
timeout -k 10 600 python -u bench.py --workload E --cache /tmp/wlE > $O/benchE.json 2> $O/benchE.err || { echo E failed; tail -20 $O/benchE.err; exit 1; }
python -c "import json; d=json.loads(open('$O/benchE.json').read().strip().splitlines()[-1]); print('E', d['value'], d['ms_per_step'], d.get('match_call_ms'), d.get('fanout_call_ms'), d['roofline']['frac'], d.get('parity'))"
cd /tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $ROOT/$O/profE -o run -- python3 $ROOT/bench.py --workload E --cache /tmp/wlE --no-cpu-baseline --steps 10 --warmup 2 > $ROOT/$O/profE.json 2> $ROOT/$O/profE.err || { echo rocprof E failed; tail -5 $ROOT/$O/profE.err; exit 1; }
cd $ROOT
timeout -k 10 600 python -u bench.py --workload D --cache /tmp/wlD --steps 10 --streams 3 --no-cpu-baseline --no-host-api > $O/benchD3.json 2> $O/benchD3.err || { echo D3 failed; tail -20 $O/benchD3.err; exit 1; }
python -c "import json; d=json.loads(open('$O/benchD3.json').read().strip().splitlines()[-1]); print('D3', d['value'], d['ms_per_step'], d['call_ms_avg'], d['step_completion_gap_ms'])"
for cfg in "32 8" "24 6" "16 8"; do
  set -- $cfg
  timeout -k 10 600 python -u bench.py --cache /tmp/wlB --no-cpu-baseline --no-host-api --walk-order on --walk-sort-bits $1 --walk-level-bits $2 > $O/benchB_s$1_l$2.json 2> $O/benchB_s$1_l$2.err || { echo B order failed; tail -20 $O/benchB_s$1_l$2.err; exit 1; }
  python -c "import json; d=json.loads(open('$O/benchB_s$1_l$2.json').read().strip().splitlines()[-1]); print('B order s$1 l$2', d['value'], d['ms_per_step'], d['call_ms_avg'], d['roofline']['kernel_ms_avg'], d['order_ms_avg'])"
done
