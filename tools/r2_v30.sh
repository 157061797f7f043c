#!/bin/bash
# Streams sweep on B; D with 30 steps (does the one long gap recur?).
set -u -o pipefail
O=gpurun_out/${1:-r2_v30}
mkdir -p $O
for k in 2 4 6; do
  timeout -k 10 600 python -u bench.py --cache /tmp/wlB --no-cpu-baseline --no-host-api --streams $k > $O/benchB_st$k.json 2> $O/benchB_st$k.err || { echo B failed; tail -20 $O/benchB_st$k.err; exit 1; }
  python -c "import json; d=json.loads(open('$O/benchB_st$k.json').read().strip().splitlines()[-1]); print('B streams $k', d['value'], d['ms_per_step'], d['step_completion_gap_ms'])"
done
timeout -k 10 600 python -u bench.py --workload D --cache /tmp/wlD --steps 30 --no-cpu-baseline --no-host-api > $O/benchD30.json 2> $O/benchD30.err || { echo D failed; tail -20 $O/benchD30.err; exit 1; }
python - $O/benchD30.json <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print('D30', d['value'], d['ms_per_step'], d['step_completion_gap_ms'], d.get('step_gaps_ms'))
PY
