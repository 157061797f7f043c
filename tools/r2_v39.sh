#!/bin/bash
# Refresh lines: R (traffic from the r2_v31 PMC passes), A with one and three streams, C1 with
# the threaded build.
set -u -o pipefail
O=gpurun_out/${1:-r2_v39}
mkdir -p $O
timeout -k 10 300 python -u bench.py --workload R --steps 20 --warmup 3 > $O/benchR.json 2> $O/benchR.err || { echo R failed; tail -5 $O/benchR.err; exit 1; }
python -c "import json; d=json.loads(open('$O/benchR.json').read().strip().splitlines()[-1]); print('R', d['value'], d['ms_per_step'], d['roofline']['traffic'], d['cpu_baseline']['value'])"
for st in 1 3; do
  timeout -k 10 300 python -u bench.py --workload A --streams $st > $O/benchA_st$st.json 2> $O/benchA_st$st.err || { echo A failed; tail -5 $O/benchA_st$st.err; exit 1; }
  python -c "import json; d=json.loads(open('$O/benchA_st$st.json').read().strip().splitlines()[-1]); print('A st$st', d['value'], d['ms_per_step'], d['call_ms_avg'], d['roofline']['kernel_ms_avg'], d.get('parity'), d['cpu_baseline']['value'])"
done
timeout -k 10 900 python -u bench.py --n-filters 100000000 --vocab-scale 4 --no-cpu-baseline --no-host-api --steps 10 > $O/benchC1.json 2> $O/benchC1.err || { echo C1 failed; tail -5 $O/benchC1.err; exit 1; }
python -c "import json; d=json.loads(open('$O/benchC1.json').read().strip().splitlines()[-1]); print('C1', d['value'], d['ms_per_step'], d['call_ms_avg'], d['roofline']['kernel_ms_avg'], d['roofline'].get('traffic'))"
grep table $O/benchC1.err
