#!/bin/bash
# Config C's 100M-filter table on one GPU (C1): bench line (batch order), the FETCH_SIZE pass,
# then the walk order forced on.  Workload cached in /tmp/wlC (generated once per box).
set -u -o pipefail
O=gpurun_out/${1:-r2_v27}
PART=${2:-a}
mkdir -p $O
export TMPDIR=/tmp
ROOT=$(pwd)
ARGS="--n-filters 100000000 --vocab-scale 4 --no-cpu-baseline --no-host-api --cache /tmp/wlC"
pmc() {  # index counters...
  local i=$1; shift
  cd /tmp
  timeout -s KILL 420 rocprofv3 --pmc "$@" --kernel-include-regex match_fast_kernel --output-format csv -d $ROOT/$O/pmc$i -o pmc -- python3 $ROOT/bench.py $ARGS --streams 1 --steps 3 --warmup 1 > $ROOT/$O/pmc$i.log 2>&1
  local rc=$?; cd $ROOT; echo "pmc $i ($*) rc=$rc"; [ $rc -eq 0 ] || { tail -5 $O/pmc$i.log; exit $rc; }
}
if [ "$PART" = a ]; then
  timeout -k 10 600 python -u bench.py $ARGS --steps 10 > $O/benchC1.json 2> $O/benchC1.err || { echo C1 failed; tail -20 $O/benchC1.err; exit 1; }
  python -c "import json; d=json.loads(open('$O/benchC1.json').read().strip().splitlines()[-1]); print('C1', d['value'], d['ms_per_step'], d['call_ms_avg'], d['roofline']['kernel_ms_avg'])"
  pmc 1 FETCH_SIZE
  timeout -k 10 420 python -u bench.py $ARGS --steps 10 --walk-order on > $O/benchC1_order.json 2> $O/benchC1_order.err || { echo C1 order failed; tail -20 $O/benchC1_order.err; exit 1; }
  python -c "import json; d=json.loads(open('$O/benchC1_order.json').read().strip().splitlines()[-1]); print('C1 order', d['value'], d['ms_per_step'], d['call_ms_avg'], d['roofline']['kernel_ms_avg'])"
else
  pmc 2 WRITE_SIZE
  pmc 3 TCC_HIT_sum TCC_MISS_sum
fi
