#!/bin/bash
# Fan-out write kernel rework: fan-out GPU tests, E bench; B walk-order phase kernel stats.
set -u -o pipefail
O=gpurun_out/${1:-r2_v29}
mkdir -p $O
export TMPDIR=/tmp
ROOT=$(pwd)
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_fanout.py > $O/pytest_fanout.log 2>&1
rc=$?; tail -2 $O/pytest_fanout.log; [ $rc -eq 0 ] || { grep -E "FAIL|Error" $O/pytest_fanout.log | head; exit $rc; }
timeout -k 10 600 python -u bench.py --workload E > $O/benchE.json 2> $O/benchE.err || { echo E failed; tail -20 $O/benchE.err; exit 1; }
python -c "import json; d=json.loads(open('$O/benchE.json').read().strip().splitlines()[-1]); print('E', d['value'], d['ms_per_step'], d.get('match_call_ms'), d.get('fanout_call_ms'), d['roofline']['frac'], d.get('parity'))"
cd /tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $ROOT/$O/profBo -o run -- python3 $ROOT/bench.py --no-cpu-baseline --no-host-api --walk-order on --walk-sort-bits 32 --steps 10 --warmup 2 --streams 1 > $ROOT/$O/profBo.json 2> $ROOT/$O/profBo.err || { echo rocprof B failed; tail -5 $ROOT/$O/profBo.err; exit 1; }
cd $ROOT
find $O/profBo -name "*kernel_stats.csv" -exec cat {} \; | cut -c1-150 | head -30
