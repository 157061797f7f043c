#!/bin/bash
# Fan-out count/final rework: fan-out GPU tests, E bench, E kernel stats.
set -u -o pipefail
O=gpurun_out/${1:-r2_v35}
mkdir -p $O
export TMPDIR=/tmp
ROOT=$(pwd)
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_fanout.py > $O/pytest_fanout.log 2>&1
rc=$?; tail -1 $O/pytest_fanout.log; [ $rc -eq 0 ] || { grep -E "FAIL|Error" $O/pytest_fanout.log | head; exit $rc; }
timeout -k 10 600 python -u bench.py --workload E > $O/benchE.json 2> $O/benchE.err || { echo E failed; tail -20 $O/benchE.err; exit 1; }
python -c "import json; d=json.loads(open('$O/benchE.json').read().strip().splitlines()[-1]); print('E', d['value'], d['ms_per_step'], d.get('match_call_ms'), d.get('fanout_call_ms'), d['roofline']['frac'], d.get('parity'))"
cd /tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $ROOT/$O/profE -o run -- python3 $ROOT/bench.py --workload E --no-cpu-baseline --steps 10 --warmup 2 > $ROOT/$O/profE.json 2> $ROOT/$O/profE.err || { echo rocprof E failed; tail -5 $ROOT/$O/profE.err; exit 1; }
cd $ROOT
python - $O <<'PY'
import csv, glob, re, sys
for p in glob.glob(sys.argv[1] + "/profE/**/*kernel_stats.csv", recursive=True):
    for r in csv.DictReader(open(p)):
        m = re.search(r'(fanout_\w+|match_fast_kernel|scatter_fast_kernel)', r["Name"])
        if m: print(m.group(1), r["Calls"], round(float(r["AverageNs"]) / 1000, 1), "us")
PY
