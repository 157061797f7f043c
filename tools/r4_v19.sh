#!/bin/bash
# Control words zeroed in-kernel, single-launch scans: fan-out + host-path tests, P and L lines.
set -u
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r4_v19}
mkdir -p $OUT
timeout -k 10 500 python -u -m pytest -x -v --timeout 240 --timeout-method thread tests/test_gpu_fanout.py \
  tests/test_gpu_fanout_state.py tests/test_gpu_share_parity.py tests/test_gpu_host.py tests/test_gpu_retain.py > $OUT/pytest.log 2>&1 || { tail -40 $OUT/pytest.log; exit 1; }
tail -2 $OUT/pytest.log
timeout -k 10 400 python -u bench.py --workload P > $OUT/bench_P.json 2> $OUT/bench_P.err || { tail -20 $OUT/bench_P.err; exit 1; }
python3 -c "
import json;d=json.load(open('$OUT/bench_P.json'))
print('P', d['value']); [print({k:r.get(k) for k in ('callers','messages_per_s','topics_per_s','p50_us','p99_us','us_per_batch_device_wait')}) for r in d.get('runs',[])]"
timeout -k 10 400 python -u bench.py --workload L > $OUT/bench_L.json 2> $OUT/bench_L.err || { tail -20 $OUT/bench_L.err; exit 1; }
python3 -c "
import json;d=json.load(open('$OUT/bench_L.json'))
print('L', d['value']); [print({k:r.get(k) for k in ('callers','topics_per_s','p50_us','p99_us','us_per_batch_device_wait','topics_per_batch')}) for r in d.get('runs',[])]"
timeout -k 10 400 python -u bench.py --workload R > $OUT/bench_R.json 2> $OUT/bench_R.err || { tail -20 $OUT/bench_R.err; exit 1; }
python3 -c "import json;d=json.load(open('$OUT/bench_R.json'));print('R', d['value'], d['ms_per_step'], d.get('parity'))"
ROOT=$(pwd)
cd /tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$ROOT/$OUT/profR" -o run -- python3 "$ROOT/bench.py" --workload R --steps 10 --no-cpu-baseline > "$ROOT/$OUT/profR.json" 2> "$ROOT/$OUT/profR.err" || { tail -20 "$ROOT/$OUT/profR.err"; exit 1; }
cd "$ROOT"
f=$(find $OUT/profR -name "*kernel_stats.csv" | head -1)
python3 - "$f" <<'PY'
import csv,sys
for r in csv.DictReader(open(sys.argv[1])):
    n=r['Name']
    if 'retain' not in n: continue
    print("%-60s %5s %10.1f us avg %10.1f min %10.1f max" % (n[:60], r['Calls'], float(r['AverageNs'])/1e3, float(r['MinNs'])/1e3, float(r['MaxNs'])/1e3))
PY
