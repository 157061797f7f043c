#!/bin/bash
# Config E (publish fan-out) round: fan-out GPU tests, the E bench line, its rocprofv3 kernel stats.
set -e
export TMPDIR=/tmp
TAG=${1:-e}
O=gpurun_out/$TAG; mkdir -p $O
ROOT=$(pwd)
timeout -k 10 300 python -u -m pytest tests/test_gpu_fanout.py -x -q --timeout 200 --timeout-method thread > $O/pytest_fanout.log 2>&1 || { tail -40 $O/pytest_fanout.log; exit 1; }
tail -2 $O/pytest_fanout.log
timeout -k 10 400 python -u bench.py --workload E > $O/benchE.json 2> $O/benchE.err || { tail -20 $O/benchE.err; exit 1; }
cat $O/benchE.json
cd /tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$ROOT/$O/profE" -o run -- python3 "$ROOT/bench.py" --workload E --no-cpu-baseline --streams 1 > "$ROOT/$O/profE_bench.json" 2> "$ROOT/$O/profE_bench.err" || { tail -20 "$ROOT/$O/profE_bench.err"; exit 1; }
cd "$ROOT"
find "$O/profE" -name "*kernel_stats.csv" -exec head -16 {} \;
