#!/bin/bash
# Scatter unroll + walk order: GPU tests, D (default: ordered) with CPU baseline and parity, B.
set -u -o pipefail
O=gpurun_out/${1:-r2_v23}
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1
rc=$?; tail -2 $O/pytest_gpu.log; [ $rc -eq 0 ] || { echo "gpu tests rc=$rc"; grep -E "FAIL|Error" $O/pytest_gpu.log | head; exit $rc; }
timeout -k 10 600 python -u bench.py --workload D --cache /tmp/wlD --steps 10 > $O/benchD.json 2> $O/benchD.err || { echo D failed; tail -20 $O/benchD.err; exit 1; }
tail -1 $O/benchD.json | cut -c1-600
timeout -k 10 600 python -u bench.py --cache /tmp/wlB --no-cpu-baseline > $O/benchB.json 2> $O/benchB.err || { echo B failed; tail -20 $O/benchB.err; exit 1; }
tail -1 $O/benchB.json | cut -c1-400
