#!/bin/bash
# Config D (adversarial) round: GPU tests, the D bench line, its rocprofv3 kernel stats, and
# the deep path's speed (variant 3 defers a quarter of D's topics to match_deep_kernel).
set -e
export TMPDIR=/tmp
TAG=${1:-d}
O=gpurun_out/$TAG; mkdir -p $O
ROOT=$(pwd)
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -30 $O/pytest_gpu.log; exit 1; }
tail -2 $O/pytest_gpu.log
timeout -k 10 400 python -u bench.py --workload D --cache /tmp/wlD > $O/benchD.json 2> $O/benchD.err || { tail -20 $O/benchD.err; exit 1; }
cat $O/benchD.json
cd /tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$ROOT/$O/profD" -o run -- python3 "$ROOT/bench.py" --workload D --cache /tmp/wlD --no-cpu-baseline --streams 1 > "$ROOT/$O/profD_bench.json" 2> "$ROOT/$O/profD_bench.err" || { tail -20 "$ROOT/$O/profD_bench.err"; exit 1; }
cd "$ROOT"
find "$O/profD" -name "*kernel_stats.csv" -exec head -8 {} \;
timeout -k 10 300 python -u bench.py --workload D --cache /tmp/wlD --ab 10,3 --ab-rounds 2 --steps 4 --no-cpu-baseline > $O/deep_ab.json 2> $O/deep_ab.err
cat $O/deep_ab.json
