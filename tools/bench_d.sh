#!/bin/bash
# Config D (adversarial) round: the D bench line, its rocprofv3 kernel stats (single stream, so
# every launch is isolated), PMC passes (HBM bytes, L2 hit rate) on the match kernel.
# Usage: bash tools/bench_d.sh <tag> [--tests]
set -e
export TMPDIR=/tmp
TAG=${1:-d}
O=gpurun_out/$TAG; mkdir -p $O
ROOT=$(pwd)
if [ "${2:-}" = "--tests" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -30 $O/pytest_gpu.log; exit 1; }
  tail -2 $O/pytest_gpu.log
fi
timeout -k 10 400 python -u bench.py --workload D --cache /tmp/wlD > $O/benchD.json 2> $O/benchD.err || { tail -20 $O/benchD.err; exit 1; }
cat $O/benchD.json
cd /tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$ROOT/$O/prof" -o run -- python3 "$ROOT/bench.py" --workload D --cache /tmp/wlD --no-cpu-baseline --streams 1 > "$ROOT/$O/prof_bench.json" 2> "$ROOT/$O/prof_bench.err" || { tail -20 "$ROOT/$O/prof_bench.err"; exit 1; }
cd "$ROOT"
find "$O/prof" -name "*kernel_stats.csv" -exec head -4 {} \;
i=0
for grp in "FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum"; do
  i=$((i+1))
  cd /tmp
  timeout -s KILL 240 rocprofv3 --pmc $grp --kernel-include-regex match_fast_kernel --output-format csv -d "$ROOT/$O/pmc$i" -o pmc -- python3 "$ROOT/bench.py" --workload D --cache /tmp/wlD --no-cpu-baseline --streams 1 --steps 3 --warmup 1 > "$ROOT/$O/pmc$i.log" 2>&1
  rc=$?; cd "$ROOT"; echo "pmc pass $i ($grp) rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
python tools/pmc_summary.py --dir "$O" --kernel match_fast_kernel > "$O/pmc_summary.json"
cat "$O/pmc_summary.json"
