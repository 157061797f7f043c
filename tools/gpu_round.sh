#!/bin/bash
# One GPU-box session: GPU parity tests, smoke, bench (1 GPU, config B), rocprofv3 kernel stats.
# Usage (on the GPU box, from the repo root): bash tools/gpu_round.sh <tag> [pytest-args...]
set -u
TAG=${1:-run}; shift || true
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
ROOT=$(pwd)
echo "== gpu tests"; date
[ -n "${SKIP_TESTS:-}" ] || timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread "$@" > "$OUT/pytest_gpu.log" 2>&1
rc=$?; tail -5 "$OUT/pytest_gpu.log"; [ $rc -eq 0 ] || { echo "gpu tests rc=$rc"; exit $rc; }
echo "== smoke"; date
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1 || { echo smoke failed; tail -20 "$OUT/smoke.log"; exit 1; }
tail -2 "$OUT/smoke.log"
echo "== bench"; date
timeout -k 10 600 python -u bench.py --cache /tmp/wlB > "$OUT/bench.json" 2> "$OUT/bench.err" || { echo bench failed; tail -20 "$OUT/bench.err"; exit 1; }
cat "$OUT/bench.json"
echo "== rocprofv3 kernel stats"; date
cd /tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$ROOT/$OUT/prof" -o run -- python3 "$ROOT/bench.py" --cache /tmp/wlB --no-cpu-baseline --no-host-api --streams 1 > "$ROOT/$OUT/prof_bench.json" 2> "$ROOT/$OUT/prof_bench.err" || { echo rocprof failed; tail -20 "$ROOT/$OUT/prof_bench.err"; exit 1; }
cd "$ROOT"
find "$OUT/prof" -name "*kernel_stats.csv" -exec head -8 {} \;
echo "== pmc passes"; date
i=0
for grp in "FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum" "TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum" "GRBM_GUI_ACTIVE GRBM_COUNT"; do
  i=$((i+1))
  cd /tmp
  timeout -s KILL 240 rocprofv3 --pmc $grp --kernel-include-regex match_fast_kernel --output-format csv -d "$ROOT/$OUT/pmc$i" -o pmc -- python3 "$ROOT/bench.py" --cache /tmp/wlB --no-cpu-baseline --no-host-api --streams 1 --steps 3 --warmup 1 > "$ROOT/$OUT/pmc$i.log" 2>&1
  rc=$?; cd "$ROOT"; echo "pmc pass $i ($grp) rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
python tools/pmc_summary.py --dir "$OUT" --kernel match_fast_kernel | tee "$OUT/pmc_summary.json"
echo "== FETCH_SIZE calibration on random 16-B gathers (tools/gather_bench.hip)"; date
if [ -x tools/_build/gather_bench ]; then
  cd /tmp
  timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE TCC_MISS_sum --kernel-include-regex indep_kernel --output-format csv -d "$ROOT/$OUT/cal" -o cal -- "$ROOT/tools/_build/gather_bench" > "$ROOT/$OUT/cal.log" 2>&1
  rc=$?; cd "$ROOT"; echo "calibration rc=$rc"; [ $rc -eq 0 ] || exit $rc
fi
echo "== done"; date
