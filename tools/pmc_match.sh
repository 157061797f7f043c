#!/bin/bash
# The match kernel's counters on one bench workload: a kernel trace and rocprofv3 --pmc passes
# (one counter group per run, never combined with tracing), the FETCH_SIZE calibration on random
# 16-B gathers, then tools/pmc_summary.py -> OUT/pmc_summary.json (tools/update_traffic.py
# --workload B|C1|D turns it into profiles/pmc_match_fast*.json).  The generated workload is
# cached in /tmp between the runs.
# Usage (GPU box, repo root): bash tools/pmc_match.sh gpurun_out/<tag> B|C1|D
set -u
OUT=${1:?out dir}; WL=${2:-B}
mkdir -p "$OUT"
export TMPDIR=/tmp
ROOT=$(pwd)
case "$WL" in
  B) W="--cache /tmp/wlB" ;;
  C1) W="--n-filters 100000000 --vocab-scale 4 --cache /tmp/wlC1" ;;
  D) W="--workload D --cache /tmp/wlD" ;;
  *) echo "unknown workload $WL"; exit 2 ;;
esac
ARGS="$W --no-cpu-baseline --no-host-api --streams 1 --steps 3 --warmup 1"
cd /tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$ROOT/$OUT/prof" -o run -- python3 "$ROOT/bench.py" $ARGS > "$ROOT/$OUT/prof.log" 2>&1
rc=$?; cd "$ROOT"; echo "kernel trace rc=$rc"; [ $rc -eq 0 ] || { tail -5 "$OUT/prof.log"; exit $rc; }
i=0
for grp in "FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum"; do
  i=$((i+1))
  cd /tmp
  timeout -s KILL 300 rocprofv3 --pmc $grp --kernel-include-regex match_fast_kernel --output-format csv -d "$ROOT/$OUT/pmc$i" -o pmc -- python3 "$ROOT/bench.py" $ARGS > "$ROOT/$OUT/pmc$i.log" 2>&1
  rc=$?; cd "$ROOT"; echo "pmc pass $i ($grp) rc=$rc"; [ $rc -eq 0 ] || { tail -5 "$OUT/pmc$i.log"; exit $rc; }
done
cd /tmp
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE TCC_MISS_sum --kernel-include-regex indep_kernel --output-format csv -d "$ROOT/$OUT/cal" -o cal -- "$ROOT/tools/_build/gather_bench" > "$ROOT/$OUT/cal.log" 2>&1
rc=$?; cd "$ROOT"; echo "calibration rc=$rc"; [ $rc -eq 0 ] || exit $rc
python3 tools/pmc_summary.py --dir "$OUT" --kernel match_fast_kernel > "$OUT/pmc_summary.json"
