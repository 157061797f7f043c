#!/bin/bash
# One parameterised driver for GPU-box sessions (replaces the per-run tools/r4_*.sh scripts).
# Every step runs under its own time limit; a failing step ends the session (chain calls with &&).
#
#   bash tools/gpu.sh tests  OUT [pytest args...]         -m gpu tests -> OUT/pytest.log
#   bash tools/gpu.sh smoke  OUT                          __graft_entry__.smoke() -> OUT/smoke.log
#   bash tools/gpu.sh bench  OUT NAME [bench.py args...]  one bench line -> OUT/NAME.json (+ .err)
#   bash tools/gpu.sh prof   OUT NAME [bench.py args...]  rocprofv3 --kernel-trace --stats of the bench
#                                                         -> OUT/NAME_prof/, top kernels printed
#   bash tools/gpu.sh pmc    OUT NAME REGEX [bench.py args...]
#                                                         one rocprofv3 --pmc pass per counter group of
#                                                         $PMC_GROUPS (';'-separated) over the kernels
#                                                         matching REGEX -> OUT/NAME_pmc<i>/
# OUT is created under gpurun_out/.  Environment: STEP_TIMEOUT (seconds, default 600).
set -u
CMD=${1:?command}; OUT=gpurun_out/${2:?out dir}; shift 2
mkdir -p "$OUT"
export TMPDIR=/tmp
ROOT=$(pwd)
T=${STEP_TIMEOUT:-600}

top_kernels() {  # kernel stats csv -> one line per kernel
  python3 - "$1" <<'PY'
import csv, sys
for r in list(csv.DictReader(open(sys.argv[1])))[:30]:
    n = r["Name"]
    if "rocprim" in n:
        n = "rocprim " + ("onesweep_iter" if "onesweep_iteration" in n else "histo" if "histogram" in n else "other")
    print("%-64s %6s %10.1f us avg %10.1f min %10.1f max" % (n[:64], r["Calls"], float(r["AverageNs"]) / 1e3,
                                                               float(r["MinNs"]) / 1e3, float(r["MaxNs"]) / 1e3))
PY
}

case "$CMD" in
  tests)
    timeout -k 10 "$T" python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu "${@:-tests}" \
      > "$OUT/pytest.log" 2>&1
    rc=$?; tail -3 "$OUT/pytest.log"; [ $rc -eq 0 ] || { grep -E "FAILED|Error" "$OUT/pytest.log" | head -20; exit $rc; }
    ;;
  smoke)
    timeout -k 10 "$T" python -u -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1
    rc=$?; tail -2 "$OUT/smoke.log"; exit $rc
    ;;
  bench)
    NAME=${1:?name}; shift
    timeout -k 10 "$T" python -u bench.py "$@" > "$OUT/$NAME.json" 2> "$OUT/$NAME.err"
    rc=$?; [ $rc -eq 0 ] || { tail -30 "$OUT/$NAME.err"; exit $rc; }
    python3 - "$OUT/$NAME.json" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
keep = ("metric", "value", "unit", "ms_per_step", "parity")
print({k: d[k] for k in keep if k in d})
r = d.get("roofline") or {}
print("roofline", {k: r.get(k) for k in ("bound", "achieved", "peak", "frac", "traffic", "kernel_ms_avg")})
for x in d.get("runs", []):
    print(" ", {k: v for k, v in x.items() if not isinstance(v, (list, dict))})
PY
    ;;
  prof)
    NAME=${1:?name}; shift
    cd /tmp
    timeout -k 10 "$T" rocprofv3 --kernel-trace --stats --output-format csv -d "$ROOT/$OUT/${NAME}_prof" -o run \
      -- python3 "$ROOT/bench.py" "$@" > "$ROOT/$OUT/${NAME}_prof.json" 2> "$ROOT/$OUT/${NAME}_prof.err"
    rc=$?; cd "$ROOT"; [ $rc -eq 0 ] || { tail -20 "$OUT/${NAME}_prof.err"; exit $rc; }
    top_kernels "$(find "$OUT/${NAME}_prof" -name "*kernel_stats.csv" | head -1)"
    ;;
  pmc)
    NAME=${1:?name}; RX=${2:?kernel regex}; shift 2
    IFS=';' read -ra PG <<< "${PMC_GROUPS:?set PMC_GROUPS}"
    i=0
    for grp in "${PG[@]}"; do
      i=$((i + 1))
      cd /tmp
      timeout -s KILL 240 rocprofv3 --pmc $grp --kernel-include-regex "$RX" --output-format csv \
        -d "$ROOT/$OUT/${NAME}_pmc$i" -o pmc -- python3 "$ROOT/bench.py" "$@" > "$ROOT/$OUT/${NAME}_pmc$i.log" 2>&1
      rc=$?; cd "$ROOT"; echo "pmc pass $i ($grp) rc=$rc"
      [ $rc -eq 0 ] || { tail -5 "$OUT/${NAME}_pmc$i.log"; exit $rc; }
    done
    ;;
  *)
    echo "unknown command $CMD"; exit 2 ;;
esac
