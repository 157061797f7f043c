#!/bin/bash
# L2 hit/miss and EA read requests of the fused match kernel under different settings
# (env assignments, one setting per argument), one rocprofv3 --pmc pass each.
# Usage (GPU box, repo root): bash tools/pmc_l2.sh <outdir> "EMQX_LAYOUT=bfs" "EMQX_FAST_VARIANT=7" ...
set -u
OUT=${1:-gpurun_out/l2}; shift
mkdir -p "$OUT"
export TMPDIR=/tmp
ROOT=$(pwd)
ARGS="--steps 3 --warmup 1 --no-cpu-baseline --cache /tmp/wlB"
timeout -k 10 300 python -u bench.py $ARGS > "$OUT/prime.json" 2> "$OUT/prime.err" || { echo prime failed; exit 1; }
i=0
for setting in "$@"; do
  i=$((i+1))
  cd /tmp
  env $setting timeout -k 10 120 python3 "$ROOT/bench.py" $ARGS > "$ROOT/$OUT/s$i.bench.json" 2> "$ROOT/$OUT/s$i.bench.err"
  rc=$?; [ $rc -eq 0 ] || { cd "$ROOT"; echo "setting $i bench rc=$rc"; exit $rc; }
  for grp in "TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum GRBM_GUI_ACTIVE"; do
    export $setting
    timeout -s KILL 90 rocprofv3 --pmc $grp --kernel-include-regex match_fast_kernel --output-format csv -d "$ROOT/$OUT/s$i" -o pmc -- python3 "$ROOT/bench.py" $ARGS > "$ROOT/$OUT/s$i.log" 2>&1
    rc=$?
    unset ${setting%%=*}
  done
  cd "$ROOT"; echo "setting $i ($setting) rc=$rc"
  [ $rc -eq 0 ] || exit $rc
  python tools/pmc_summary.py --dir "$OUT/s$i" --kernel match_fast_kernel > "$OUT/s$i.summary.json"
  python - "$OUT/s$i" "$setting" <<'PY'
import json, sys
d = json.load(open(sys.argv[1] + ".summary.json"))["counters_avg_per_dispatch"]
b = json.load(open(sys.argv[1] + ".bench.json"))
h, m = d["TCC_HIT_sum"], d["TCC_MISS_sum"]
print(json.dumps({"setting": sys.argv[2], "kernel_ms": b["roofline"]["kernel_ms_avg"], "l2_hit": round(h / (h + m), 4),
                  "l2_miss_per_topic": round(m / 1e6, 3), "ea_rdreq_per_topic": round(d["TCC_EA0_RDREQ_sum"] / 1e6, 3),
                  "l2_req_per_topic": round((h + m) / 1e6, 3)}))
PY
done
