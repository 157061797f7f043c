#!/bin/bash
# Round 4: fan-out lines per $share strategy (config E) and the single-publisher batch.
# Usage (GPU box, repo root): bash tools/r4_fanout_bench.sh <tag>
set -u
TAG=${1:-r4}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
run() {  # name, args...
  local name=$1; shift
  echo "== $name $(date +%T)"
  timeout -k 10 400 python -u bench.py --workload E "$@" > "$OUT/bench_$name.json" 2> "$OUT/bench_$name.err"
  local rc=$?
  tail -c 600 "$OUT/bench_$name.json"; echo
  [ $rc -eq 0 ] || { echo "$name rc=$rc"; tail -20 "$OUT/bench_$name.err"; exit $rc; }
}
run E_hash --strategy hash_clientid
run E_rr --strategy round_robin
run E_sticky --strategy sticky --no-cpu-baseline
run E_random --strategy random --no-cpu-baseline
run E_rr_pub1 --strategy round_robin --publishers 1 --no-cpu-baseline
run E_sticky_pub1 --strategy sticky --publishers 1 --no-cpu-baseline
run E_rr_pub1000 --strategy round_robin --publishers 1000 --no-cpu-baseline
echo "== rocprof E rr $(date +%T)"
cd /tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$OLDPWD/$OUT/prof_rr" -o run -- python3 "$OLDPWD/bench.py" --workload E --strategy round_robin --no-cpu-baseline --streams 1 --steps 10 > "$OLDPWD/$OUT/prof_rr.json" 2> "$OLDPWD/$OUT/prof_rr.err" || { echo rocprof failed; tail "$OLDPWD/$OUT/prof_rr.err"; exit 1; }
cd "$OLDPWD"
find "$OUT/prof_rr" -name "*kernel_stats.csv" -exec head -24 {} \;
echo "== done $(date +%T)"
