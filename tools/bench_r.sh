#!/bin/bash
# Config R (retained lookup) round: the bench line, its rocprofv3 kernel stats, and the
# FETCH_SIZE / WRITE_SIZE passes over every retain_* kernel (one rocprofv3 run per counter,
# never combined with tracing) that tools/pmc_retain.py turns into bytes per call.
# Usage (GPU box, repo root): bash tools/bench_r.sh <outdir>
set -u
O=${1:-gpurun_out/benchR}
mkdir -p "$O"
export TMPDIR=/tmp
ROOT=$(pwd)
timeout -k 10 300 python3 bench.py --workload R > "$O/benchR.json" 2> "$O/benchR.err" || { tail -20 "$O/benchR.err"; exit 1; }
cat "$O/benchR.json"
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$ROOT/$O/prof" -o run -- python3 "$ROOT/bench.py" --workload R --no-cpu-baseline > "$ROOT/$O/prof_bench.json" 2> "$ROOT/$O/prof_bench.err" || { tail -20 "$ROOT/$O/prof_bench.err"; exit 1; }
i=0
for c in FETCH_SIZE WRITE_SIZE; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $c --kernel-include-regex retain_ --output-format csv -d "$ROOT/$O/pmc$i" -o pmc -- python3 "$ROOT/bench.py" --workload R --steps 8 --warmup 1 --no-cpu-baseline > "$ROOT/$O/pmc$i.log" 2>&1 || { tail -5 "$ROOT/$O/pmc$i.log"; exit 1; }
done
cd "$ROOT"
python3 tools/pmc_retain.py --dir "$O" --retained 864333 --filters 100000 --out "$O/pmc_retain.json"
