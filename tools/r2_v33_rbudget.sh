#!/bin/bash
# Config R: step budget vs time and fetched bytes (FETCH_SIZE pass per setting).
set -u -o pipefail
O=gpurun_out/${1:-r2_v33}
mkdir -p $O
ROOT=$(pwd)
export TMPDIR=/tmp
for b in 128 256 512 2048; do
  timeout -k 10 300 python -u bench.py --workload R --no-cpu-baseline --steps 20 --warmup 3 --retain-budget $b > $O/benchR_b$b.json 2> $O/benchR_b$b.err || { echo R failed; tail -5 $O/benchR_b$b.err; exit 1; }
  cd /tmp
  timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex retain_ --output-format csv -d $ROOT/$O/pmc_b$b -o pmc -- python3 $ROOT/bench.py --workload R --no-cpu-baseline --steps 5 --warmup 1 --retain-budget $b > $ROOT/$O/pmc_b$b.log 2>&1
  rc=$?; cd $ROOT; [ $rc -eq 0 ] || { echo pmc failed; tail -5 $O/pmc_b$b.log; exit $rc; }
  python - $O $b <<'PY'
import csv, glob, json, sys, collections
O, b = sys.argv[1], sys.argv[2]
d = json.loads(open(f"{O}/benchR_b{b}.json").read().strip().splitlines()[-1])
per = collections.defaultdict(float); calls = collections.Counter()
for p in glob.glob(f"{O}/pmc_b{b}/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(p)):
        k = r["Kernel_Name"].split("(")[0][-40:]
        per[k] += float(r["Counter_Value"]) * 1024
n_calls = 6  # 1 warmup + 5 steps (+ sizing calls excluded roughly)
print("budget", b, "filters/s", d["value"], "ms", d["ms_per_step"], "walk", d.get("walk_ms_median"), "spilled", d.get("walk_spilled_items"),
      {k: round(v / 1e6) for k, v in per.items()})
PY
done
