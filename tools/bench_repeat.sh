#!/bin/bash
# Repeat one bench.py line R times (A/B runs on one box): bash tools/bench_repeat.sh OUT R [bench args...]
set -u
OUT=gpurun_out/${1:?out}; R=${2:?repeats}; shift 2
mkdir -p "$OUT"
for r in $(seq 1 "$R"); do
  timeout -k 10 300 python bench.py "$@" > "$OUT/run_$r.json" 2> "$OUT/run_$r.err" || { tail -20 "$OUT/run_$r.err"; exit 1; }
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], d['value'], {k: d[k] for k in ('ms_per_step','fanout_call_ms','match_call_ms','call_ms_median','kernel_ms_median') if k in d})" "$OUT/run_$r.json" "$r"
done
