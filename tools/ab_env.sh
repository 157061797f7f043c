#!/bin/bash
# Interleaved A/B of one environment switch on one box: bash tools/ab_env.sh OUT VAR "A B" R [bench args...]
# -> OUT/<value>_<round>.json, one summary line per run.
set -u
OUT=gpurun_out/${1:?out}; VAR=${2:?var}; VALS=${3:?values}; R=${4:?rounds}; shift 4
mkdir -p "$OUT"
for r in $(seq 1 "$R"); do
  for v in $VALS; do
    env "$VAR=$v" timeout -k 10 300 python bench.py "$@" > "$OUT/${v}_$r.json" 2> "$OUT/${v}_$r.err" || { tail -20 "$OUT/${v}_$r.err"; exit 1; }
    python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], d['value'], {k: d[k] for k in ('ms_per_step','fanout_call_ms','match_call_ms','call_ms_median') if k in d})" "$OUT/${v}_$r.json" "$VAR=$v r=$r"
  done
done
