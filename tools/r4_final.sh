#!/bin/bash
# Round-end rehearsal: every GPU test, smoke(), the default bench line (B).
set -u
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r4_final}
mkdir -p $OUT
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { tail -40 $OUT/pytest_gpu.log; exit 1; }
tail -2 $OUT/pytest_gpu.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $OUT/smoke.log 2>&1 || { tail -20 $OUT/smoke.log; exit 1; }
tail -1 $OUT/smoke.log
timeout -k 10 400 python -u bench.py > $OUT/bench.json 2> $OUT/bench.err || { tail -20 $OUT/bench.err; exit 1; }
python3 -c "import json;d=json.load(open('$OUT/bench.json'));print('B', d['value'], d['ms_per_step'], d['roofline']['frac'], d.get('cpu_baseline',{}).get('value'))"
