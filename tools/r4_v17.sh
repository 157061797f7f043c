#!/bin/bash
# Two-pass fan-out restored (+ coalesced entry-topic kernel); faster sharded step (window-load
# routing, 16-B packing, copy-engine unpack, request-order merge).
set -u
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r4_v17}
mkdir -p $OUT
timeout -k 10 500 python -u -m pytest -x -v --timeout 240 --timeout-method thread tests/test_gpu_fanout.py \
  tests/test_gpu_fanout_state.py tests/test_gpu_share_parity.py tests/test_gpu_shard_step.py \
  "tests/test_gpu_parity.py::test_sharded_matcher_world1_rccl" "tests/test_gpu_parity.py::test_sharded_matcher_config_c_generator" \
  > $OUT/pytest.log 2>&1 || { tail -40 $OUT/pytest.log; exit 1; }
tail -2 $OUT/pytest.log
for st in hash_clientid round_robin; do
timeout -k 10 300 python -u bench.py --workload E --strategy $st --steps 20 > $OUT/bench_E_$st.json 2> $OUT/bench_E_$st.err || { tail -20 $OUT/bench_E_$st.err; exit 1; }
python3 -c "import json;d=json.load(open('$OUT/bench_E_$st.json'));print('E $st',d['value'],d['ms_per_step'],d['fanout_call_ms'],d['match_call_ms'],d.get('parity',{}).get('mismatches'))"
done
timeout -k 10 500 python -u bench.py --sharded --steps 20 --warmup 3 > $OUT/bench_sharded_B.json 2> $OUT/bench_sharded_B.err || { tail -20 $OUT/bench_sharded_B.err; exit 1; }
head -c 1200 $OUT/bench_sharded_B.json; echo
ROOT=$(pwd)
cd /tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$ROOT/$OUT/prof" -o run -- python3 "$ROOT/bench.py" --sharded --steps 10 --warmup 2 > "$ROOT/$OUT/prof.json" 2> "$ROOT/$OUT/prof.err" || { tail -20 "$ROOT/$OUT/prof.err"; exit 1; }
cd "$ROOT"
f=$(find $OUT/prof -name "*kernel_stats.csv" | head -1)
python3 - "$f" <<'PY'
import csv,sys
for r in csv.DictReader(open(sys.argv[1])):
    n=r['Name']
    if 'rocprim' in n: n='rocprim '+('onesweep_iter' if 'onesweep_iteration' in n else 'histo' if 'histogram' in n else 'other')
    print("%-60s %5s %10.1f us avg %10.1f min %10.1f max" % (n[:60], r['Calls'], float(r['AverageNs'])/1e3, float(r['MinNs'])/1e3, float(r['MaxNs'])/1e3))
PY
