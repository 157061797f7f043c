#!/bin/bash
# Coalesced entry-topic kernel (fan-out tests + E); sharded step profile and 2-rank rehearsal.
set -u
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r4_v15}
mkdir -p $OUT
timeout -k 10 500 python -u -m pytest -x -v --timeout 240 --timeout-method thread tests/test_gpu_fanout.py \
  tests/test_gpu_fanout_state.py tests/test_gpu_share_parity.py > $OUT/pytest.log 2>&1 || { tail -40 $OUT/pytest.log; exit 1; }
tail -2 $OUT/pytest.log
for st in hash_clientid round_robin; do
timeout -k 10 300 python -u bench.py --workload E --strategy $st --steps 20 > $OUT/bench_E_$st.json 2> $OUT/bench_E_$st.err || { tail -20 $OUT/bench_E_$st.err; exit 1; }
python3 -c "import json;d=json.load(open('$OUT/bench_E_$st.json'));print('E $st',d['value'],d['ms_per_step'],d['fanout_call_ms'],d['match_call_ms'],d.get('parity',{}).get('mismatches'))"
done
EMQX_BENCH_REHEARSE=1 timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
  --master-port 29611 bench.py --sharded --n-filters 1000000 --batch 200000 --steps 5 --warmup 2 \
  > $OUT/rehearse2.json 2> $OUT/rehearse2.err || { tail -20 $OUT/rehearse2.err; exit 1; }
head -c 1500 $OUT/rehearse2.json; echo
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
