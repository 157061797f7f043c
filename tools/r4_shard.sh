#!/bin/bash
# Sharded device step (shard_step.hip): GPU tests, world-1 bench on B, 2-rank same-GPU rehearsal.
set -u
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r4_shard}
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_shard_step.py \
  "tests/test_gpu_parity.py::test_sharded_matcher_world1_rccl" "tests/test_gpu_parity.py::test_sharded_matcher_config_c_generator" \
  > $OUT/pytest.log 2>&1 || { tail -40 $OUT/pytest.log; exit 1; }
tail -3 $OUT/pytest.log
timeout -k 10 500 python -u bench.py --sharded --steps 20 --warmup 3 > $OUT/bench_sharded_B.json 2> $OUT/bench_sharded_B.err || { tail -20 $OUT/bench_sharded_B.err; exit 1; }
cat $OUT/bench_sharded_B.json
EMQX_BENCH_REHEARSE=1 timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
  --master-port 29611 bench.py --sharded --n-filters 1000000 --batch 200000 --steps 5 --warmup 2 \
  > $OUT/rehearse2.json 2> $OUT/rehearse2.err || { tail -20 $OUT/rehearse2.err; exit 1; }
cat $OUT/rehearse2.json
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
