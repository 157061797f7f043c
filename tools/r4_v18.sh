#!/bin/bash
# Sharded step: tests (device routing vs host), world-1 B line, kernel stats, 2-rank rehearsal.
set -u
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r4_v18}
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest -x -v --timeout 240 --timeout-method thread tests/test_gpu_shard_step.py \
  > $OUT/pytest.log 2>&1 || { tail -40 $OUT/pytest.log; exit 1; }
tail -2 $OUT/pytest.log
timeout -k 10 500 python -u bench.py --sharded --steps 20 --warmup 3 > $OUT/bench_sharded_B.json 2> $OUT/bench_sharded_B.err || { tail -20 $OUT/bench_sharded_B.err; exit 1; }
head -c 400 $OUT/bench_sharded_B.json; echo
EMQX_BENCH_REHEARSE=1 timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
  --master-port 29611 bench.py --sharded --n-filters 1000000 --batch 200000 --steps 5 --warmup 2 \
  > $OUT/rehearse2.json 2> $OUT/rehearse2.err || { tail -20 $OUT/rehearse2.err; exit 1; }
head -c 300 $OUT/rehearse2.json; echo
ROOT=$(pwd)
cd /tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$ROOT/$OUT/prof" -o run -- python3 "$ROOT/bench.py" --sharded --steps 10 --warmup 2 > "$ROOT/$OUT/prof.json" 2> "$ROOT/$OUT/prof.err" || { tail -20 "$ROOT/$OUT/prof.err"; exit 1; }
cd "$ROOT"
f=$(find $OUT/prof -name "*kernel_stats.csv" | head -1)
python3 - "$f" <<'PY'
import csv,sys
for r in csv.DictReader(open(sys.argv[1])):
    n=r['Name']
    if 'shard' not in n and 'match_fast' not in n and 'rccl' not in n and 'copyBuffer' not in n: continue
    print("%-60s %5s %10.1f us avg" % (n[:60], r['Calls'], float(r['AverageNs'])/1e3))
PY
