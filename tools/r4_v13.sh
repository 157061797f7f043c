#!/bin/bash
# Round-4 checkpoint: sharded step tests, fan-out tests (fused offsets, threaded subscription
# bookkeeping), E and S benches.
set -u
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r4_v13}
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_shard_step.py \
  > $OUT/pytest_shard.log 2>&1 || { tail -40 $OUT/pytest_shard.log; exit 1; }
tail -2 $OUT/pytest_shard.log
timeout -k 10 500 python -u -m pytest -x -v --timeout 240 --timeout-method thread tests/test_gpu_fanout.py \
  tests/test_gpu_fanout_state.py tests/test_gpu_share_parity.py > $OUT/pytest_fanout.log 2>&1 || { tail -40 $OUT/pytest_fanout.log; exit 1; }
tail -2 $OUT/pytest_fanout.log
timeout -k 10 300 python -u bench.py --workload E --steps 20 > $OUT/bench_E.json 2> $OUT/bench_E.err || { tail -20 $OUT/bench_E.err; exit 1; }
python3 -c "import json;d=json.load(open('$OUT/bench_E.json'));print('E',d['value'],d['ms_per_step'],d['fanout_call_ms'],d['match_call_ms'],d.get('parity'))"
timeout -k 10 300 python -u bench.py --workload S > $OUT/bench_S.json 2> $OUT/bench_S.err || { tail -20 $OUT/bench_S.err; exit 1; }
python3 -c "import json;d=json.load(open('$OUT/bench_S.json'));print('S',d['value'],d['ms_per_step'],d['commit_ms'],d['cpu_baseline']['value'])"
