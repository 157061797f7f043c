#!/bin/bash
# Round-4 checkpoint 2: async subtab commits + worker pool; sharded device step measured.
set -u
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r4_v14}
mkdir -p $OUT
timeout -k 10 500 python -u -m pytest -x -v --timeout 240 --timeout-method thread tests/test_gpu_shard_step.py tests/test_gpu_fanout.py \
  tests/test_gpu_fanout_state.py tests/test_gpu_share_parity.py tests/test_gpu_concurrent_commit.py > $OUT/pytest.log 2>&1 || { tail -40 $OUT/pytest.log; exit 1; }
tail -2 $OUT/pytest.log
timeout -k 10 300 python -u bench.py --workload S > $OUT/bench_S.json 2> $OUT/bench_S.err || { tail -20 $OUT/bench_S.err; exit 1; }
python3 -c "import json;d=json.load(open('$OUT/bench_S.json'));print('S',d['value'],d['ms_per_step'],d['commit_ms'],d['commit_stats']['host_us_last_commit'],d['cpu_baseline']['value'])"
timeout -k 10 400 python -u bench.py --workload T > $OUT/bench_T.json 2> $OUT/bench_T.err || { tail -20 $OUT/bench_T.err; exit 1; }
head -c 2500 $OUT/bench_T.json; echo
timeout -k 10 500 python -u bench.py --sharded --steps 20 --warmup 3 > $OUT/bench_sharded_B.json 2> $OUT/bench_sharded_B.err || { tail -20 $OUT/bench_sharded_B.err; exit 1; }
head -c 2500 $OUT/bench_sharded_B.json; echo
