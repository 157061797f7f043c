#!/bin/bash
# Threaded subscription bookkeeping: fan-out GPU tests (churn parity), S and T benches.
set -u
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r4_sub}
mkdir -p $OUT
timeout -k 10 500 python -u -m pytest -x -v --timeout 240 --timeout-method thread tests/test_gpu_fanout.py \
  tests/test_gpu_fanout_state.py tests/test_gpu_share_parity.py tests/test_gpu_concurrent_commit.py \
  > $OUT/pytest.log 2>&1 || { tail -40 $OUT/pytest.log; exit 1; }
tail -3 $OUT/pytest.log
timeout -k 10 500 python -u bench.py --workload S > $OUT/bench_S.json 2> $OUT/bench_S.err || { tail -20 $OUT/bench_S.err; exit 1; }
head -c 1500 $OUT/bench_S.json; echo
timeout -k 10 500 python -u bench.py --workload T > $OUT/bench_T.json 2> $OUT/bench_T.err || { tail -20 $OUT/bench_T.err; exit 1; }
head -c 3000 $OUT/bench_T.json; echo
