#!/bin/bash
# Prefetched serial subscription ops: churn tests, S, T; E line with the round-4 PMC traffic.
set -u
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r4_v21}
mkdir -p $OUT
timeout -k 10 500 python -u -m pytest -x -q --timeout 240 --timeout-method thread tests/test_gpu_fanout.py \
  tests/test_gpu_fanout_state.py tests/test_gpu_share_parity.py tests/test_gpu_concurrent_commit.py > $OUT/pytest.log 2>&1 || { tail -40 $OUT/pytest.log; exit 1; }
tail -2 $OUT/pytest.log
timeout -k 10 300 python -u bench.py --workload S > $OUT/bench_S.json 2> $OUT/bench_S.err || { tail -20 $OUT/bench_S.err; exit 1; }
python3 -c "import json;d=json.load(open('$OUT/bench_S.json'));print('S',d['value'],d['ms_per_step'],d['host_ms_p50'],d['cpu_baseline']['value'])"
timeout -k 10 400 python -u bench.py --workload T > $OUT/bench_T.json 2> $OUT/bench_T.err || { tail -20 $OUT/bench_T.err; exit 1; }
python3 -c "
import json;d=json.load(open('$OUT/bench_T.json'));print('T single', d['single_op']['subscribe']['p50_us'], d['single_op']['subscribe']['p99_us']); [print(r['callers'], r['ops_per_s'], r['p99_us']) for r in d['storm']]; print(d['publish_alone']['messages_per_s'], d['publish_during_storm']['messages_per_s'])"
timeout -k 10 300 python -u bench.py --workload E --steps 20 > $OUT/bench_E.json 2> $OUT/bench_E.err || { tail -20 $OUT/bench_E.err; exit 1; }
python3 -c "import json;d=json.load(open('$OUT/bench_E.json'));print('E',d['value'],d['ms_per_step'],d['fanout_call_ms'],d['roofline']['frac'],d['roofline']['traffic'])"
