#!/bin/bash
# Work-sharing retained walk: queue-mode parity tests, then a tuning sweep against the spill rounds.
set -u
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r4_q2}
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_retain.py -k "queue or spill or fuzz or large or tile" > $OUT/pytest.log 2>&1 || { tail -40 $OUT/pytest.log; exit 1; }
tail -2 $OUT/pytest.log
timeout -k 10 400 python -u tools/retain_sweep.py 'balance=0' 'balance=1,queue_check=8,queue_wait=2048,queue_piece=256,queue_sleep=1,queue_shards=64' 'balance=1,queue_check=8,queue_wait=2048,queue_piece=256,queue_sleep=1,queue_shards=16' 'balance=1,queue_check=8,queue_wait=2048,queue_piece=256,queue_sleep=1,queue_shards=128' 'balance=1,queue_check=16,queue_wait=2048,queue_piece=256,queue_sleep=1,queue_shards=64' 'balance=1,queue_check=8,queue_wait=2048,queue_piece=128,queue_sleep=1,queue_shards=64' 'balance=1,queue_check=8,queue_wait=8192,queue_piece=256,queue_sleep=1,queue_shards=64' 'balance=0,spill_budget=48' > $OUT/sweep.jsonl 2> $OUT/sweep.err || { tail -20 $OUT/sweep.err; exit 1; }
cat $OUT/sweep.jsonl
EMQX_LIB=$(pwd)/emqx_amd/_build_prof/libemqxmatch.so EMQX_RETAIN_PROF=1 timeout -k 10 300 python -u tools/retain_sweep.py --calls=4 'balance=0' 'balance=1,queue_check=8,queue_wait=2048,queue_piece=256,queue_sleep=1,queue_shards=64' > $OUT/prof.jsonl 2> $OUT/prof.err || { tail -20 $OUT/prof.err; exit 1; }
grep -E "RETAIN_PROF|RETAIN_QPROF" $OUT/prof.err | tail -2
